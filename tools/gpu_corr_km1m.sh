set -u
O=gpurun_out/R9c; mkdir -p $O; export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
for r in 1 2; do for v in 6 4; do
  KRCA_CORR_KM_EXTRA=$v timeout -k 10 300 python3 tools/prof_kernels.py corr --pods 1000000 --reps 3 --tau 0.5 > $O/km${v}_$r.log 2>&1
  rc=$?; echo "km${v}_$r EXIT=$rc" >> $O/status; [ $rc -eq 0 ] || exit $rc
  echo "km$v r$r $(grep '^{' $O/km${v}_$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print([round(x,1) for x in d["ms"]])')"
done; done
