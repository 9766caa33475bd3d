#!/bin/bash
# GPU call: the 1M-pod correlation (1440 steps, tau 0.5, 3 calls per process) with KRCA_CORR_BATCH
# alternated over the given values, two rounds.  Usage: bash tools/gpu_corr_batch1m.sh TAG V1 V2 ...
set -u
TAG=$1; shift
O=gpurun_out/$TAG; mkdir -p $O; export TMPDIR=/tmp; cd $GRAFT_REPO_ROOT
for r in 1 2; do for v in "$@"; do
  KRCA_CORR_BATCH=$v timeout -k 10 300 python3 tools/prof_kernels.py corr --pods 1000000 --reps 3 --tau 0.5 > $O/b${v}_$r.log 2>&1
  rc=$?; echo "b${v}_$r EXIT=$rc" >> $O/status; [ $rc -eq 0 ] || { tail -5 $O/b${v}_$r.log; exit $rc; }
  echo "batch$v r$r $(grep '^{' $O/b${v}_$r.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print([round(x,1) for x in d["ms"]])')"
done; done
