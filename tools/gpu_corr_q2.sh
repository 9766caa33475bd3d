#!/bin/bash
# GPU call: correlation GPU tests, then the exact-count re-score A/B: KRCA_CORR_RS_Q16 = 2 (both rows
# int16, integer products) against 1 (int16 partner rows, fp32 row pod), at C3 and 1M, kernel-traced.
set -u
TAG=${1:-corrq2}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 900 python3 -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu tests/test_gpu_corr.py > $O/tests.log 2>&1
  rc=$?; echo "tests EXIT=$rc" >> $O/status; tail -3 $O/tests.log
  [ $rc -eq 0 ] || { tail -40 $O/tests.log; exit $rc; }
fi
for pods in 100000 1000000; do
for q in 2 1 2 1; do
  D=q${q}_${pods}_$(ls -d $O/q${q}_${pods}_* 2>/dev/null | wc -l)
  reps=5; [ $pods -ge 1000000 ] && reps=1
  KRCA_CORR_RS_Q16=$q timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$D -o run -- python3 tools/prof_kernels.py corr --pods $pods --reps $reps > $O/$D.log 2>&1
  rc=$?; echo "$D EXIT=$rc" >> $O/status
  [ $rc -eq 0 ] || { tail -5 $O/$D.log; exit $rc; }
  find $O/$D -name '*.db' -delete
  echo "$D $(grep '^{' $O/$D.log | cut -c1-110)"
  python3 -c "import csv;[print('   ', r['Name'][32:62], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us') for r in csv.DictReader(open('$O/$D/run_kernel_stats.csv')) if 'rescore' in r['Name'] or 'corr_tiles<12, 0' in r['Name']]"
done
done
echo all-done >> $O/status
