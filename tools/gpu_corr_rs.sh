#!/bin/bash
# GPU call: correlation GPU tests, then C3 timing per KRCA_CORR_RS_IMPL (re-score grouped by row pod
# vs per pair), kernel-traced.
set -u
TAG=${1:-corrrs}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_corr.py tests/test_gpu_scale.py -k "corr or c2mini" > $O/tests.log 2>&1
rc=$?; echo "tests EXIT=$rc" >> $O/status; tail -3 $O/tests.log
[ $rc -eq 0 ] || { tail -40 $O/tests.log; exit $rc; }
for ri in ${RSI:-0 1}; do
  D=rs$ri
  KRCA_CORR_RS_IMPL=$ri timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$D -o run -- python3 tools/prof_kernels.py corr --pods ${PODS:-100000} --reps 3 > $O/$D.log 2>&1
  rc=$?; echo "$D EXIT=$rc" >> $O/status
  [ $rc -eq 0 ] || { tail -5 $O/$D.log; exit $rc; }
  find $O/$D -name '*.db' -delete
  echo "rs_impl $ri $(grep '^{' $O/$D.log | cut -c1-100)"
  python3 -c "import csv;[print('   ', r['Name'][32:70], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us') for r in csv.DictReader(open('$O/$D/run_kernel_stats.csv')) if 'corr_' in r['Name']]"
done
