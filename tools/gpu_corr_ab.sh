#!/bin/bash
# GPU call: correlation GPU tests, then the main-pass tile kernel at C3 per re-score grid (A/B on
# one box) and per KRCA_CORR_DEBUG mode, kernel-traced.
set -u
TAG=${1:-corrab}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_corr.py > $O/tests.log 2>&1
  rc=$?; echo "tests EXIT=$rc" >> $O/status; tail -3 $O/tests.log
  [ $rc -eq 0 ] || { tail -40 $O/tests.log; exit $rc; }
fi
for rsg in ${RSGS:-4096}; do
for tc in ${TCS:-256}; do
for m in ${MODES:-0 1}; do
  D=t${tc}m${m}g$rsg
  KRCA_CORR_RS_GRID=$rsg KRCA_CORR_DEBUG=$m timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/t${tc}m${m}g$rsg -o run -- python3 tools/prof_kernels.py corr --pods ${PODS:-100000} --reps 3 > $O/t${tc}m${m}g$rsg.log 2>&1
  rc=$?; echo "$D EXIT=$rc" >> $O/status
  [ $rc -eq 0 ] || { tail -5 $O/$D.log; exit $rc; }
  find $O/$D -name '*.db' -delete
  echo "tc $tc mode $m rsg $rsg $(grep '^{' $O/$D.log | cut -c1-100)"
  python3 -c "import csv;[print('   ', r['Name'][32:62], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us') for r in csv.DictReader(open('$O/$D/run_kernel_stats.csv')) if 'corr_tiles<' in r['Name'] or 'rescore' in r['Name']]"
done
done
done
