#!/bin/bash
# GPU call: correlation iteration loop: C3 timings (full, product only, L2-resident product) and the
# correlation GPU tests.
set -u
TAG=${1:-corriter}
O=gpurun_out/$TAG
mkdir -p $O
cd $GRAFT_REPO_ROOT
for m in ${MODES:-0 1 4}; do
  KRCA_CORR_DEBUG=$m timeout -k 10 200 python3 tools/prof_kernels.py corr --pods 100000 --reps 3 > $O/dbg$m.log 2>&1
  rc=$?; echo "dbg$m EXIT=$rc" >> $O/status
  [ $rc -eq 0 ] || { tail -5 $O/dbg$m.log; exit $rc; }
  echo "dbg$m $(grep '^{' $O/dbg$m.log | cut -c1-150)"
done
if [ "${STATS:-1}" = 1 ]; then
  export TMPDIR=/tmp
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 tools/prof_kernels.py corr --pods 100000 --reps 3 > $O/prof.log 2>&1
  rc=$?; echo "prof EXIT=$rc" >> $O/status
  [ $rc -eq 0 ] || { tail -5 $O/prof.log; exit $rc; }
  find $O/prof -name '*.db' -delete
  python3 tools/corr_stats_table.py $O/prof
fi
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_corr.py > $O/tests.log 2>&1
  rc=$?; echo "tests EXIT=$rc" >> $O/status; tail -3 $O/tests.log; exit $rc
fi
