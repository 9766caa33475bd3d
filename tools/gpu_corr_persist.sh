#!/bin/bash
# GPU call: correlation GPU tests, then the main pass A/B, persistent workgroups (KRCA_CORR_PERSIST=1)
# against one workgroup per tile (0), full (mode 0) and product only (mode 1), at C3 and at 1M pods.
set -u
TAG=${1:-corrpersist}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 900 python3 -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu tests/test_gpu_corr.py > $O/tests.log 2>&1
  rc=$?; echo "tests EXIT=$rc" >> $O/status; tail -3 $O/tests.log
  [ $rc -eq 0 ] || { tail -40 $O/tests.log; exit $rc; }
fi
for pods in ${PODSL:-100000 1000000}; do
for m in ${MODES:-0 1}; do
for pe in ${PERSISTS:-1 0}; do
  D=p${pods}m${m}pe$pe
  reps=3; [ $pods -ge 1000000 ] && reps=1
  KRCA_CORR_PERSIST=$pe KRCA_CORR_DEBUG=$m timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$D -o run -- python3 tools/prof_kernels.py corr --pods $pods --reps $reps > $O/$D.log 2>&1
  rc=$?; echo "$D EXIT=$rc" >> $O/status
  [ $rc -eq 0 ] || { tail -5 $O/$D.log; exit $rc; }
  find $O/$D -name '*.db' -delete
  echo "pods $pods mode $m persist $pe $(grep '^{' $O/$D.log | cut -c1-120)"
  python3 -c "import csv;[print('   ', r['Name'][32:70], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us') for r in csv.DictReader(open('$O/$D/run_kernel_stats.csv')) if 'corr_tiles<' in r['Name'] or 'persist' in r['Name'] or 'rescore' in r['Name']]"
done
done
done
echo all-done >> $O/status
