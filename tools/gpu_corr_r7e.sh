#!/bin/bash
# GPU call: correlation GPU tests on the current library (4096 candidate slots, projections beside
# the sample), then C3 / 1M timings against lib/libkrca_capc2k.so (2048 slots), kernel-traced.
set -u
TAG=${1:-corrr7e}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu tests/test_gpu_corr.py > $O/tests.log 2>&1
rc=$?; echo "tests EXIT=$rc" >> $O/status; tail -3 $O/tests.log
[ $rc -eq 0 ] || { tail -40 $O/tests.log; exit $rc; }
for pods in 100000 1000000; do
for lib in cur capc2k cur; do
  D=${lib}_${pods}_$(ls -d $O/${lib}_${pods}_* 2>/dev/null | wc -l)
  if [ $lib = capc2k ]; then export KRCA_LIB=$PWD/kubernetes-rca-system_amd/lib/libkrca_capc2k.so; else unset KRCA_LIB; fi
  reps=5; [ $pods -ge 1000000 ] && reps=1
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$D -o run -- python3 tools/prof_kernels.py corr --pods $pods --reps $reps > $O/$D.log 2>&1
  rc=$?; echo "$D EXIT=$rc" >> $O/status
  [ $rc -eq 0 ] || { tail -5 $O/$D.log; exit $rc; }
  find $O/$D -name '*.db' -delete
  echo "$D $(grep '^{' $O/$D.log | cut -c1-160)"
done
done
echo all-done >> $O/status
