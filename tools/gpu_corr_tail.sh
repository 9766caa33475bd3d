#!/bin/bash
# GPU call: the correlation GPU tests on the current library, then C3 timings alternated over
#   base  lib/libkrca_olddeep.so (the previous corr.hip: deep merge over the whole buffer, scalar
#         projection loads)
#   cur   the current library
# then a kernel trace of each at C3, and base / cur at 1M pods.
# (R7q / R7r also ran two variants since removed: the error norms on the side stream beside the
# sample, KRCA_CORR_DNORM_SIDE, and the projections after a one-batch main pass, KRCA_CORR_PROJ=3.)
set -u
TAG=${1:-corrtail}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
L=$PWD/kubernetes-rca-system_amd/lib
timeout -k 10 900 python3 -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu tests/test_gpu_corr.py > $O/tests.log 2>&1
rc=$?; echo "tests EXIT=$rc" >> $O/status; tail -3 $O/tests.log
[ $rc -eq 0 ] || { tail -40 $O/tests.log; exit $rc; }
run() {  # run NAME PODS REPS [trace]
  local v=$1 pods=$2 reps=$3 tr=${4:-}
  unset KRCA_LIB
  case $v in base) export KRCA_LIB=$L/libkrca_olddeep.so;; esac
  local D=${v}_${pods}_$(ls $O/${v}_${pods}_*.log 2>/dev/null | wc -l)
  if [ -n "$tr" ]; then
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$D -o run -- python3 tools/prof_kernels.py corr --pods $pods --reps $reps > $O/$D.log 2>&1
  else
    timeout -k 10 300 python3 tools/prof_kernels.py corr --pods $pods --reps $reps > $O/$D.log 2>&1
  fi
  local rc=$?; echo "$D EXIT=$rc" >> $O/status
  [ $rc -eq 0 ] || { tail -5 $O/$D.log; exit $rc; }
  if [ -n "$tr" ]; then find $O/$D -name '*.db' -delete; fi
  echo "$D $(grep '^{' $O/$D.log | python3 -c 'import json,sys,statistics as s; d=json.loads(sys.stdin.read()); print(round(s.median(d["ms"]),3), round(min(d["ms"]),3))')"
}
for r in 1 2 3; do for v in base cur; do run $v 100000 10; done; done
run cur 100000 5 trace
run base 100000 5 trace
run base 1000000 1
run cur 1000000 1
echo all-done >> $O/status
