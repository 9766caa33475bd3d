#!/bin/bash
# GPU call: a correlation variant library (lib/libkrca_<VAR>.so, tools/build_variant.sh) against the
# current build: the correlation GPU tests on the variant, then C3 timings alternated (three rounds),
# a kernel trace of each, and one 1M-pod call of each.  Usage: tools/gpu_corr_lib_ab.sh TAG VAR
set -u
TAG=${1:-corrlib}
VAR=${2:?variant name}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
VLIB=$PWD/kubernetes-rca-system_amd/lib/libkrca_$VAR.so
KRCA_LIB=$VLIB timeout -k 10 900 python3 -u -m pytest -x -v --timeout 400 --timeout-method thread -m gpu tests/test_gpu_corr.py > $O/tests.log 2>&1
rc=$?; echo "tests EXIT=$rc" >> $O/status; tail -1 $O/tests.log
[ $rc -eq 0 ] || { tail -40 $O/tests.log; exit $rc; }
run() {  # run NAME PODS REPS [trace]
  local v=$1 pods=$2 reps=$3 tr=${4:-}
  if [ $v = base ]; then unset KRCA_LIB; else export KRCA_LIB=$VLIB; fi
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
for r in 1 2 3; do for v in base $VAR; do run $v 100000 10; done; done
run base 100000 5 trace
run $VAR 100000 5 trace
run base 1000000 1
run $VAR 1000000 1
echo all-done >> $O/status
