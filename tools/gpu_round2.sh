#!/bin/bash
# One GPU call: score cache-policy A/B, correlation C3 timing + tests, betweenness timing, log PMC.
set -u
TAG=${1:-r2}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
step() {  # step NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $O/$name.log 2>&1
  local rc=$?; echo "$name EXIT=$rc" >> $O/status
  [ $rc -eq 0 ] || { tail -5 $O/$name.log; exit $rc; }
}
step score_ab 240 python3 tools/score_ab.py --only pipe_c20,pipe_c20_nt,pipe_c20,pipe_c20_nt --reps 6
step corr_tests 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_corr.py
step corr_prof 240 python3 tools/prof_kernels.py corr --pods 100000 --reps 3
step bc 600 bash tools/gpu_bc.sh $TAG/bc
step pmc_logs 600 bash tools/gpu_pmc_logs.sh $TAG/pmclogs
echo all-done >> $O/status
