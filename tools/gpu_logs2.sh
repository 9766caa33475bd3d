#!/bin/bash
# GPU call: log-scan parity tests + 1M-container timing (kernel trace).  bash tools/gpu_logs2.sh TAG
set -u
TAG=${1:-logs}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
step() {  # step NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $O/$name.log 2>&1
  local rc=$?; echo "$name EXIT=$rc" >> $O/status
  [ $rc -eq 0 ] || { tail -30 $O/$name.log; exit $rc; }
}
step tests 300 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_kernels.py -k "log or template" tests/test_gpu_agents.py tests/test_gpu_stream.py
step prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 tools/prof_kernels.py logs --reps 3
find $O -name '*.db' -delete; find $O -name '*kernel_trace.csv' -delete
grep kernel $O/prof.log
echo all-done >> $O/status
