#!/bin/bash
# GPU call: f4 group-by tests + timing of krca_group_reduce over 10M events (kernel trace).
set -u
TAG=${1:-f4}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
step() {  # step NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $O/$name.log 2>&1
  local rc=$?; echo "$name EXIT=$rc" >> $O/status
  [ $rc -eq 0 ] || { tail -20 $O/$name.log; exit $rc; }
}
step tests 400 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_groupby.py tests/test_gpu_agents.py
step prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o ev -- python3 tools/prof_kernels.py events --reps 5
KRCA_GROUP_IMPL=1 step direct 120 python3 tools/prof_kernels.py events --reps 5
grep kernel $O/prof.log $O/direct.log
find $O/prof -name "*kernel_stats.csv" -exec cp {} $O/events_kernel_stats.csv \;
echo all-done >> $O/status
