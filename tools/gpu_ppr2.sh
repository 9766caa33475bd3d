#!/bin/bash
# GPU call: PageRank dictionary-block A/B at C4 + kernel traces, then the PPR / RCA tests.
set -u
TAG=${1:-ppr2}
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
step tests 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_scale.py tests/test_gpu_kernels.py tests/test_gpu_stream.py -k "ppr or rca or ranking or c2 or c4 or stream or coordinator"
step dict1 300 python3 tools/ppr_bench.py --dict 1 --check
step dict0 300 python3 tools/ppr_bench.py --dict 0 --check
step prof1 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof1 -o run -- python3 tools/ppr_bench.py --dict 1
step prof0 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof0 -o run -- python3 tools/ppr_bench.py --dict 0
cat $O/dict1.log $O/dict0.log
grep -h ppr_step $O/prof1/run_kernel_stats.csv $O/prof0/run_kernel_stats.csv | cut -c1-40,200-300
echo all-done >> $O/status
