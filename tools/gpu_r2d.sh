#!/bin/bash
# GPU call: template / log tests, the C5 bench and its kernel trace.
set -u
TAG=${1:-r2d}
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
step tests 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_stream.py tests/test_gpu_stream_dist.py tests/test_gpu_scale.py -k "template or log or stream or c2mini"
step stream1 400 python3 tools/bench_stream.py
step stream_prof 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 tools/bench_stream.py --windows 4
tail -3 $O/tests.log; grep '^{' $O/stream1.log | cut -c1-900
python3 -c "import csv;[print(r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e3,1)) for r in csv.DictReader(open('$O/prof/run_kernel_stats.csv')) if any(k in r['Name'] for k in ('tmpl','log_','ppr_step','stream_score','topk'))]"
echo all-done >> $O/status
