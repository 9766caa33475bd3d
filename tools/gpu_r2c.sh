#!/bin/bash
# GPU call: C5 streaming tests (single device + 2 ranks sharing the GPU over gloo), the C5 bench
# (1 rank; 2 ranks over gloo as a rehearsal of the sharded path), a kernel trace, the counter list.
set -u
TAG=${1:-r2c}
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
step tests 600 python3 -u -m pytest -x -v --timeout 500 --timeout-method thread tests/test_gpu_stream.py tests/test_gpu_stream_dist.py
step stream1 400 python3 tools/bench_stream.py
step stream2 500 env KRCA_BENCH_BACKEND=gloo python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 tools/bench_stream.py --windows 4
step stream_prof 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 tools/bench_stream.py --windows 4
timeout -s KILL 60 rocprofv3 -L > $O/counters.txt 2>&1; echo "list EXIT=$?" >> $O/status
tail -3 $O/tests.log; grep '^{' $O/stream1.log | cut -c1-1500; grep '^{' $O/stream2.log | cut -c1-600
echo all-done >> $O/status
