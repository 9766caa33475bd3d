#!/bin/bash
# GPU call: bench pipelined (default) vs --no-pipeline, plus the 2-rank gloo rehearsal.
set -u
TAG=${1:-pipe}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
step() {  # step NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $O/$name.json 2> $O/$name.err
  local rc=$?; echo "$name EXIT=$rc" >> $O/status
  [ $rc -eq 0 ] || { tail -20 $O/$name.err; exit $rc; }
}
step pipe 300 python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline

KRCA_BENCH_BACKEND=gloo step dist2 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1
echo all-done >> $O/status
