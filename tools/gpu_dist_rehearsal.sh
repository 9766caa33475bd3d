#!/bin/bash
# GPU call: rehearse the N-rank bench path (sharded scoring, one all-gather per PageRank iteration,
# max-over-ranks timing) with 2 ranks sharing the box's one GPU over gloo.  bash tools/gpu_dist_rehearsal.sh TAG
set -u
TAG=${1:-dist}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
KRCA_BENCH_BACKEND=gloo timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 3 --warmup 1 > $O/bench2.json 2> $O/bench2.err
rc=$?; echo "bench2 EXIT=$rc" >> $O/status; cat $O/bench2.json; tail -5 $O/bench2.err
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/bench1.json 2> $O/bench1.err
rc=$?; echo "bench1 EXIT=$rc" >> $O/status; cat $O/bench1.json
[ $rc -eq 0 ] || exit $rc
