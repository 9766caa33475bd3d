#!/bin/bash
# GPU call: C5 streaming bench (plain + kernel-traced) and the f1 pod-classify kernel timing.
set -u
TAG=${1:-stream}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u tools/bench_stream.py > $OUT/stream.json 2> $OUT/stream.err
rc=$?; echo "stream EXIT=$rc" >> $OUT/status; cat $OUT/stream.json | cut -c1-1500; [ $rc -eq 0 ] || { tail -5 $OUT/stream.err; exit $rc; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_stream -o run -- python3 tools/bench_stream.py --windows 4 > $OUT/stream_traced.json 2> $OUT/trace.err
rc=$?; echo "trace EXIT=$rc" >> $OUT/status; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_pods -o run -- python3 tools/prof_kernels.py pods --reps 5 > $OUT/pods.json 2> $OUT/pods.err
rc=$?; echo "pods EXIT=$rc" >> $OUT/status; cat $OUT/pods.json
find $OUT -name '*.db' -delete; find $OUT -name '*kernel_trace.csv' -size +3M -delete
exit $rc
