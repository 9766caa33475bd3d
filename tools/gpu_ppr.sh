#!/bin/bash
# GPU call: PPR/RCA parity tests, then the bench (step time) and a kernel trace of the bench.
set -u
TAG=${1:-ppr}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 200 --timeout-method thread -k "ppr or rca" > $OUT/tests.log 2>&1
rc=$?; echo "tests EXIT=$rc" >> $OUT/status; tail -12 $OUT/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "bench EXIT=$rc" >> $OUT/status; cat $OUT/bench.json
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-verify > /dev/null 2> $OUT/trace.err
rc=$?; echo "trace EXIT=$rc" >> $OUT/status
find $OUT -name '*.db' -delete
exit $rc
