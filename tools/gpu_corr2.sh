#!/bin/bash
# GPU call: correlation parity tests, then timing + kernel trace at C3 (100k pods).
set -u
TAG=${1:-corr2}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_corr.py -x -v --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1
rc=$?; echo "tests EXIT=$rc" >> $OUT/status; tail -12 $OUT/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 tools/prof_kernels.py corr --pods 100000 --reps 3 > $OUT/corr.json 2> $OUT/corr.err
rc=$?; echo "corr EXIT=$rc" >> $OUT/status; cat $OUT/corr.json
find $OUT -name '*.db' -delete; find $OUT -name '*kernel_trace.csv' -delete
exit $rc
