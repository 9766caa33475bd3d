#!/bin/bash
# GPU call: log-scan / template parity tests, then the 1M-container log scan timing and trace.
set -u
TAG=${1:-logs}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -k "log or template or agents" > $OUT/tests.log 2>&1
rc=$?; echo "tests EXIT=$rc" >> $OUT/status; grep -E "passed|failed|FAIL" $OUT/tests.log | tail -5
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 tools/prof_kernels.py logs --reps 3 > $OUT/logs.json 2> $OUT/logs.err
rc=$?; echo "logs EXIT=$rc" >> $OUT/status; cat $OUT/logs.json
find $OUT -name '*.db' -delete; find $OUT -name '*kernel_trace.csv' -delete
exit $rc
