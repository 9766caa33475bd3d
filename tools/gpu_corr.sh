#!/bin/bash
# GPU call: correlation + PPR parity tests, then a timed / traced correlation run.
set -u
TAG=${1:-corr}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_corr.py tests/test_gpu_kernels.py -x -v --timeout 200 --timeout-method thread -k "corr or ppr or rca" > $OUT/tests.log 2>&1
echo "tests EXIT=$?" >> $OUT/status
tail -3 $OUT/tests.log
timeout -k 10 300 python tools/prof_kernels.py corr --pods 100000 --reps 3 > $OUT/corr.json 2>> $OUT/err.log || { echo "corr failed" >> $OUT/status; exit 1; }
cat $OUT/corr.json
timeout -k 10 300 python tools/prof_kernels.py ppr --reps 3 > $OUT/ppr.json 2>> $OUT/err.log || { echo "ppr failed" >> $OUT/status; exit 1; }
cat $OUT/ppr.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_corr -o run -- python3 tools/prof_kernels.py corr --pods 100000 --reps 2 > /dev/null 2>> $OUT/err.log || echo "trace failed" >> $OUT/status
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_ppr -o run -- python3 tools/prof_kernels.py ppr --reps 2 > /dev/null 2>> $OUT/err.log || echo "trace failed" >> $OUT/status
find $OUT -name '*.db' -delete
find $OUT -name 'run_kernel_trace.csv' -size +2M -delete
