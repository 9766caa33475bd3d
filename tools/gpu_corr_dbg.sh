#!/bin/bash
# GPU call: correlation product-only (KRCA_CORR_DEBUG=1) vs full, kernel-traced.
set -u
TAG=${1:-corrdbg}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
for d in 0 1 2 3; do
  KRCA_CORR_DEBUG=$d timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_d$d -o run -- python3 tools/prof_kernels.py corr --pods 100000 --reps 3 > $OUT/corr_d$d.json 2> $OUT/err_d$d.log
  rc=$?; echo "d$d EXIT=$rc" >> $OUT/status; [ $rc -eq 0 ] || exit $rc
done
find $OUT -name '*.db' -delete; find $OUT -name '*kernel_trace.csv' -delete
