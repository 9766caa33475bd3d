#!/bin/bash
# GPU call: scoring parity (all kernel variants) + A/B timing of the variants at C4 size.
set -u
TAG=${1:-score_ab}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 200 --timeout-method thread -k "rolling_score" > $OUT/tests.log 2>&1
rc=$?; echo "tests EXIT=$rc" >> $OUT/status; tail -3 $OUT/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/score_ab.py --reps 6 > $OUT/ab.json 2> $OUT/ab.err
rc=$?; echo "ab EXIT=$rc" >> $OUT/status; cat $OUT/ab.json
exit $rc
