#!/bin/bash
# GPU call: a subset (or all) of the -m gpu tests.  usage: tools/gpu_tests.sh TAG [pytest -k expr]
set -u
TAG=${1:-t}
K=${2:-}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
if [ -n "$K" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -k "$K" > $OUT/tests.log 2>&1
else
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $OUT/tests.log 2>&1
fi
rc=$?; echo "tests EXIT=$rc" >> $OUT/status; grep -E "PASS|FAIL|Error|passed|failed" $OUT/tests.log | tail -40
exit $rc
