#!/bin/bash
# GPU call 1: parity tests (-m gpu), smoke(), then the headline bench.
# usage: tools/gpu_check.sh TAG
set -u
TAG=${1:-chk}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/gpu_tests.log 2>&1
rc=$?; echo "tests EXIT=$rc" >> $OUT/status; tail -3 $OUT/gpu_tests.log
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 150 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?; echo "smoke EXIT=$rc" >> $OUT/status; tail -2 $OUT/smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 450 python -u bench.py --steps 10 --warmup 2 > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "bench EXIT=$rc" >> $OUT/status; cat $OUT/bench.json; tail -3 $OUT/bench.err
exit $rc
