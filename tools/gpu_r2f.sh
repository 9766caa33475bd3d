#!/bin/bash
# GPU call (round-2 final evidence): full -m gpu suite, smoke, bench + kernel-traced bench,
# correlation C3 / 1M traces, C5 stream bench + trace.
set -u
TAG=${1:-r2f}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
step() {  # step NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $O/$name.log 2>&1
  local rc=$?; echo "$name EXIT=$rc" >> $O/status
  [ $rc -eq 0 ] || { tail -30 $O/$name.log; exit $rc; }
}
step tests 1000 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
step smoke 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
step bench 400 python3 bench.py --steps 20 --warmup 5
step bench_prof 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-verify
step corr_prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/corrprof -o run -- python3 tools/prof_kernels.py corr --pods 100000 --reps 3
step corr08 300 python3 tools/prof_kernels.py corr --pods 100000 --reps 3 --tau 0.8
step corr1m 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/corr1m -o run -- python3 tools/prof_kernels.py corr --pods 1000000 --reps 1 --tau 0.9
step stream1 400 python3 tools/bench_stream.py
step stream_prof 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/sprof -o run -- python3 tools/bench_stream.py --windows 4
find $O -name '*.db' -delete
tail -3 $O/tests.log; tail -1 $O/smoke.log; tail -1 $O/bench.log | cut -c1-600
grep '^{' $O/corr_prof.log | cut -c1-300; grep '^{' $O/corr08.log | cut -c1-200; grep '^{' $O/corr1m.log | cut -c1-300
grep '^{' $O/stream1.log | cut -c1-400
echo all-done >> $O/status
