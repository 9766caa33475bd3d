#!/bin/bash
# GPU call: full -m gpu suite, the bench, a kernel-traced bench and the PPR microbench trace.
set -u
TAG=${1:-r2b}
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
step bench 400 python3 bench.py --steps 20 --warmup 5
step bench_prof 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-verify
step ppr_prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/pprprof -o run -- python3 tools/ppr_bench.py --check
tail -3 $O/tests.log; tail -1 $O/bench.log; tail -1 $O/ppr_prof.log
python3 -c "import csv;[print(r[\"Name\"][:50], r[\"Calls\"], r[\"AverageNs\"], r[\"MinNs\"]) for r in csv.DictReader(open(\"$O/pprprof/run_kernel_stats.csv\")) if \"ppr\" in r[\"Name\"]]"
echo all-done >> $O/status
