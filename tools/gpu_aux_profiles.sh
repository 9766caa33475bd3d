#!/bin/bash
# GPU call: kernel-trace profiles of a13 template hashing, f2 graph construction and f3 betweenness.
set -u
TAG=${1:-aux}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
run() {  # run NAME SECONDS ARGS...
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs rocprofv3 --kernel-trace --stats --output-format csv -d $O/$name -o run -- python3 tools/prof_kernels.py "$@" > $O/$name.log 2>&1
  local rc=$?; echo "$name EXIT=$rc" >> $O/status
  [ $rc -eq 0 ] || { tail -20 $O/$name.log; exit $rc; }
  find $O/$name -name '*.db' -delete
  grep '^{' $O/$name.log | cut -c1-400
}
run tmpl1M 300 tmpl --docs 1000000 --reps 5
run f2 300 f2 --pods 1000000 --reps 3
run bc20k 300 bc --pods 20000 --reps 2
run bc50k 300 bc --pods 50000 --reps 1
echo all-done >> $O/status
