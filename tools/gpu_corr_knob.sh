#!/bin/bash
# GPU call: C3 correlation timings alternated over the values of one knob (environment variable),
# three rounds, then a kernel trace per value.  Usage: tools/gpu_corr_knob.sh TAG KNOB V1 V2 ...
set -u
TAG=${1:-corrknob}
KNOB=${2:?knob}
shift 2
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
run() {  # run VALUE [trace]
  local v=$1 tr=${2:-}
  local D=${KNOB}_${v}_$(ls $O/${KNOB}_${v}_*.log 2>/dev/null | wc -l)
  export "$KNOB=$v"
  if [ -n "$tr" ]; then
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$D -o run -- python3 tools/prof_kernels.py corr --pods 100000 --reps 5 > $O/$D.log 2>&1
  else
    timeout -k 10 300 python3 tools/prof_kernels.py corr --pods 100000 --reps 10 > $O/$D.log 2>&1
  fi
  local rc=$?; echo "$D EXIT=$rc" >> $O/status
  [ $rc -eq 0 ] || { tail -5 $O/$D.log; exit $rc; }
  if [ -n "$tr" ]; then find $O/$D -name '*.db' -delete; fi
  echo "$D $(grep '^{' $O/$D.log | python3 -c 'import json,sys,statistics as s; d=json.loads(sys.stdin.read()); print(round(s.median(d["ms"]),3), round(min(d["ms"]),3))')"
}
for r in 1 2 3; do for v in "$@"; do run $v; done; done
for v in "$@"; do run $v trace; done
echo all-done >> $O/status
