#!/bin/bash
# GPU call: the C4 bench step (no correlation leg, no CPU baseline) per PageRank grid cap
# (KRCA_PPR_GRID: persistent step workgroups; 0 = the occupancy API's 5 per CU), alternated twice.
set -u
TAG=${1:-pprgrid}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
for r in 1 2; do
for g in ${GRIDS:-0 512 256 128}; do
  D=g${g}_$r
  KRCA_PPR_GRID=$g timeout -k 10 300 python3 bench.py --no-corr --no-cpu-baseline --steps 10 --warmup 2 > $O/$D.log 2>&1
  rc=$?; echo "$D EXIT=$rc" >> $O/status
  [ $rc -eq 0 ] || { tail -5 $O/$D.log; exit $rc; }
  grep '^{' $O/$D.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); r=d["roofline"]; print("'$D'", "ms_per_step", round(d["ms_per_step"],3), "step_med", round(d["step_ms_median"],3), "e2e", round(d["e2e_rca_latency_ms"],3), "score_co", round(r["avg_launch_ms"],3), "score_solo", round(r["solo_avg_launch_ms"],3), "frac", round(r["frac"],3), "verify", all(v for v in d["verify"].values() if isinstance(v,bool)))'
done
done
echo all-done >> $O/status
