#!/bin/bash
# GPU call: C3 correlation timing with the profiling switches (KRCA_CORR_DEBUG: 1 product only,
# 2 no global candidate appends, 3 no candidate slow path; results are wrong when set).
set -u
TAG=${1:-corrdbg}
O=gpurun_out/$TAG
mkdir -p $O
cd $GRAFT_REPO_ROOT
for m in ${MODES:-0 1 2 3}; do
  KRCA_CORR_DEBUG=$m timeout -k 10 200 python3 tools/prof_kernels.py corr --pods 100000 --reps 3 > $O/dbg$m.log 2>&1
  rc=$?; echo "dbg$m EXIT=$rc" >> $O/status
  [ $rc -eq 0 ] || { tail -5 $O/dbg$m.log; exit $rc; }
  echo "dbg$m $(grep '^{' $O/dbg$m.log | cut -c1-120)"
done
