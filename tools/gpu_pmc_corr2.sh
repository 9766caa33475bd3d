#!/bin/bash
# GPU call: issue-side counters of the correlation tile kernel, product only (KRCA_CORR_DEBUG=1) at C3,
# with the GPU clock (GRBM_GUI_ACTIVE) to turn cycles into time.  One counter group per run.
set -u
TAG=${1:-pmccorr2}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
C="SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_INSTS_VALU SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT"
for mode in ${MODES:-1}; do
  KRCA_CORR_DEBUG=$mode timeout -s KILL 200 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $O/dbg$mode -o run -- python3 tools/prof_kernels.py corr --pods 100000 --reps 1 > $O/dbg$mode.out 2> $O/dbg$mode.err
  rc=$?; echo "dbg$mode EXIT=$rc" >> $O/status
  [ $rc -eq 0 ] || { tail -3 $O/dbg$mode.err; exit $rc; }
done
find $O -name '*.db' -delete
for mode in ${MODES:-1}; do python3 tools/pmc_summary.py $O/dbg$mode "corr_tiles<16, 0>"; done > $O/summary.txt
echo all-done >> $O/status
