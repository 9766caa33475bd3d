#!/bin/bash
# GPU call: counters of the correlation main-pass tile kernel at C3 per KRCA_CORR_DEBUG mode
# (0 full, 1 product only, 4 product only with L2-resident operands): issue / wait / MFMA-busy
# cycles and the GPU clock in one pass, LDS and vector-memory activity in a second.
set -u
TAG=${1:-pmccorr3}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
P1="SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_INSTS_VALU SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT"
P2="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INST_CYCLES_VMEM_RD SQ_WAVES SQ_INSTS_MFMA"
for mode in ${MODES:-1 4 0}; do
  for pass in 1 2; do
    C=$P1; [ $pass = 2 ] && C=$P2
    KRCA_CORR_DEBUG=$mode timeout -s KILL 200 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $O/m${mode}p$pass -o run -- python3 tools/prof_kernels.py corr --pods 100000 --reps 1 > $O/m${mode}p$pass.out 2> $O/m${mode}p$pass.err
    rc=$?; echo "m${mode}p$pass EXIT=$rc" >> $O/status
    [ $rc -eq 0 ] || { tail -3 $O/m${mode}p$pass.err; exit $rc; }
  done
done
find $O -name '*.db' -delete
for mode in ${MODES:-1 4 0}; do echo "== mode $mode"; python3 tools/pmc_summary.py $O/m${mode}p1 "corr_tiles<12, 0, 256>"; python3 tools/pmc_summary.py $O/m${mode}p2 "corr_tiles<12, 0, 256>"; done > $O/summary.txt
cat $O/summary.txt
echo all-done >> $O/status
