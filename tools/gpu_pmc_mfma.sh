#!/bin/bash
# GPU call: MFMA utilisation and memory counters of the correlation kernels
# at C3 (100k pods) and 1M pods, tau 0.5, one timed call after the warm-up (tools/prof_kernels.py
# corr).  Pass 1: MFMA-busy / issue / wait cycles and the GPU clock (8 SQ + 2 GRBM counters); pass 2:
# DRAM-side bytes (TCC 32-B units) and MFMA / LDS / VMEM instruction counts.  Each pass its own
# run under a kill timeout.  Report: tools/pmc_mfma_report.py.
set -u
TAG=${1:-pmcmfma}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
P1="SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_SALU SQ_INSTS_VALU SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT"
P2="TCC_EA0_RDREQ_DRAM_32B TCC_EA0_WRREQ_WRITE_DRAM_32B SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_WAVES"
for pods in ${PODS:-100000 1000000}; do
  for pass in 1 2; do
    C=$P1; [ $pass = 2 ] && C=$P2
    n=p${pods}_pass$pass
    timeout -s KILL ${PMC_SECS:-240} rocprofv3 --pmc $C --kernel-trace --output-format csv -d $O/$n -o run -- python3 tools/prof_kernels.py corr --pods $pods --reps 1 --tau 0.5 > $O/$n.out 2> $O/$n.err
    rc=$?; echo "$n EXIT=$rc" >> $O/status
    [ $rc -eq 0 ] || { tail -3 $O/$n.err; exit $rc; }
  done
done
find $O -name '*.db' -delete
python3 tools/pmc_mfma_report.py $O --out $O/pmc_mfma.json > $O/report.txt 2>&1
cat $O/report.txt
echo all-done >> $O/status
