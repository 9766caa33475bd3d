#!/bin/bash
# GPU call: PMC passes over the correlation kernels (one counter group per run).
set -u
TAG=${1:-corrpmc}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
run() {  # name counters...
  local name=$1; shift
  timeout -s KILL 120 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$name -o run -- python3 tools/prof_kernels.py corr --pods 100000 --reps 1 > /dev/null 2>> $OUT/err.log || { echo "$name failed" >> $OUT/status; return 1; }
  echo "$name ok" >> $OUT/status
}
run sq1 SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE && \
run sq2 SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_WAIT_INST_ANY && \
run grbm GRBM_GUI_ACTIVE GRBM_COUNT && \
run fetch FETCH_SIZE
find $OUT -name '*.db' -delete
