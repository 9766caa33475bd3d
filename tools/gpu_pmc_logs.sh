#!/bin/bash
# PMC passes on the log scan kernels (log_count / log_match / log_hist): one counter group per run,
# no trace domains, each pass under its own kill timeout.  bash tools/gpu_pmc_logs.sh TAG
set -u
TAG=${1:-pmclogs}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
pass() {  # pass NAME COUNTERS...
  local name=$1; shift
  timeout -s KILL 150 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$name -o run -- python3 tools/prof_kernels.py logs --docs 300000 --reps 1 > $OUT/$name.out 2> $OUT/$name.err
  local rc=$?; echo "$name EXIT=$rc" >> $OUT/status
  [ $rc -eq 0 ] || { tail -3 $OUT/$name.err; exit $rc; }
}
pass sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD
pass sq2 SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM_RD
pass mem TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCC_HIT_sum TCC_MISS_sum
find $OUT -name '*.db' -delete
echo done >> $OUT/status
