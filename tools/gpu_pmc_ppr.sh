#!/bin/bash
# GPU call: list the counters, then PMC passes (one block group per pass) on the PPR step and the
# correlation tiles.  Each pass is a separate short run under its own kill timeout.
set -u
TAG=${1:-pmc}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -s KILL 60 rocprofv3 -L > $OUT/counters.txt 2>&1; echo "list EXIT=$?" >> $OUT/status
pass() {  # pass NAME WHAT COUNTERS...
  local name=$1 what=$2; shift 2
  timeout -s KILL 90 rocprofv3 --pmc "$@" --output-format csv -d $OUT/$name -o run -- python3 tools/prof_kernels.py $what --reps 1 > $OUT/$name.out 2> $OUT/$name.err
  local rc=$?; echo "$name EXIT=$rc" >> $OUT/status
  [ $rc -eq 0 ] || { tail -3 $OUT/$name.err; exit $rc; }
}
pass ppr_tcc ppr TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum
pass ppr_ea ppr TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum
pass ppr_tcp ppr TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum
pass ppr_sq ppr SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_LDS
pass ppr_grbm ppr GRBM_GUI_ACTIVE GRBM_COUNT
find $OUT -name '*.db' -delete
echo done >> $OUT/status
