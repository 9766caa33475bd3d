#!/bin/bash
# GPU call: FETCH_SIZE calibration (tools/pmc_calib) and PMC passes on the C4 PageRank step
# (tools/ppr_bench.py), one counter group per run (MI355X_MICROARCH.md §HBM / rocprofv3 limits).
set -u
TAG=${1:-pmc2}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
pass() {  # pass NAME COUNTERS -- CMD...
  local name=$1; shift
  local ctr=()
  while [ "$1" != "--" ]; do ctr+=("$1"); shift; done; shift
  timeout -s KILL 120 rocprofv3 --pmc "${ctr[@]}" --output-format csv -d $O/$name -o run -- "$@" > $O/$name.out 2> $O/$name.err
  local rc=$?; echo "$name EXIT=$rc" >> $O/status
  [ $rc -eq 0 ] || { tail -3 $O/$name.err; exit $rc; }
}
pass cal_fetch FETCH_SIZE -- tools/bin/pmc_calib
pass cal_write WRITE_SIZE -- tools/bin/pmc_calib
pass cal_ea TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum -- tools/bin/pmc_calib
pass cal_tcc TCC_HIT_sum TCC_MISS_sum -- tools/bin/pmc_calib
pass ppr_fetch FETCH_SIZE -- python3 tools/ppr_bench.py --reps 2
pass ppr_write WRITE_SIZE -- python3 tools/ppr_bench.py --reps 2
pass ppr_ea TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum -- python3 tools/ppr_bench.py --reps 2
pass ppr_tcc TCC_HIT_sum TCC_MISS_sum -- python3 tools/ppr_bench.py --reps 2
pass ppr_sq SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_LDS -- python3 tools/ppr_bench.py --reps 2
cat $O/cal_fetch.out
find $O -name '*.db' -delete
echo all-done >> $O/status
