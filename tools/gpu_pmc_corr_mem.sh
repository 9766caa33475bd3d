#!/bin/bash
# GPU call: memory-side counters of the correlation tile kernel (C3, product only, KRCA_CORR_DEBUG=1):
# DRAM-side read bytes (32-B units) and the L2 hit / miss split.  One counter group per run.
set -u
TAG=${1:-pmccorrmem}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
n=0
for C in "TCC_EA0_RDREQ_DRAM_32B TCC_EA0_WRREQ_WRITE_DRAM_32B" "TCC_HIT_sum TCC_MISS_sum" "TCC_EA0_RDREQ_sum TCC_REQ_sum"; do
  n=$((n+1))
  KRCA_CORR_DEBUG=1 timeout -s KILL 200 rocprofv3 --pmc $C --output-format csv -d $O/p$n -o run -- python3 tools/prof_kernels.py corr --pods 100000 --reps 1 > $O/p$n.out 2> $O/p$n.err
  rc=$?; echo "p$n EXIT=$rc" >> $O/status
  [ $rc -eq 0 ] || { tail -3 $O/p$n.err; exit $rc; }
done
find $O -name '*.db' -delete
for p in 1 2 3; do python3 tools/pmc_summary.py $O/p$p "corr_tiles<16, 0>"; done > $O/summary.txt
echo all-done >> $O/status
