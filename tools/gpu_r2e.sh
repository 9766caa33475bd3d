#!/bin/bash
# GPU call: tools/gpu_r2b.sh (full -m gpu suite, bench, traces) then the exact-bytes counter
# passes on the C4 PageRank step (tools/gpu_pmc_exact.sh's formulas).
set -u
TAG=${1:-r2e}
bash tools/gpu_r2b.sh $TAG || exit $?
O=gpurun_out/$TAG
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
for p in "rd TCC_EA0_RDREQ_sum TCC_BUBBLE_sum TCC_EA0_RDREQ_32B_sum" "dram TCC_EA0_RDREQ_DRAM_32B TCC_EA0_WRREQ_WRITE_DRAM_32B" "wr TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum"; do
  set -- $p
  name=ppr_$1; shift
  timeout -s KILL 150 rocprofv3 --pmc "$@" --output-format csv -d $O/$name -o run -- python3 tools/ppr_bench.py --reps 2 > $O/$name.out 2> $O/$name.err
  rc=$?; echo "$name EXIT=$rc" >> $O/status
  [ $rc -eq 0 ] || { tail -3 $O/$name.err; exit $rc; }
done
find $O -name '*.db' -delete
python3 tools/pmc_exact_report.py $O --out $O/pmc_exact.json > $O/report.txt 2>&1
echo pmc-done >> $O/status
