#!/bin/bash
# GPU call: exact HBM-side bytes per kernel from the TCC/EA request-size counters (no FETCH_SIZE
# correction factor): read bytes = 32*RDREQ_32B + 64*(RDREQ - RDREQ_32B - BUBBLE) + 128*BUBBLE
# (TCC_BUBBLE = 128-B read requests), DRAM-side bytes = 32*RDREQ_DRAM_32B / 32*WRREQ_WRITE_DRAM_32B
# (the 32-B unit counters).  Targets: tools/pmc_calib (known byte counts), the C4 PageRank step
# and the bench step (TARGETS="..." picks others: corr = the C3 correlation, with an L2 hit pass).  One counter group per run, each under its own kill timeout.
set -u
TAG=${1:-pmcx}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
pass() {  # pass NAME COUNTERS -- CMD...
  local name=$1; shift
  local ctr=()
  while [ "$1" != "--" ]; do ctr+=("$1"); shift; done; shift
  timeout -s KILL 150 rocprofv3 --pmc "${ctr[@]}" --output-format csv -d $O/$name -o run -- "$@" > $O/$name.out 2> $O/$name.err
  local rc=$?; echo "$name EXIT=$rc" >> $O/status
  [ $rc -eq 0 ] || { tail -3 $O/$name.err; exit $rc; }
}
for t in ${TARGETS:-cal ppr bench logs logs_fused}; do
  unset KRCA_LOG_FUSED
  case $t in
    cal) cmd=(tools/bin/pmc_calib) ;;
    ppr) cmd=(python3 tools/ppr_bench.py --reps 2) ;;
    bench) cmd=(python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-verify --no-pipeline --no-corr) ;;
    logs) cmd=(python3 tools/prof_kernels.py logs --docs 1000000 --reps 1) ;;
    logs250k) cmd=(python3 tools/prof_kernels.py logs --docs 250000 --reps 1) ;;
    logs_fused) export KRCA_LOG_FUSED=2; cmd=(python3 tools/prof_kernels.py logs --docs 1000000 --reps 1) ;;
    corr) cmd=(python3 tools/prof_kernels.py corr --pods 100000 --reps 1) ;;
    tmpl) cmd=(python3 tools/prof_kernels.py tmpl --docs 1000000 --reps 1) ;;
  esac
  [ $t = corr ] && pass ${t}_l2 TCC_HIT_sum TCC_MISS_sum -- "${cmd[@]}"
  pass ${t}_rd TCC_EA0_RDREQ_sum TCC_BUBBLE_sum TCC_EA0_RDREQ_32B_sum -- "${cmd[@]}"
  pass ${t}_dram TCC_EA0_RDREQ_DRAM_32B TCC_EA0_WRREQ_WRITE_DRAM_32B -- "${cmd[@]}"
  pass ${t}_wr TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum -- "${cmd[@]}"
done
find $O -name '*.db' -delete
python3 tools/pmc_exact_report.py $O --out $O/pmc_exact.json > $O/report.txt 2>&1
echo all-done >> $O/status
