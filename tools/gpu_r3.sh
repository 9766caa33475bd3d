#!/bin/bash
# Round-3 GPU call: a chosen list of named steps, each under its own time limit, stopping at the
# first failure.  usage: tools/gpu_r3.sh TAG step [step ...]
#   tests        all -m gpu tests            bench        bench.py default line
#   bench_trace  rocprofv3 stats of bench.py corr100k     rocprofv3 stats, C3 correlation (tau 0.5)
#   corr1m       rocprofv3 stats, 1M-pod correlation (tau 0.5)
#   ranking      tools/ranking_ablation_c4.py (C4 mesh, 2 seeds)
#   ppr          rocprofv3 stats of the C4 PageRank propagate   logs / tmpl  same for logs / templates
#   c5           tools/bench_stream.py (C5 window)
set -u
TAG=$1; shift
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
finish() {
  find $O -name '*.db' -delete
  find $O -name '*kernel_trace.csv' -size +4M -delete
}
trap finish EXIT
step() {  # step NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $O/$name.log 2>&1
  local rc=$?; echo "$name EXIT=$rc" >> $O/status
  [ $rc -eq 0 ] || { echo "stop after $name"; tail -30 $O/$name.log; exit $rc; }
  tail -3 $O/$name.log
}
prof() {  # prof NAME SECONDS ARGS... (rocprofv3 kernel-trace stats of python3 ARGS)
  local name=$1 secs=$2; shift 2
  step $name $secs rocprofv3 --kernel-trace --stats --output-format csv -d $O/$name -o run -- python3 "$@"
}
for s in "$@"; do
  case $s in
    tests) step tests 900 python3 -u -m pytest tests -m gpu -x -v -rP --timeout 240 --timeout-method thread ;;
    tests_corr) step tests_corr 600 python3 -u -m pytest tests/test_gpu_corr.py -x -v -rP --timeout 240 --timeout-method thread ;;
    bench) step bench 300 python3 bench.py ;;
    bench_trace) prof bench_trace 400 bench.py --steps 10 --warmup 2 --no-cpu-baseline ;;
    corr100k) prof corr100k 300 tools/prof_kernels.py corr --pods 100000 --reps 3 --tau 0.5 ;;
    corr1m) prof corr1m 600 tools/prof_kernels.py corr --pods 1000000 --reps 1 --tau 0.5 ;;
    ranking) step ranking 600 python3 -u tools/ranking_ablation_c4.py --seeds 2 --out $O/ranking_ablation_c4.json ;;
    ppr) prof ppr 300 tools/prof_kernels.py ppr --reps 5 ;;
    logs) prof logs 300 tools/prof_kernels.py logs --reps 5 ;;
    tmpl) prof tmpl 300 tools/prof_kernels.py tmpl --reps 5 ;;
    c5) step c5 400 python3 -u tools/bench_stream.py ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo all-done >> $O/status
