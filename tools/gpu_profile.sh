#!/bin/bash
# GPU call 2: rocprofv3 kernel-trace stats of the bench command itself, FETCH/WRITE PMC passes
# (separate runs, no tracing domains combined with --pmc), and per-kernel traces of corr/logs.
# usage: tools/gpu_profile.sh TAG
set -u
TAG=${1:-prof}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
finish() {
  find $OUT -name '*.db' -delete
  find $OUT -name '*kernel_trace.csv' -size +4M -delete
  find $OUT -type f -size +4M | while read f; do tail -c 2000000 "$f" > "$f.tail" && mv "$f.tail" "$f"; done
}
trap finish EXIT
step() {  # step NAME TIMEOUT CMD...
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $OUT/$name.out 2> $OUT/$name.err
  local rc=$?; echo "$name EXIT=$rc" >> $OUT/status
  case $rc in 0) ;; *) echo "stop after $name"; tail -5 $OUT/$name.err; exit $rc;; esac
}
step bench_trace 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/bench_trace -o run -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline
step pmc_fetch 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-verify
step pmc_write 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-verify
step corr_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/corr_trace -o run -- python3 tools/prof_kernels.py corr --pods 100000 --reps 3
step logs_trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/logs_trace -o run -- python3 tools/prof_kernels.py logs --reps 3
cat $OUT/bench_trace.out
echo done >> $OUT/status
