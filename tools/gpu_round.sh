#!/bin/bash
# One GPU call: tests, smoke, A/B of the scoring kernel, rocprof trace + PMC passes.
# usage: tools/gpu_round.sh TAG [quick]
set -u
TAG=${1:-r}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
finish() {  # keep the merge-back under gpurun's 64 MiB: drop databases, cap every file at 2 MiB
  find $OUT -name '*.db' -delete
  find $OUT -type f -size +2M | while read f; do tail -c 2000000 "$f" > "$f.tail" && mv "$f.tail" "$f"; done
}
trap finish EXIT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $OUT/gpu_tests.log 2>&1
echo "tests EXIT=$?" >> $OUT/status
for impl in 0 1 0 1; do
  KRCA_SCORE_IMPL=$impl timeout -k 10 120 python tools/prof_kernels.py score --reps 5 >> $OUT/score_ab_impl$impl.json 2>> $OUT/err.log || { echo "score ab failed" >> $OUT/status; exit 1; }
done
echo "ab done" >> $OUT/status
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 tools/prof_kernels.py score --reps 3 > $OUT/trace_score.json 2>> $OUT/err.log || echo "trace failed" >> $OUT/status
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- python3 tools/prof_kernels.py score --reps 2 > /dev/null 2>> $OUT/err.log || echo "pmc fetch failed" >> $OUT/status
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- python3 tools/prof_kernels.py score --reps 2 > /dev/null 2>> $OUT/err.log || echo "pmc write failed" >> $OUT/status
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU --output-format csv -d $OUT/pmc_sq -o run -- python3 tools/prof_kernels.py score --reps 2 > /dev/null 2>> $OUT/err.log || echo "pmc sq failed" >> $OUT/status
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $OUT/pmc_grbm -o run -- python3 tools/prof_kernels.py score --reps 2 > /dev/null 2>> $OUT/err.log || echo "pmc grbm failed" >> $OUT/status
echo "pmc done" >> $OUT/status
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_ppr -o run -- python3 tools/prof_kernels.py ppr --reps 3 > $OUT/trace_ppr.json 2>> $OUT/err.log || echo "ppr trace failed" >> $OUT/status
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_logs -o run -- python3 tools/prof_kernels.py logs --reps 3 > $OUT/trace_logs.json 2>> $OUT/err.log || echo "logs trace failed" >> $OUT/status
timeout -k 10 400 python -u bench.py --steps 10 --warmup 2 > $OUT/bench.json 2> $OUT/bench.err || echo "bench failed" >> $OUT/status
echo "extra done" >> $OUT/status
