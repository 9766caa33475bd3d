#!/bin/bash
set -u
OUT=gpurun_out/diag1
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-verify > $OUT/bench_default.json 2> $OUT/e1 && \
timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --iters 0 --no-cpu-baseline --no-verify > $OUT/bench_noppr.json 2> $OUT/e2 && \
timeout -k 10 300 python -u tools/score_ab.py --reps 20 --only ring_buf,pipe_c20,pipe_c30 > $OUT/ab.json 2> $OUT/e3
rc=$?
for f in bench_default bench_noppr; do python3 -c "import json;d=json.load(open('$OUT/$f.json'));print('$f', d['ms_per_step'], d['roofline']['avg_launch_ms'])"; done
cat $OUT/ab.json
exit $rc
