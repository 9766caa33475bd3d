cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out/dbg && export TMPDIR=/tmp && \
KRCA_CORR_DEBUG=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/dbg/t1 -o run -- python3 tools/prof_kernels.py corr --pods 100000 --reps 2 > gpurun_out/dbg/c1.json 2>gpurun_out/dbg/e1.log && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/dbg/t0 -o run -- python3 tools/prof_kernels.py corr --pods 100000 --reps 2 > gpurun_out/dbg/c0.json 2>gpurun_out/dbg/e0.log; find gpurun_out/dbg -name '*trace.csv' -delete
