#!/bin/bash
# f3 betweenness timing + kernel trace: bash tools/gpu_bc.sh TAG
set -e
T=${1:-bc}; O=gpurun_out/$T; mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for n in 20000 50000; do
  for b in 1024 2048; do
    timeout -k 10 240 python3 tools/prof_kernels.py bc --pods $n --reps 1 --batch $b >> $O/bc.log 2>&1
  done
done
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/prof -o bc -- python3 tools/prof_kernels.py bc --pods 20000 --reps 1 > $O/prof.log 2>&1
find $O/prof -name '*kernel_stats.csv' -exec cp {} $O/bc20k_kernel_stats.csv \;
cat $O/bc.log
