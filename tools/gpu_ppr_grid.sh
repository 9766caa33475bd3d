#!/bin/bash
set -u
OUT=gpurun_out/pprgrid
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
for G in 0 512 1024 1280 1536 2048 3072; do
  if [ $G -eq 0 ]; then unset KRCA_PPR_GRID; else export KRCA_PPR_GRID=$G; fi
  timeout -k 10 200 python tools/prof_kernels.py ppr --reps 5 > $OUT/g$G.json 2>> $OUT/err.log || exit 1
  echo "G=$G $(cat $OUT/g$G.json)"
done
