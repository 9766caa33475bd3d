#!/bin/bash
# GPU call: PageRank step variants (libkrca_v*.so builds) at C4, kernel-traced.
set -u
TAG=${1:-ppr3}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
L=kubernetes-rca-system_amd/lib
for v in v1 v2 v3 v4; do
  for d in 1 0; do
    KRCA_LIB=$L/libkrca_$v.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$v-d$d -o run -- python3 tools/ppr_bench.py --dict $d --check > $O/$v-d$d.log 2>&1
    rc=$?; echo "$v-d$d EXIT=$rc" >> $O/status
    [ $rc -eq 0 ] || { tail -20 $O/$v-d$d.log; exit $rc; }
    echo "$v dict=$d $(grep -h '"ppr_step' $O/$v-d$d/run_kernel_stats.csv | cut -d, -f2-4 | tr '\n' ' ') $(grep -o '"us_per_iter": [0-9.]*\|"bit_identical": [a-z]*' $O/$v-d$d.log | tr '\n' ' ')"
  done
done
echo all-done >> $O/status
