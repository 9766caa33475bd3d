#!/bin/bash
# GPU call: krca_corr_topk at 1M pods x 1440 steps on one GPU (k = 10, tau = 0.9), kernel trace.
set -u
TAG=${1:-corr1m}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 tools/prof_kernels.py corr --pods 1000000 --reps 1 --tau 0.9 > $O/prof.log 2>&1
rc=$?; echo "prof EXIT=$rc" >> $O/status
[ $rc -eq 0 ] || { tail -20 $O/prof.log; exit $rc; }
grep '^{' $O/prof.log | cut -c1-600
python3 -c "import csv;[print(r['Name'][:70], r['Calls'], round(float(r['AverageNs'])/1e6,2), 'ms') for r in csv.DictReader(open('$O/prof/run_kernel_stats.csv')) if 'corr' in r['Name']]"
echo all-done >> $O/status
