#!/bin/bash
# GPU call: correlation tests, then the 100k and 1M-pod profiles (chunked threshold sample).
set -u
TAG=${1:-corr4}
bash tools/gpu_corr3.sh $TAG || exit $?
O=gpurun_out/$TAG
cd $GRAFT_REPO_ROOT
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof1m -o run -- python3 tools/prof_kernels.py corr --pods 1000000 --reps 1 --tau 0.9 > $O/prof1m.log 2>&1
rc=$?; echo "prof1m EXIT=$rc" >> $O/status
[ $rc -eq 0 ] || { tail -20 $O/prof1m.log; exit $rc; }
grep '^{' $O/prof1m.log | cut -c1-600
python3 -c "import csv;[print(r['Name'][:70], r['Calls'], round(float(r['AverageNs'])/1e6,2), 'ms') for r in csv.DictReader(open('$O/prof1m/run_kernel_stats.csv')) if 'corr' in r['Name']]"
echo all1m-done >> $O/status
