#!/bin/bash
# GPU call: correlation tests (exact counts, certificates, C3 every row), the C3 profile.
set -u
TAG=${1:-corr3}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
step() {  # step NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $O/$name.log 2>&1
  local rc=$?; echo "$name EXIT=$rc" >> $O/status
  [ $rc -eq 0 ] || { tail -30 $O/$name.log; exit $rc; }
}
step tests 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_corr.py tests/test_gpu_scale.py -k "corr or c2mini"
step prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 tools/prof_kernels.py corr --pods 100000 --reps 3
tail -3 $O/tests.log; grep '^{' $O/prof.log | cut -c1-600
python3 -c "import csv;[print(r['Name'][:70], r['Calls'], round(float(r['AverageNs'])/1e3,1)) for r in csv.DictReader(open('$O/prof/run_kernel_stats.csv')) if 'corr' in r['Name']]"
echo all-done >> $O/status
timeout -k 10 300 python3 tools/prof_kernels.py corr --pods 100000 --reps 3 --tau 0.8 > $O/prof_tau08.log 2>&1; echo "tau08 EXIT=$?" >> $O/status
grep '^{' $O/prof_tau08.log | cut -c1-300
