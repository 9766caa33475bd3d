#!/bin/bash
# GPU call: main-pass tile kernel time per KRCA_CORR_DEBUG mode (0 full, 1 product only, 4 product
# only with L2-resident operands), kernel-traced at C3.
set -u
TAG=${1:-corrmodes}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
for m in ${MODES:-0 1 4}; do
  KRCA_CORR_DEBUG=$m timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/m$m -o run -- python3 tools/prof_kernels.py corr --pods ${PODS:-100000} --reps 3 > $O/m$m.log 2>&1
  rc=$?; echo "m$m EXIT=$rc" >> $O/status
  [ $rc -eq 0 ] || { tail -5 $O/m$m.log; exit $rc; }
  find $O/m$m -name '*.db' -delete
  python3 -c "import csv;[print('mode $m', r['Name'][:40], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us') for r in csv.DictReader(open('$O/m$m/run_kernel_stats.csv')) if 'corr_tiles<16, 0>' in r['Name']]"
done
