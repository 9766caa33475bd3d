#!/bin/bash
# GPU call: the correlation at C3 and 1M per KRCA_CORR_KM_EXTRA (candidates the merge re-scores in
# float64 past the k-th), kernel-traced.
set -u
TAG=${1:-corrkm}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
for pods in ${PODSL:-100000 1000000}; do
for km in ${KMS:-6 2 4 6 2 4}; do
  D=km${km}_${pods}_$(ls -d $O/km${km}_${pods}_* 2>/dev/null | wc -l)
  reps=5; [ $pods -ge 1000000 ] && reps=1
  KRCA_CORR_KM_EXTRA=$km timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$D -o run -- python3 tools/prof_kernels.py corr --pods $pods --reps $reps > $O/$D.log 2>&1
  rc=$?; echo "$D EXIT=$rc" >> $O/status
  [ $rc -eq 0 ] || { tail -5 $O/$D.log; exit $rc; }
  find $O/$D -name '*.db' -delete
  echo "$D $(grep '^{' $O/$D.log | cut -c1-130)"
  python3 -c "import csv;[print('   ', r['Name'][32:60], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us') for r in csv.DictReader(open('$O/$D/run_kernel_stats.csv')) if 'merge' in r['Name']]"
done
done
echo all-done >> $O/status
