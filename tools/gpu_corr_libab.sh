#!/bin/bash
# GPU call: correlation at C3 per library variant (lib/libkrca_<v>.so, "base" = libkrca.so), in
# interleaved rounds on one box, kernel-traced; optional GPU correlation tests per variant.
set -u
TAG=${1:-corrlib}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
L=kubernetes-rca-system_amd/lib
lib() { [ $1 = base ] && echo $L/libkrca.so || echo $L/libkrca_$1.so; }
if [ "${TESTS:-0}" = 1 ]; then
  for v in ${VARIANTS:-base}; do
    KRCA_LIB=$(lib $v) timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_corr.py > $O/tests_$v.log 2>&1
    rc=$?; echo "tests_$v EXIT=$rc" >> $O/status; echo "tests $v: $(tail -1 $O/tests_$v.log)"
    [ $rc -eq 0 ] || { tail -40 $O/tests_$v.log; exit $rc; }
  done
fi
for r in $(seq ${ROUNDS:-2}); do
for v in ${VARIANTS:-base}; do
  D=$v-r$r
  KRCA_LIB=$(lib $v) KRCA_CORR_DEBUG=${MODE:-0} timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$D -o run -- python3 tools/prof_kernels.py corr --pods ${PODS:-100000} --reps ${REPS:-3} --tau ${TAU:-0.5} > $O/$D.log 2>&1
  rc=$?; echo "$D EXIT=$rc" >> $O/status
  [ $rc -eq 0 ] || { tail -5 $O/$D.log; exit $rc; }
  find $O/$D -name '*.db' -delete
  echo "$D $(grep '^{' $O/$D.log | cut -c1-90)"
  python3 -c "import csv;[print('   ', r['Name'][32:62], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us') for r in csv.DictReader(open('$O/$D/run_kernel_stats.csv')) if 'corr_tiles<' in r['Name'] or 'rescore' in r['Name'] or 'merge' in r['Name']]"
done
done
echo all-done >> $O/status
