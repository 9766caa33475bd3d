#!/bin/bash
# GPU call: PageRank GPU tests on the current library, then the C4 step A/B: the current build
# (16 edges per ppr_step lane) against lib/libkrca_pprold.so (the previous build, 8 edges per lane),
# each bit-checked against the C oracle, kernel-traced.
set -u
TAG=${1:-pprseg}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "ppr or rca" > $O/tests.log 2>&1
  rc=$?; echo "tests EXIT=$rc" >> $O/status; tail -3 $O/tests.log
  [ $rc -eq 0 ] || { tail -40 $O/tests.log; exit $rc; }
fi
for v in new old new old; do
  if [ $v = old ]; then export KRCA_LIB=$PWD/kubernetes-rca-system_amd/lib/libkrca_pprold.so; else unset KRCA_LIB; fi
  D=$v$(ls -d $O/${v}[0-9] 2>/dev/null | wc -l)
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$D -o run -- python3 tools/ppr_bench.py --reps 10 --check > $O/$D.log 2>&1
  rc=$?; echo "$D EXIT=$rc" >> $O/status
  [ $rc -eq 0 ] || { tail -5 $O/$D.log; exit $rc; }
  find $O/$D -name '*.db' -delete
  echo "$D $(grep '^{' $O/$D.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print({k: d[k] for k in ("us_per_iter","bit_identical","top10_identical","blocks","dict_blocks")})')"
  python3 -c "import csv;[print('   ', r['Name'][:40], r['Calls'], round(float(r['AverageNs'])/1e3,2), 'us') for r in csv.DictReader(open('$O/$D/run_kernel_stats.csv')) if 'ppr_step' in r['Name']]"
done
echo all-done >> $O/status
