#!/bin/bash
# GPU call: a PageRank step variant (lib/libkrca_<VAR>.so, tools/build_variant.sh) against the current
# build: the PageRank / RCA GPU tests on the variant, then the C4 step alternated base / variant, each
# bit-checked against the C oracle and kernel-traced.  Usage: tools/gpu_ppr_ab.sh TAG VAR
set -u
TAG=${1:-pprab}
VAR=${2:?variant name}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
VLIB=$PWD/kubernetes-rca-system_amd/lib/libkrca_$VAR.so
KRCA_LIB=$VLIB timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_kernels.py -k "ppr or rca" > $O/tests.log 2>&1
rc=$?; echo "tests EXIT=$rc" >> $O/status; tail -3 $O/tests.log
[ $rc -eq 0 ] || { tail -40 $O/tests.log; exit $rc; }
for D in base1 $VAR'1' base2 $VAR'2'; do
  case $D in base*) unset KRCA_LIB;; *) export KRCA_LIB=$VLIB;; esac
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$D -o run -- python3 tools/ppr_bench.py --reps 10 --check > $O/$D.log 2>&1
  rc=$?; echo "$D EXIT=$rc" >> $O/status
  [ $rc -eq 0 ] || { tail -5 $O/$D.log; exit $rc; }
  find $O/$D -name '*.db' -delete
  echo "$D $(grep '^{' $O/$D.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print({k: d.get(k) for k in ("us_per_working_iter","iters_run","bit_identical","top10_identical")})')"
  python3 -c "import csv;[print('   ', r['Name'][:40], r['Calls'], round(float(r['AverageNs'])/1e3,2), 'us') for r in csv.DictReader(open('$O/$D/run_kernel_stats.csv')) if 'ppr_step' in r['Name']]"
done
echo all-done >> $O/status
