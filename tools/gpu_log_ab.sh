#!/bin/bash
# GPU call: log-scan variants (lib/libkrca_<VAR>.so, tools/build_variant.sh) against the current build:
# the log GPU tests on each variant, then the two-pass scan's kernels (tools/prof_kernels.py logs)
# alternated base / variants, twice.  Usage: tools/gpu_log_ab.sh TAG VAR [VAR ...]
set -u
TAG=${1:-logab}; shift
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
L=$PWD/kubernetes-rca-system_amd/lib
for V in "$@"; do
  KRCA_LIB=$L/libkrca_$V.so timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_kernels.py tests/test_gpu_c5_full.py tests/test_gpu_stream.py -k "log or c5 or stream" > $O/tests_$V.log 2>&1
  rc=$?; echo "tests_$V EXIT=$rc" >> $O/status; tail -1 $O/tests_$V.log
  [ $rc -eq 0 ] || { tail -40 $O/tests_$V.log; exit $rc; }
done
for r in 1 2; do
for V in base "$@"; do
  D=${V}_$r
  if [ $V = base ]; then unset KRCA_LIB; else export KRCA_LIB=$L/libkrca_$V.so; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$D -o run -- python3 tools/prof_kernels.py logs --reps 5 > $O/$D.log 2>&1
  rc=$?; echo "$D EXIT=$rc" >> $O/status
  [ $rc -eq 0 ] || { tail -5 $O/$D.log; exit $rc; }
  find $O/$D -name '*.db' -delete
  python3 -c "import csv;[print('$D', r['Name'][22:48], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us') for r in csv.DictReader(open('$O/$D/run_kernel_stats.csv')) if 'log_' in r['Name'] and int(r['Calls']) > 2]"
done
done
echo all-done >> $O/status
