#!/bin/bash
# GPU call: the C3 correlation (100k pods) A/B: the projection bound at one batch (KRCA_CORR_PROJ=2
# against the default 1) and 4096 candidate slots per pod (lib/libkrca_capc4k.so, no rectangle pass)
# against 2048, kernel-traced, alternated twice on one box.
set -u
TAG=${1:-corrc3ab}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
for r in 1 2; do
for lib in base capc4k; do
for pj in 1 2; do
  D=${lib}_p${pj}_$r
  if [ $lib = capc4k ]; then export KRCA_LIB=$PWD/kubernetes-rca-system_amd/lib/libkrca_capc4k.so; else unset KRCA_LIB; fi
  KRCA_CORR_PROJ=$pj timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$D -o run -- python3 tools/prof_kernels.py corr --pods ${PODS:-100000} --reps 5 > $O/$D.log 2>&1
  rc=$?; echo "$D EXIT=$rc" >> $O/status
  [ $rc -eq 0 ] || { tail -5 $O/$D.log; exit $rc; }
  find $O/$D -name '*.db' -delete
  echo "$D $(grep '^{' $O/$D.log | cut -c1-200)"
done
done
done
echo all-done >> $O/status
