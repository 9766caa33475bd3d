#!/bin/bash
# GPU call: PageRank step variants (libkrca_<v>.so) at C4: per-iteration time, bit identity, and
# the per-phase cycle split of the timer builds (t<v>).
set -u
TAG=${1:-ppr4}
O=gpurun_out/$TAG
mkdir -p $O
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
L=kubernetes-rca-system_amd/lib
for v in ${VARIANTS:-a b c}; do
  for d in 1 0; do
    KRCA_LIB=$L/libkrca_$v.so timeout -k 10 200 python3 tools/ppr_bench.py --dict $d --check > $O/$v-d$d.log 2>&1
    rc=$?; echo "$v-d$d EXIT=$rc" >> $O/status
    [ $rc -eq 0 ] || { tail -20 $O/$v-d$d.log; exit $rc; }
    echo "$v dict=$d $(grep -o '"us_per_iter": [0-9.]*\|"bit_identical": [a-z]*' $O/$v-d$d.log | tr '\n' ' ')"
  done
  if [ -f $L/libkrca_t$v.so ]; then
    KRCA_LIB=$L/libkrca_t$v.so timeout -k 10 200 python3 tools/ppr_timing.py > $O/t$v.log 2>&1
    rc=$?; echo "t$v EXIT=$rc" >> $O/status
    [ $rc -eq 0 ] || { tail -20 $O/t$v.log; exit $rc; }
    echo "t$v $(tail -1 $O/t$v.log)"
  fi
done
echo all-done >> $O/status
