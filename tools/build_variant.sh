#!/bin/bash
# Build lib/libkrca_<name>.so: one source (corr / ppr / logscan / ...) compiled with extra defines,
# linked with the other objects of the current build (run `make` first).  Load it with KRCA_LIB.
# Usage: tools/build_variant.sh <name> <source stem> [-DX ...]
set -eu
N=$1; SRC=$2; shift 2
C=kubernetes-rca-system_amd/csrc
mkdir -p $C/build/v_$N
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -ffp-contract=off "$@" \
  -c $C/$SRC.hip -o $C/build/v_$N/$SRC.o
# the objects of the product build only (one per source file; not the ltime / gdbg / tcls variants)
OBJS=$(for f in $C/*.hip $C/*.cpp; do b=$(basename ${f%.*}); [ $b != $SRC ] && echo $C/build/$b.o; done)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o kubernetes-rca-system_amd/lib/libkrca_$N.so $OBJS $C/build/v_$N/$SRC.o
echo built kubernetes-rca-system_amd/lib/libkrca_$N.so
