#!/bin/bash
# Build lib/libkrca_<name>.so: corr.hip compiled with extra defines, linked with the other objects
# of the current build (run `make` first).  Usage: tools/build_corr_variant.sh <name> [-DX ...]
set -eu
N=$1; shift
C=kubernetes-rca-system_amd/csrc
mkdir -p $C/build/v_$N
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -ffp-contract=off "$@" \
  -c $C/corr.hip -o $C/build/v_$N/corr.o
OBJS=$(ls $C/build/*.o | grep -v '/corr.o$')
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o kubernetes-rca-system_amd/lib/libkrca_$N.so $OBJS $C/build/v_$N/corr.o
echo built kubernetes-rca-system_amd/lib/libkrca_$N.so
