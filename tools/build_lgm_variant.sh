#!/bin/bash
# A/B variant of libalignn_hip.so that recompiles only lgmma.hip with extra flags and links it with the
# in-tree objects (csrc/build/*.o, from `make`): tools/build_lgm_variant.sh NAME [FLAGS...]
#   -> gnn-elasticity-predictor_amd/alignn_mi355x/variants/libalignn_hip_NAME.so (ALIGNN_HIP_LIB=<path>)
set -e
name=$1; shift
root=$(cd "$(dirname "$0")/.." && pwd)
src=$root/gnn-elasticity-predictor_amd/csrc
out=$root/gnn-elasticity-predictor_amd/alignn_mi355x/variants
mkdir -p "$out" "$src/build_$name"
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function "$@" -c "$src/lgmma.hip" \
  -o "$src/build_$name/lgmma.o"
objs=$(ls "$src"/build/*.o | grep -v '/lgmma.o$')
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -fPIC $objs "$src/build_$name/lgmma.o" -o "$out/libalignn_hip_$name.so"
echo "$out/libalignn_hip_$name.so"
