#!/bin/bash
# Builds an A/B variant of libalignn_hip.so with extra compile flags, for kernel experiments:
#   tools/build_variant.sh NAME [FLAGS...]  ->  gnn-elasticity-predictor_amd/alignn_mi355x/variants/libalignn_hip_NAME.so
# Select it at run time with ALIGNN_HIP_LIB=<path>.
set -e
name=$1; shift
root=$(cd "$(dirname "$0")/.." && pwd)
src=$root/gnn-elasticity-predictor_amd/csrc
out=$root/gnn-elasticity-predictor_amd/alignn_mi355x/variants
bdir=$src/build_$name
mkdir -p "$out" "$bdir"
pids=()
for path in "$src"/*.hip; do
  f=$(basename "$path" .hip)
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function "$@" \
    -c "$path" -o "$bdir/$f.o" &
  pids+=($!)
done
for p in "${pids[@]}"; do wait "$p"; done
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -fPIC "$bdir"/*.o -o "$out/libalignn_hip_$name.so"
echo "$out/libalignn_hip_$name.so"
