#!/bin/bash
# Variant of libalignn_hip.so that recompiles one source with extra flags and links it with the
# in-tree objects (csrc/build/*.o, run `make` first):
#   tools/build_lgvariant.sh NAME SOURCE.hip [FLAGS...] -> alignn_mi355x/variants/libalignn_hip_NAME.so
set -e
name=$1; src_name=$2; shift 2
root=$(cd "$(dirname "$0")/.." && pwd)
src=$root/gnn-elasticity-predictor_amd/csrc
out=$root/gnn-elasticity-predictor_amd/alignn_mi355x/variants
bdir=$src/build_$name
mkdir -p "$out" "$bdir"
base=$(basename "$src_name" .hip)
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wall -Wno-unused-function "$@" \
  -c "$src/$base.hip" -o "$bdir/$base.o"
objs=()
for o in "$src"/build/*.o; do
  if [ "$(basename "$o")" = "$base.o" ]; then objs+=("$bdir/$base.o"); else objs+=("$o"); fi
done
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -fPIC "${objs[@]}" -o "$out/libalignn_hip_$name.so"
echo "$out/libalignn_hip_$name.so"
