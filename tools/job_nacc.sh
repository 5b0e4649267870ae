#!/bin/bash
O=${1:-gpurun_out/nacc}
mkdir -p "$O"
V=$PWD/gnn-elasticity-predictor_amd/alignn_mi355x/variants
ok() { local rc=$1; [ "$rc" -le 1 ] || { echo "stop rc=$rc"; exit "$rc"; }; }
ALIGNN_HIP_LIB=$V/libalignn_hip_nacc4.so timeout -k 10 300 python -u -m pytest tests/test_gpu_x_gemm_pipe.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > "$O/t4.log" 2>&1; ok $?; tail -1 "$O/t4.log"
for lib in - $V/libalignn_hip_nacc2.so $V/libalignn_hip_nacc4.so; do
  if [ "$lib" = "-" ]; then unset ALIGNN_HIP_LIB; else export ALIGNN_HIP_LIB=$lib; fi
  timeout -k 10 300 python tools/gemm_bench.py --quick --reps 10 > "$O/gq_$(basename $lib).log" 2>&1; ok $?; tail -1 "$O/gq_$(basename $lib).log"
done
unset ALIGNN_HIP_LIB
bash tools/ab_libs.sh 2 - $V/libalignn_hip_nacc2.so $V/libalignn_hip_nacc4.so; ok $?
cp gpurun_out/ab.log "$O/ab.log"
