#!/bin/bash
O=${1:-gpurun_out/plan}
mkdir -p "$O"
V=$PWD/gnn-elasticity-predictor_amd/alignn_mi355x/variants
ok() { local rc=$1; [ "$rc" -le 1 ] || { echo "stop rc=$rc"; exit "$rc"; }; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_x_gemm_pipe.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > "$O/t.log" 2>&1; rc=$?; tail -1 "$O/t.log"; ok $rc
timeout -k 10 300 python tools/gemm_bench.py --quick --reps 10 > "$O/gq_new.log" 2>&1; ok $?; tail -1 "$O/gq_new.log"
ALIGNN_HIP_LIB=$V/libalignn_hip_planv1.so timeout -k 10 300 python tools/gemm_bench.py --quick --reps 10 > "$O/gq_v1.log" 2>&1; ok $?; tail -1 "$O/gq_v1.log"
bash tools/ab_libs.sh 3 - $V/libalignn_hip_planv1.so; ok $?
cp gpurun_out/ab.log "$O/ab.log"
