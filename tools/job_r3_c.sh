#!/bin/bash
O=${1:-gpurun_out/r3_c}
mkdir -p "$O"
ok() { local rc=$1; [ "$rc" -le 1 ] || { echo "stop rc=$rc"; exit "$rc"; }; }
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu tests/test_gpu_x_gemm_pipe.py tests/test_gpu_x_bf16_stream.py tests/test_gpu_x_bf16.py tests/test_gpu_kernels.py > "$O/tests_gemm.log" 2>&1; ok $?
tail -2 "$O/tests_gemm.log"
timeout -k 10 400 python tools/gemm_bench.py --quick --reps 10 --flag 1024 > "$O/gemm_kw.log" 2>&1; ok $?
tail -1 "$O/gemm_kw.log"
V=gnn-elasticity-predictor_amd/alignn_mi355x/variants/libalignn_hip_kwauto.so
timeout -k 10 900 bash tools/ab_libs.sh 3 - $V > "$O/ab.log" 2>&1; ok $?
cat "$O/ab.log"
