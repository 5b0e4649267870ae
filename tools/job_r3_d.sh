#!/bin/bash
# Multi-rank bench rehearsal on a one-GPU box (2 ranks on cuda:0, gloo), then the gemm tests, then the
# default bench line.
O=${1:-gpurun_out/r3_d}
mkdir -p "$O"
ok() { local rc=$1; [ "$rc" -le 1 ] || { echo "stop rc=$rc"; exit "$rc"; }; }
timeout -k 10 600 python bench.py --gpus 2 --dist-backend gloo --share-device --steps 5 --warmup 2 --e2e 600 > "$O/bench_2rank_rehearsal.log" 2>&1; ok $?
grep '^{' "$O/bench_2rank_rehearsal.log" | cut -c1-400
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread -p no:cacheprovider -m gpu tests/test_gpu_x_gemm_pipe.py tests/test_gpu_x_bf16_stream.py tests/test_gpu_x_bf16.py > "$O/tests_gemm.log" 2>&1; ok $?
tail -1 "$O/tests_gemm.log"
timeout -k 10 600 python bench.py > "$O/bench_default.log" 2>&1; ok $?
grep '^{' "$O/bench_default.log" | cut -c1-300
