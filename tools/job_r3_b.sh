#!/bin/bash
O=${1:-gpurun_out/r3_b}
mkdir -p "$O"
ok() { local rc=$1; [ "$rc" -le 1 ] || { echo "stop rc=$rc"; exit "$rc"; }; }
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests/test_gpu_graph.py tests/test_gpu_x_capacity.py tests/test_gpu_x_configs.py tests/test_gpu_x_dataset.py > "$O/tests.log" 2>&1; ok $?
grep -E "passed|failed" "$O/tests.log" | tail -2
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$O/rocprof" -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-secondary --e2e 0 > "$O/rocprof.log" 2>&1; ok $?
python tools/timeline.py "$O/rocprof/run_kernel_trace.csv" --by-kernel --top 25 > "$O/timeline.txt" 2>&1
timeout -k 10 300 python tools/prof_prepare.py --batch 32 --graphs 2000 --steps 30 > "$O/prof_prepare_b32.txt" 2>&1; ok $?
head -3 "$O/prof_prepare_b32.txt"
timeout -k 10 300 python tools/prof_prepare.py --batch 32 --graphs 2000 --steps 30 --variable > "$O/prof_prepare_b32_var.txt" 2>&1; ok $?
head -3 "$O/prof_prepare_b32_var.txt"
