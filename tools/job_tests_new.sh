#!/bin/bash
# New-round GPU tests first (configs C3/C4/C5, plan/workspace safety), then a quick bench line.
O=${1:-gpurun_out/t}
mkdir -p "$O"
ok() { local rc=$1; [ "$rc" -le 1 ] || { echo "stop rc=$rc"; exit "$rc"; }; }
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu tests/test_gpu_x_configs.py tests/test_gpu_graph.py > "$O/tests.log" 2>&1; ok $?
tail -25 "$O/tests.log"
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-secondary --e2e 0 > "$O/bench_quick.log" 2>&1; ok $?
tail -c 600 "$O/bench_quick.log"
