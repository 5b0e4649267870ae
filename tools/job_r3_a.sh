#!/bin/bash
O=${1:-gpurun_out/r3_a}
mkdir -p "$O"
ok() { local rc=$1; [ "$rc" -le 1 ] || { echo "stop rc=$rc"; exit "$rc"; }; }
bash tools/job_tests_all.sh "$O" ; ok $?
timeout -k 10 500 python tools/gemm_bench.py --reps 10 --json "$O/gemm_sweep.json" > "$O/gemm_sweep.log" 2>&1; ok $?
tail -3 "$O/gemm_sweep.log"
