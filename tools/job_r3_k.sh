#!/bin/bash
# Split-K reduce with several threads per element + finer column-sum chunks: every -m gpu test + smoke,
# two default bench lines, a rocprofv3 kernel trace of the B = 32 step.  Usage: bash tools/job_r3_k.sh OUTDIR
O=${1:-gpurun_out/r3_k}
mkdir -p "$O"
ok() { local rc=$1; [ "$rc" -le 1 ] || { echo "stop rc=$rc"; exit "$rc"; }; }
bash tools/job_tests_all.sh "$O"; ok $?
timeout -k 10 600 python bench.py > "$O/bench1.json" 2> "$O/bench1.err"; ok $?
timeout -k 10 300 python bench.py --no-secondary --no-cpu-baseline --e2e 0 > "$O/bench2.json" 2> "$O/bench2.err"; ok $?
cut -c1-200 "$O/bench1.json" "$O/bench2.json"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$O/rocprof" -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --no-secondary --no-cpu-baseline --e2e 0 > "$O/rocprof.log" 2>&1; ok $?
python tools/timeline.py "$O/rocprof/run_kernel_trace.csv" --by-kernel > "$O/timeline.txt" 2>&1
head -3 "$O/timeline.txt"
