#!/bin/bash
# Evidence at HEAD: every -m gpu test, smoke, the default bench line, C3 kernel trace timeline.
O=${1:-gpurun_out/r3_ev}
mkdir -p "$O"
ok() { local rc=$1; [ "$rc" -le 1 ] || { echo "stop rc=$rc"; exit "$rc"; }; }
bash tools/job_tests_all.sh "$O"; ok $?
timeout -k 10 600 python bench.py > "$O/bench.json" 2> "$O/bench.err"; ok $?
cut -c1-300 "$O/bench.json"
timeout -k 10 400 rocprofv3 --kernel-trace -d "$O/rocprof3" -o run --output-format csv -- python bench.py --steps 6 --warmup 2 --batch 256 --precision bf16 --no-cpu-baseline --no-secondary --no-roofline --e2e 0 > "$O/rocprof3.log" 2>&1; ok $?
f=$(find "$O/rocprof3" -name "run_kernel_trace.csv" | head -1)
python tools/timeline.py "$f" --by-kernel --sequence > "$O/timeline_c3.txt" 2>&1
rm -rf "$O/rocprof3"
echo done
