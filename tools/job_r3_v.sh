#!/bin/bash
# After the bf16 matrix-core encoder backward: the kernel/config/parity/plan tests, the default bench
# line (all secondary fields), and a C3 kernel trace + timeline.  Usage: bash tools/job_r3_v.sh OUTDIR
O=${1:-gpurun_out/r3_v}
mkdir -p "$O"
export TMPDIR=/tmp
ok() { local rc=$1; [ "$rc" -le 1 ] || { echo "stop rc=$rc"; exit "$rc"; }; }
timeout -k 10 500 python -u -m pytest tests/test_gpu_x_encbwd.py tests/test_gpu_x_configs.py tests/test_gpu_x_bf16.py tests/test_gpu_parity.py tests/test_gpu_graph.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > "$O/tests.log" 2>&1
rc=$?; tail -2 "$O/tests.log"; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" "$O/tests.log" | head -20; exit $rc; }
timeout -k 10 600 python bench.py > "$O/bench.json" 2> "$O/bench.err"; ok $?
cut -c1-200 "$O/bench.json"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$O/prof_c3" -o run --output-format csv -- python bench.py --batch 256 --precision bf16 --steps 6 --warmup 2 --no-cpu-baseline --no-secondary --no-roofline --e2e 0 > "$O/prof_c3.log" 2>&1; ok $?
python tools/timeline.py "$O/prof_c3/run_kernel_trace.csv" --by-kernel > "$O/timeline_c3.txt" 2>&1
head -4 "$O/timeline_c3.txt"
echo done
