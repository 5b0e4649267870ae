#!/bin/bash
# Wave-grouped CSR atomics + plan-referenced re-binding copies: the CSR and capture tests first, then
# every -m gpu test + smoke, the default bench line (e2e fields), and a kernel trace of the e2e loop.
# Usage: bash tools/job_r3_m.sh OUTDIR
O=${1:-gpurun_out/r3_m}
mkdir -p "$O"
ok() { local rc=$1; [ "$rc" -le 1 ] || { echo "stop rc=$rc"; exit "$rc"; }; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_graph.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > "$O/tests_first.log" 2>&1
rc=$?; tail -3 "$O/tests_first.log"; [ $rc -eq 0 ] || { grep -E "FAIL|Error" "$O/tests_first.log" | head; exit $rc; }
bash tools/job_tests_all.sh "$O"; ok $?
timeout -k 10 600 python bench.py > "$O/bench.json" 2> "$O/bench.err"; ok $?
cut -c1-300 "$O/bench.json"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$O/rocprof_e2e" -o run --output-format csv -- python tools/prof_prepare.py --batch 32 --graphs 2000 --steps 30 > "$O/rocprof_e2e.log" 2>&1; ok $?
echo done
