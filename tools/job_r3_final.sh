#!/bin/bash
# Round-3 evidence at HEAD: every -m gpu test + smoke, the default bench line, a rocprofv3 kernel
# trace + stats of the default single-GPU bench (config C2 timed region), FETCH_SIZE / WRITE_SIZE /
# MFMA-busy passes of the C2 step (each in its own run), and a kernel trace of the e2e loop (what the
# loader stream adds per step).  Usage: bash tools/job_r3_final.sh OUTDIR
O=${1:-gpurun_out/r3_final}
mkdir -p "$O"
ok() { local rc=$1; [ "$rc" -le 1 ] || { echo "stop rc=$rc"; exit "$rc"; }; }
bash tools/job_tests_all.sh "$O"; ok $?
timeout -k 10 600 python bench.py > "$O/bench.json" 2> "$O/bench.err"; ok $?
cut -c1-300 "$O/bench.json"
B=(bench.py --no-secondary --no-cpu-baseline --e2e 0)
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$O/rocprof" -o run --output-format csv -- python "${B[@]}" --steps 10 --warmup 3 > "$O/rocprof.log" 2>&1; ok $?
python tools/timeline.py "$O/rocprof/run_kernel_trace.csv" --by-kernel > "$O/timeline.txt" 2>&1
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$O/pmc_fetch" -o run --output-format csv -- python "${B[@]}" --steps 3 --warmup 1 --no-roofline > "$O/pmc_fetch.log" 2>&1; ok $?
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$O/pmc_write" -o run --output-format csv -- python "${B[@]}" --steps 3 --warmup 1 --no-roofline > "$O/pmc_write.log" 2>&1; ok $?
timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d "$O/pmc_mfma" -o run --output-format csv -- python "${B[@]}" --steps 3 --warmup 1 --no-roofline > "$O/pmc_mfma.log" 2>&1; ok $?
python tools/pmc_traffic.py "$O/pmc_fetch" "$O/pmc_write" --json "$O/pmc_traffic.json" > "$O/pmc_traffic.txt" 2>&1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$O/rocprof_e2e" -o run --output-format csv -- python tools/prof_prepare.py --batch 32 --graphs 2000 --steps 30 > "$O/rocprof_e2e.log" 2>&1; ok $?
echo done
