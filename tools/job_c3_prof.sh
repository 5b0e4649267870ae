#!/bin/bash
# Config C3 evidence (B = 256, bf16): bench line, kernel trace + stats, FETCH_SIZE / WRITE_SIZE /
# MFMA-busy passes (each its own run).  Every GPU step under its own time limit; stops at the first
# crash/timeout.  Usage: bash tools/job_c3_prof.sh OUTDIR [extra bench args...]
O=${1:-gpurun_out/c3}
shift || true
mkdir -p "$O"
ok() { local rc=$1; [ "$rc" -le 1 ] || { echo "stop rc=$rc"; exit "$rc"; }; }
B=(bench.py --batch 256 --precision bf16 --no-cpu-baseline --no-secondary --e2e 0 "$@")
timeout -k 10 300 python "${B[@]}" --steps 10 --warmup 3 --dump-probes "$O/probes.json" > "$O/bench.log" 2>&1; ok $?
tail -c 1500 "$O/bench.log"
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$O/rocprof" -o run --output-format csv -- python "${B[@]}" --steps 10 --warmup 3 > "$O/rocprof.log" 2>&1; ok $?
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$O/pmc_fetch" -o run --output-format csv -- python "${B[@]}" --steps 3 --warmup 1 --no-roofline > "$O/pmc_fetch.log" 2>&1; ok $?
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$O/pmc_write" -o run --output-format csv -- python "${B[@]}" --steps 3 --warmup 1 --no-roofline > "$O/pmc_write.log" 2>&1; ok $?
timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d "$O/pmc_mfma" -o run --output-format csv -- python "${B[@]}" --steps 3 --warmup 1 --no-roofline > "$O/pmc_mfma.log" 2>&1; ok $?
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU --kernel-trace -d "$O/pmc_sq" -o run --output-format csv -- python "${B[@]}" --steps 3 --warmup 1 --no-roofline > "$O/pmc_sq.log" 2>&1; ok $?
python tools/pmc_traffic.py "$O/pmc_fetch" "$O/pmc_write" --json "$O/pmc_traffic.json" > "$O/pmc_traffic.txt" 2>&1
echo done
