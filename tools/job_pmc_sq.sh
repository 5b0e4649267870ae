#!/bin/bash
# SQ instruction-mix counters of the step's kernels (one pass, 8 SQ counters) + FETCH/WRITE passes.
O=${1:-gpurun_out/sq}
mkdir -p "$O"
ok() { local rc=$1; [ "$rc" -le 1 ] || { echo "stop rc=$rc"; exit "$rc"; }; }
B="python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-secondary --no-roofline --e2e 0"
timeout -s KILL 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU --kernel-trace -d "$O/sq" -o run --output-format csv -- $B > "$O/sq.log" 2>&1; ok $?
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$O/fetch" -o run --output-format csv -- $B > "$O/fetch.log" 2>&1; ok $?
timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$O/write" -o run --output-format csv -- $B > "$O/write.log" 2>&1; ok $?
echo done
