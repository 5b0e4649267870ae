#!/bin/bash
# C3 (B = 256 bf16) step timeline: rocprofv3 kernel trace of the replayed step, per-queue busy time
# and the largest idle gaps (tools/timeline.py), by kernel.  Usage: bash tools/job_r3_o.sh OUTDIR
O=${1:-gpurun_out/r3_o}
mkdir -p "$O"
export TMPDIR=/tmp
ok() { local rc=$1; [ "$rc" -le 1 ] || { echo "stop rc=$rc"; exit "$rc"; }; }
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$O/prof_c3" -o run --output-format csv -- python bench.py --batch 256 --precision bf16 --steps 6 --warmup 2 --no-cpu-baseline --no-secondary --no-roofline --e2e 0 > "$O/prof_c3.log" 2>&1; ok $?
python tools/timeline.py "$O/prof_c3/run_kernel_trace.csv" --by-kernel > "$O/timeline_c3.txt" 2>&1
python tools/timeline.py "$O/prof_c3/run_kernel_trace.csv" --top 40 > "$O/timeline_c3_gaps.txt" 2>&1
head -5 "$O/timeline_c3.txt"
echo done
