#!/bin/bash
# HEAD evidence: encbwd test, kernel trace + stats of the bench step, per-op probes, GEMM sweep
# (auto plan vs hipBLASLt), one PMC pass of MFMA counters.  Every GPU step under its own time limit;
# stops at the first crash/timeout.  Usage: bash tools/job_prof.sh OUTDIR
O=${1:-gpurun_out/prof}
mkdir -p "$O"
ok() { local rc=$1; [ "$rc" -le 1 ] || { echo "stop rc=$rc"; exit "$rc"; }; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_x_encbwd.py -q --timeout 120 --timeout-method thread -p no:cacheprovider > "$O/t_encbwd.log" 2>&1; ok $?; tail -2 "$O/t_encbwd.log"
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-secondary --e2e 0 --dump-probes "$O/probes.json" > "$O/bench_probes.log" 2>&1; ok $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$O/rocprof" -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-secondary --e2e 0 > "$O/rocprof.log" 2>&1; ok $?
timeout -k 10 300 python tools/gemm_bench.py --quick --reps 10 > "$O/gemm_quick.log" 2>&1; ok $?; tail -2 "$O/gemm_quick.log"
timeout -s KILL 60 rocprofv3 -L > "$O/counters.txt" 2>&1
timeout -s KILL 180 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d "$O/pmc_mfma" -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-secondary --no-roofline --e2e 0 > "$O/pmc_mfma.log" 2>&1; ok $?
echo done
