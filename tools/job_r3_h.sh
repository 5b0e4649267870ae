#!/bin/bash
# Every -m gpu test + smoke at HEAD, then SQ / MFMA / LDS counters of the matrix-core line-graph
# attention prototype (gnn-elasticity-predictor_amd/ab/libalignn_hip_lgmx.so) on the C3 line graph.
# Usage: bash tools/job_r3_h.sh OUTDIR
O=${1:-gpurun_out/r3_h}
mkdir -p "$O"
ok() { local rc=$1; [ "$rc" -le 1 ] || { echo "stop rc=$rc"; exit "$rc"; }; }
bash tools/job_tests_all.sh "$O"; ok $?
export ALIGNN_HIP_LIB=$PWD/gnn-elasticity-predictor_amd/ab/libalignn_hip_lgmx.so
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU --kernel-trace -d "$O/pmc_sq" -o run --output-format csv -- python tools/lgm_bench.py --reps 3 > "$O/pmc_sq.log" 2>&1; ok $?
python tools/pmc_sq.py "$O/pmc_sq" --top 8 > "$O/pmc_sq.txt" 2>&1
timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_LDS_BANK_CONFLICT --kernel-trace -d "$O/pmc_mfma" -o run --output-format csv -- python tools/lgm_bench.py --reps 3 > "$O/pmc_mfma.log" 2>&1; ok $?
echo done
