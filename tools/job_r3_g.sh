#!/bin/bash
# MFMA bf16 line-graph attention: standalone A/B vs the VALU kernels, then every -m gpu test + smoke,
# then the default bench.  Usage: bash tools/job_r3_g.sh OUTDIR
O=${1:-gpurun_out/r3_g}
mkdir -p "$O"
ok() { local rc=$1; [ "$rc" -le 1 ] || { echo "stop rc=$rc"; exit "$rc"; }; }
timeout -k 10 60 tools/bin/mfma_probe > "$O/mfma_probe_4x4x4.json"; ok $?
timeout -k 10 300 python tools/lgm_bench.py > "$O/lgm_new.json" 2> "$O/lgm_new.err"; ok $?
cat "$O/lgm_new.json"
ALIGNN_HIP_LIB=$PWD/gnn-elasticity-predictor_amd/alignn_mi355x/libalignn_hip_lgmx.so timeout -k 10 300 python tools/lgm_bench.py > "$O/lgm_x.json" 2> "$O/lgm_x.err"; ok $?
cat "$O/lgm_x.json"
ALIGNN_HIP_LIB=$PWD/gnn-elasticity-predictor_amd/alignn_mi355x/libalignn_hip_lgm16.so timeout -k 10 300 python tools/lgm_bench.py > "$O/lgm_16.json" 2> "$O/lgm_16.err"; ok $?
cat "$O/lgm_16.json"
ALIGNN_HIP_LIB=$PWD/gnn-elasticity-predictor_amd/alignn_mi355x/libalignn_hip_lg3bf.so timeout -k 10 300 python tools/lgm_bench.py > "$O/lgm_old.json" 2> "$O/lgm_old.err"; ok $?
cat "$O/lgm_old.json"
bash tools/job_tests_all.sh "$O"; ok $?
timeout -k 10 600 python bench.py > "$O/bench.json" 2> "$O/bench.err"; ok $?
cut -c1-600 "$O/bench.json"
