#!/bin/bash
# Batch-preparation host syncs removed: every -m gpu test + smoke, the host profile of the e2e loop
# (fixed and variable-size graphs), a bench line; then the matrix-core attention prototype's second
# iteration (ab/libalignn_hip_lgm2.so) against the in-tree VALU kernels.  Usage: bash tools/job_r3_i.sh OUTDIR
O=${1:-gpurun_out/r3_i}
mkdir -p "$O"
ok() { local rc=$1; [ "$rc" -le 1 ] || { echo "stop rc=$rc"; exit "$rc"; }; }
bash tools/job_tests_all.sh "$O"; ok $?
timeout -k 10 300 python tools/prof_prepare.py --batch 32 --graphs 2000 --steps 30 > "$O/host_prepare_b32.txt" 2>&1; ok $?
head -3 "$O/host_prepare_b32.txt"
timeout -k 10 300 python tools/prof_prepare.py --batch 32 --graphs 2000 --steps 30 --variable > "$O/host_prepare_b32_variable.txt" 2>&1; ok $?
head -3 "$O/host_prepare_b32_variable.txt"
timeout -k 10 300 python tools/lgm_bench.py > "$O/lgm_old.json" 2> "$O/lgm_old.err"; ok $?
ALIGNN_HIP_LIB=$PWD/gnn-elasticity-predictor_amd/ab/libalignn_hip_lgm2.so timeout -k 10 300 python tools/lgm_bench.py > "$O/lgm_2.json" 2> "$O/lgm_2.err"; ok $?
cat "$O/lgm_old.json" "$O/lgm_2.json"
timeout -k 10 600 python bench.py > "$O/bench.json" 2> "$O/bench.err"; ok $?
cut -c1-400 "$O/bench.json"
