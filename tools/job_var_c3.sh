#!/bin/bash
# C3 (B=256 bf16) A/B of the in-tree library against a variant: tools/job_var_c3.sh OUTDIR VARIANT [TESTS...]
O=$1; V=$PWD/gnn-elasticity-predictor_amd/alignn_mi355x/variants/libalignn_hip_$2.so; shift 2
mkdir -p "$O"
ok() { local rc=$1; [ "$rc" -le 1 ] || { echo "stop rc=$rc"; exit "$rc"; }; }
if [ $# -gt 0 ]; then
  timeout -k 10 400 python -u -m pytest "$@" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > "$O/t.log" 2>&1; rc=$?; tail -1 "$O/t.log"; ok $rc
  [ $rc -eq 0 ] || exit 1
fi
timeout -k 10 300 python tools/gemm_bench.py --quick --reps 5 --batch 256 --precision bf16 > "$O/gq.log" 2>&1; ok $?; tail -1 "$O/gq.log"
for r in 1 2; do for lib in - $V; do
  if [ "$lib" = "-" ]; then unset ALIGNN_HIP_LIB; else export ALIGNN_HIP_LIB=$lib; fi
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --batch 256 --precision bf16 --no-cpu-baseline --no-secondary --e2e 0 > "$O/b.log" 2>&1; ok $?
  echo "round $r lib $(basename $lib): $(tail -1 "$O/b.log" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")" | tee -a "$O/ab.log"
done; done
