#!/bin/bash
# A/B of the in-tree library against one variant build, with optional GPU tests on the variant:
#   tools/job_var.sh OUTDIR VARIANT_NAME [TESTS...]
O=$1; V=$PWD/gnn-elasticity-predictor_amd/alignn_mi355x/variants/libalignn_hip_$2.so; shift 2
mkdir -p "$O"
ok() { local rc=$1; [ "$rc" -le 1 ] || { echo "stop rc=$rc"; exit "$rc"; }; }
if [ $# -gt 0 ]; then
  ALIGNN_HIP_LIB=$V timeout -k 10 400 python -u -m pytest "$@" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > "$O/t.log" 2>&1; rc=$?; tail -1 "$O/t.log"; ok $rc
  [ $rc -eq 0 ] || exit 1
fi
rm -f gpurun_out/ab.log
bash tools/ab_libs.sh 3 - $V; ok $?
cp gpurun_out/ab.log "$O/ab.log"
ALIGNN_HIP_LIB=$V timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-secondary --e2e 0 --dump-probes "$O/probes_var.json" > "$O/bp.log" 2>&1; ok $?
