#!/bin/bash
# Deferred encoder backward with its gradient sums on the matrix cores: the encoder-backward tests,
# every -m gpu test + smoke, then a same-box A/B of bench lines against the previous kernel
# (ab/libalignn_hip_ebold.so) at B = 32 (fp32) and config C3.  Usage: bash tools/job_r3_l.sh OUTDIR
O=${1:-gpurun_out/r3_l}
mkdir -p "$O"
ok() { local rc=$1; [ "$rc" -le 1 ] || { echo "stop rc=$rc"; exit "$rc"; }; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_x_encbwd.py -v --timeout 120 --timeout-method thread -p no:cacheprovider > "$O/encbwd_tests.log" 2>&1; ok $?
tail -2 "$O/encbwd_tests.log"
bash tools/job_tests_all.sh "$O"; ok $?
OLD=$PWD/gnn-elasticity-predictor_amd/ab/libalignn_hip_ebold.so
for r in 1 2; do
  timeout -k 10 300 python bench.py --no-secondary --no-cpu-baseline --e2e 0 > "$O/ab_new_$r.json" 2>&1; ok $?
  ALIGNN_HIP_LIB=$OLD timeout -k 10 300 python bench.py --no-secondary --no-cpu-baseline --e2e 0 > "$O/ab_old_$r.json" 2>&1; ok $?
  timeout -k 10 300 python bench.py --batch 256 --precision bf16 --no-secondary --no-cpu-baseline --e2e 0 --steps 10 --warmup 3 > "$O/ab_c3_new_$r.json" 2>&1; ok $?
  ALIGNN_HIP_LIB=$OLD timeout -k 10 300 python bench.py --batch 256 --precision bf16 --no-secondary --no-cpu-baseline --e2e 0 --steps 10 --warmup 3 > "$O/ab_c3_old_$r.json" 2>&1; ok $?
done
for f in "$O"/ab_*.json; do python -c "
import json; d=json.loads([l for l in open('$f') if l.startswith('{')][-1]); print('$f', d['value'], d['ms_per_step'])"; done
