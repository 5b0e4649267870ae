#!/bin/bash
# Packed edge-pair encoder backward: its tests, then a same-box A/B against the previous kernel
# (B = 32 fp32 and C3 B = 256 bf16, alternating), a kernel trace of each, then every -m gpu test.
# Usage: bash tools/job_r3_n.sh OUTDIR
O=${1:-gpurun_out/r3_n}
mkdir -p "$O"
export TMPDIR=/tmp
OLD=gnn-elasticity-predictor_amd/alignn_mi355x/variants/libalignn_hip_encold.so
ok() { local rc=$1; [ "$rc" -le 1 ] || { echo "stop rc=$rc"; exit "$rc"; }; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_x_encbwd.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > "$O/tests_encbwd.log" 2>&1
rc=$?; tail -3 "$O/tests_encbwd.log"; [ $rc -eq 0 ] || { grep -E "FAIL|Error" "$O/tests_encbwd.log" | head; exit $rc; }
ab() {  # ab TAG ROUNDS FLAGS...
  local tag=$1 rounds=$2; shift 2
  for r in $(seq "$rounds"); do
    for lib in new old; do
      if [ $lib = old ]; then export ALIGNN_HIP_LIB=$OLD; else unset ALIGNN_HIP_LIB; fi
      timeout -k 10 240 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-secondary --e2e 0 "$@" > "$O/ab_one.json" 2>&1 || { tail -20 "$O/ab_one.json"; exit 3; }
      v=$(grep '^{' "$O/ab_one.json" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")
      echo "$tag round $r $lib: $v" | tee -a "$O/ab.log"
    done
  done
  unset ALIGNN_HIP_LIB
}
ab b32 3
ab c3 2 --batch 256 --precision bf16
for lib in new old; do
  if [ $lib = old ]; then export ALIGNN_HIP_LIB=$OLD; else unset ALIGNN_HIP_LIB; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof_$lib" -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-secondary --no-roofline --e2e 0 > "$O/prof_$lib.log" 2>&1; ok $?
  grep -h "enc_bwd" "$O/prof_$lib/run_kernel_stats.csv" | cut -c1-160
done
unset ALIGNN_HIP_LIB
bash tools/job_tests_all.sh "$O"; ok $?
echo done
