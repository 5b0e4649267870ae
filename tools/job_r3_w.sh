#!/bin/bash
# bf16 encoder backward, one 32-column tile per wave (8-wave workgroups, 4 waves/SIMD) vs two (4-wave
# workgroups, 3 waves/SIMD): its tests under the variant, standalone timings, C3 A/B.
O=${1:-gpurun_out/r3_w}
mkdir -p "$O"
V=gnn-elasticity-predictor_amd/alignn_mi355x/variants/libalignn_hip_ebnt1.so
ALIGNN_HIP_LIB=$V timeout -k 10 300 python -u -m pytest tests/test_gpu_x_encbwd.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > "$O/tests_nt1.log" 2>&1
rc=$?; tail -1 "$O/tests_nt1.log"; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" "$O/tests_nt1.log" | head; exit $rc; }
timeout -k 10 300 python tools/encbwd_bench.py 2>&1 | grep -v amdgpu.ids | sed 's/^/nt2 /' | tee "$O/encbwd_bench.txt"
ALIGNN_HIP_LIB=$V timeout -k 10 300 python tools/encbwd_bench.py 2>&1 | grep -v amdgpu.ids | sed 's/^/nt1 /' | tee -a "$O/encbwd_bench.txt"
one() {
  local tag=$1 lib=$2; shift 2
  if [ "$lib" = "-" ]; then unset ALIGNN_HIP_LIB; else export ALIGNN_HIP_LIB=$lib; fi
  timeout -k 10 240 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-secondary --no-roofline --e2e 0 "$@" > "$O/one.json" 2>&1 || { tail -20 "$O/one.json"; exit 3; }
  echo "$tag: $(grep '^{' "$O/one.json" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")" | tee -a "$O/ab.log"
  unset ALIGNN_HIP_LIB
}
for r in 1 2; do
  one "c3 nt2 r$r" - --batch 256 --precision bf16
  one "c3 nt1 r$r" $V --batch 256 --precision bf16
done
echo done
