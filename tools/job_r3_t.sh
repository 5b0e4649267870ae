#!/bin/bash
# Matrix-core deferred encoder backward, fp32 and bf16: its tests, standalone timings (C3 and B = 32
# sizes), same-box A/B against the VALU kernel (B = 32 and C3), then every -m gpu test + smoke.
# Usage: bash tools/job_r3_t.sh OUTDIR
O=${1:-gpurun_out/r3_t}
mkdir -p "$O"
ok() { local rc=$1; [ "$rc" -le 1 ] || { echo "stop rc=$rc"; exit "$rc"; }; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_x_encbwd.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > "$O/tests_encbwd.log" 2>&1
rc=$?; tail -2 "$O/tests_encbwd.log"; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" "$O/tests_encbwd.log" | head -20; exit $rc; }
timeout -k 10 300 python tools/encbwd_bench.py 2>&1 | grep -v amdgpu.ids | tee "$O/encbwd_bench.txt"
timeout -k 10 300 python tools/encbwd_bench.py --b32 2>&1 | grep -v amdgpu.ids | tee -a "$O/encbwd_bench.txt"
one() {
  local tag=$1; shift
  timeout -k 10 240 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-secondary --no-roofline --e2e 0 "$@" > "$O/one.json" 2>&1 || { tail -20 "$O/one.json"; exit 3; }
  echo "$tag: $(grep '^{' "$O/one.json" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")" | tee -a "$O/ab.log"
}
for r in 1 2 3; do
  one "b32 mfma r$r"
  one "b32 valu r$r" --set engine.enc_bwd_mfma=0
done
one "c3 mfma" --batch 256 --precision bf16
one "c3 valu" --batch 256 --precision bf16 --set engine.enc_bwd_mfma=0
bash tools/job_tests_all.sh "$O"; ok $?
echo done
