#!/bin/bash
# bf16 encoder backward on the matrix cores: its tests and the C3/bf16 step tests, then same-box A/B
# (C3: matrix-core kernel vs the fp32 VALU kernel, and a 768-workgroup grid; B = 32: the grid), and a
# kernel trace of C3.  Usage: bash tools/job_r3_q.sh OUTDIR
O=${1:-gpurun_out/r3_q}
mkdir -p "$O"
export TMPDIR=/tmp
V768=gnn-elasticity-predictor_amd/alignn_mi355x/variants/libalignn_hip_eb768.so
ok() { local rc=$1; [ "$rc" -le 1 ] || { echo "stop rc=$rc"; exit "$rc"; }; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_x_encbwd.py tests/test_gpu_x_configs.py tests/test_gpu_x_bf16.py -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > "$O/tests_first.log" 2>&1
rc=$?; tail -3 "$O/tests_first.log"; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" "$O/tests_first.log" | head -20; exit $rc; }
one() {  # one TAG LIB FLAGS...
  local tag=$1 lib=$2; shift 2
  if [ "$lib" = "-" ]; then unset ALIGNN_HIP_LIB; else export ALIGNN_HIP_LIB=$lib; fi
  timeout -k 10 240 python bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-secondary --no-roofline --e2e 0 "$@" > "$O/one.json" 2>&1 || { tail -20 "$O/one.json"; exit 3; }
  echo "$tag: $(grep '^{' "$O/one.json" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")" | tee -a "$O/ab.log"
  unset ALIGNN_HIP_LIB
}
for r in 1 2; do
  one "c3 mfma r$r" - --batch 256 --precision bf16
  one "c3 valu r$r" - --batch 256 --precision bf16 --set engine.enc_bwd_mfma=0
  one "c3 mfma768 r$r" $V768 --batch 256 --precision bf16
done
for r in 1 2 3; do
  one "b32 r$r" -
  one "b32 eb768 r$r" $V768
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/prof_c3" -o run --output-format csv -- python bench.py --batch 256 --precision bf16 --steps 6 --warmup 2 --no-cpu-baseline --no-secondary --no-roofline --e2e 0 > "$O/prof_c3.log" 2>&1; ok $?
grep -h "enc_bwd" "$O/prof_c3/run_kernel_stats.csv" | cut -c1-150
python tools/timeline.py "$O/prof_c3/run_kernel_trace.csv" --by-kernel > "$O/timeline_c3.txt" 2>&1
head -4 "$O/timeline_c3.txt"
echo done
