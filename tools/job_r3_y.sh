#!/bin/bash
# wgrad_early levels 1 vs 2 (with skip_early + angle_side) at C2, then C3 base vs best: tools/job_r3_y.sh OUT
O=${1:-gpurun_out/r3_y}
mkdir -p "$O"
timeout -k 10 300 python -u -m pytest tests/test_gpu_x_pending.py -m gpu -x -q -k third_stream --timeout 120 --timeout-method thread -p no:cacheprovider > "$O/tests.log" 2>&1
rc=$?; tail -1 "$O/tests.log"; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" "$O/tests.log" | head; exit $rc; }
one() {
  local tag=$1; shift
  timeout -k 10 240 python bench.py --no-cpu-baseline --no-secondary --no-roofline --e2e 0 "$@" > "$O/one.json" 2>&1 || { tail -20 "$O/one.json"; exit 3; }
  echo "$tag: $(grep '^{' "$O/one.json" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")" | tee -a "$O/ab.log"
}
F="--set engine.skip_early=1 --set engine.angle_side=1"
for r in 1 2; do
  one "c2 base r$r" --steps 30 --warmup 5
  one "c2 w1 r$r" --steps 30 --warmup 5 $F --set engine.wgrad_early=1
  one "c2 w2 r$r" --steps 30 --warmup 5 $F --set engine.wgrad_early=2
done
for r in 1 2; do
  one "c3 base r$r" --steps 15 --warmup 3 --batch 256 --precision bf16
  one "c3 w1 r$r" --steps 15 --warmup 3 --batch 256 --precision bf16 $F --set engine.wgrad_early=1
  one "c3 w2 r$r" --steps 15 --warmup 3 --batch 256 --precision bf16 $F --set engine.wgrad_early=2
done
echo done
