#!/bin/bash
# Stream-placement options (skip_early, angle_side, wgrad_early): their bitwise tests, then a same-box
# A/B at C2 (B = 32 fp32), interleaved rounds; optional C3 pair: tools/job_r3_x.sh OUT [c3]
O=${1:-gpurun_out/r3_x}
mkdir -p "$O"
timeout -k 10 300 python -u -m pytest tests/test_gpu_x_pending.py -m gpu -x -q -k third_stream --timeout 120 --timeout-method thread -p no:cacheprovider > "$O/tests.log" 2>&1
rc=$?; tail -1 "$O/tests.log"; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" "$O/tests.log" | head; exit $rc; }
one() {
  local tag=$1; shift
  timeout -k 10 240 python bench.py --no-cpu-baseline --no-secondary --no-roofline --e2e 0 "$@" > "$O/one.json" 2>&1 || { tail -20 "$O/one.json"; exit 3; }
  echo "$tag: $(grep '^{' "$O/one.json" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")" | tee -a "$O/ab.log"
}
ALL="--set engine.skip_early=1 --set engine.angle_side=1 --set engine.wgrad_early=1"
if [ "$2" = "c3" ]; then
  for r in 1 2; do
    one "c3 base r$r" --steps 15 --warmup 3 --batch 256 --precision bf16
    one "c3 all r$r" --steps 15 --warmup 3 --batch 256 --precision bf16 $ALL
  done
  exit 0
fi
for r in 1 2; do
  one "c2 base r$r" --steps 30 --warmup 5
  one "c2 skip_early r$r" --steps 30 --warmup 5 --set engine.skip_early=1
  one "c2 angle_side r$r" --steps 30 --warmup 5 --set engine.angle_side=1
  one "c2 wgrad_early r$r" --steps 30 --warmup 5 --set engine.wgrad_early=1
  one "c2 all r$r" --steps 30 --warmup 5 $ALL
done
echo done
