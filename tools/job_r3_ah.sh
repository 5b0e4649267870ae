#!/bin/bash
# Re-measure switches at C3 (B = 256 bf16) at HEAD, same box, interleaved.  Usage: tools/job_r3_ah.sh OUT
O=${1:-gpurun_out/r3_ah}
mkdir -p "$O"
one() {
  local tag=$1; shift
  timeout -k 10 240 python bench.py --no-cpu-baseline --no-secondary --no-roofline --e2e 0 --steps 15 --warmup 3 --batch 256 --precision bf16 "$@" > "$O/one.json" 2>&1 || { tail -20 "$O/one.json"; exit 3; }
  echo "$tag: $(grep '^{' "$O/one.json" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")" | tee -a "$O/ab.log"
}
for r in 1 2; do
  one "c3 base r$r"
  one "c3 wgrad_early=2 r$r" --set engine.wgrad_early=2
  one "c3 gate_reduce_side=0 r$r" --set engine.gate_reduce_side=0
  one "c3 overlap_forward=0 r$r" --set engine.overlap_forward=0
done
echo done
