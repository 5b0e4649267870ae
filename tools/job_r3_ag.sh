#!/bin/bash
# Re-measure stream-placement switches at HEAD (C2, same box, interleaved): overlap_forward 1/0,
# gate_reduce_side 1/0, enc_bwd_aux default/1.  Usage: tools/job_r3_ag.sh OUT
O=${1:-gpurun_out/r3_ag}
mkdir -p "$O"
one() {
  local tag=$1; shift
  timeout -k 10 240 python bench.py --no-cpu-baseline --no-secondary --no-roofline --e2e 0 --steps 30 --warmup 5 "$@" > "$O/one.json" 2>&1 || { tail -20 "$O/one.json"; exit 3; }
  echo "$tag: $(grep '^{' "$O/one.json" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")" | tee -a "$O/ab.log"
}
for r in 1 2; do
  one "base r$r"
  one "overlap_forward=0 r$r" --set engine.overlap_forward=0
  one "gate_reduce_side=0 r$r" --set engine.gate_reduce_side=0
  one "enc_bwd_aux=1 r$r" --set engine.enc_bwd_aux=1
done
echo done
