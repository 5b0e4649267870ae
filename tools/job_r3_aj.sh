#!/bin/bash
# HIP-graph replay vs native plans at HEAD (C2 bare step and the e2e loop), same box.
O=${1:-gpurun_out/r3_aj}
mkdir -p "$O"
for r in 1 2; do
  for m in plan graph; do
    timeout -k 10 300 python bench.py --launch $m --steps 30 --warmup 5 --no-cpu-baseline --no-secondary --no-roofline --e2e 3000 > "$O/$m.json" 2> "$O/$m.err" || { tail -20 "$O/$m.err"; exit 3; }
    echo "r$r $m: $(grep '^{' "$O/$m.json" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], 'e2e', d['e2e']['value'], d['e2e']['host_ms_per_step'], 'var', d['e2e_variable']['value'])")" | tee -a "$O/ab.log"
  done
done
echo done
