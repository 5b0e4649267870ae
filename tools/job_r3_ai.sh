#!/bin/bash
# proj_per_layer: its test + the stream tests, then a same-box A/B at C2 and C3.
O=${1:-gpurun_out/r3_ai}
mkdir -p "$O"
timeout -k 10 300 python -u -m pytest tests/test_gpu_x_pending.py -m gpu -x -q -k "third_stream or atom_blocks or proj_per_layer" --timeout 120 --timeout-method thread -p no:cacheprovider > "$O/tests.log" 2>&1
rc=$?; tail -1 "$O/tests.log"; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" "$O/tests.log" | head -20; exit $rc; }
one() {
  local tag=$1; shift
  timeout -k 10 240 python bench.py --no-cpu-baseline --no-secondary --no-roofline --e2e 0 "$@" > "$O/one.json" 2>&1 || { tail -20 "$O/one.json"; exit 3; }
  echo "$tag: $(grep '^{' "$O/one.json" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")" | tee -a "$O/ab.log"
}
for r in 1 2 3; do
  one "c2 base r$r" --steps 30 --warmup 5
  one "c2 proj_per_layer r$r" --steps 30 --warmup 5 --set engine.proj_per_layer=1
done
for r in 1 2; do
  one "c3 base r$r" --steps 15 --warmup 3 --batch 256 --precision bf16
  one "c3 proj_per_layer r$r" --steps 15 --warmup 3 --batch 256 --precision bf16 --set engine.proj_per_layer=1
done
echo done
