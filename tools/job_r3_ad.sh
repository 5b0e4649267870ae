#!/bin/bash
# Issue-order options (tail_main_first, side_issue_late): their bitwise tests, then a same-box A/B at
# C2 and C3.  Usage: tools/job_r3_ad.sh OUT
O=${1:-gpurun_out/r3_ad}
mkdir -p "$O"
timeout -k 10 300 python -u -m pytest tests/test_gpu_x_pending.py -m gpu -x -q -k "third_stream or atom_blocks" --timeout 120 --timeout-method thread -p no:cacheprovider > "$O/tests.log" 2>&1
rc=$?; tail -1 "$O/tests.log"; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" "$O/tests.log" | head -20; exit $rc; }
one() {
  local tag=$1; shift
  timeout -k 10 240 python bench.py --no-cpu-baseline --no-secondary --no-roofline --e2e 0 "$@" > "$O/one.json" 2>&1 || { tail -20 "$O/one.json"; exit 3; }
  echo "$tag: $(grep '^{' "$O/one.json" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")" | tee -a "$O/ab.log"
}
for r in 1 2; do
  one "c2 base r$r" --steps 30 --warmup 5
  one "c2 tail_main_first r$r" --steps 30 --warmup 5 --set engine.tail_main_first=1
  one "c2 side_issue_late r$r" --steps 30 --warmup 5 --set engine.side_issue_late=1
  one "c2 both r$r" --steps 30 --warmup 5 --set engine.tail_main_first=1 --set engine.side_issue_late=1
done
for r in 1 2; do
  one "c3 base r$r" --steps 15 --warmup 3 --batch 256 --precision bf16
  one "c3 both r$r" --steps 15 --warmup 3 --batch 256 --precision bf16 --set engine.tail_main_first=1 --set engine.side_issue_late=1
done
echo done
