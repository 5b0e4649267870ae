#!/bin/bash
# After recording the phase-1 join in the plan: repeat the bucketed-DP bitwise test, the stream and
# graph tests, then the wt_copies A/B at C2.  Usage: tools/job_r3_am.sh OUT
O=${1:-gpurun_out/r3_am}
mkdir -p "$O"
timeout -k 10 300 python -u tools/dp_race_probe.py 20 2>&1 | grep -v amdgpu.ids | tee "$O/probe.log" || exit 3
timeout -k 10 400 python -u -m pytest tests/test_gpu_x_pending.py tests/test_gpu_graph.py -m gpu -q -k "third_stream or atom_blocks or graph or side_stream or bucketed" --timeout 120 --timeout-method thread -p no:cacheprovider > "$O/tests.log" 2>&1
rc=$?; tail -1 "$O/tests.log"; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" "$O/tests.log" | head -20; exit $rc; }
one() {
  local tag=$1; shift
  timeout -k 10 240 python bench.py --no-cpu-baseline --no-secondary --no-roofline --e2e 0 "$@" > "$O/one.json" 2>&1 || { tail -20 "$O/one.json"; exit 3; }
  echo "$tag: $(grep '^{' "$O/one.json" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")" | tee -a "$O/ab.log"
}
for r in 1 2; do
  one "c2 base r$r" --steps 30 --warmup 5
  one "c2 wt_copies r$r" --steps 30 --warmup 5 --set engine.wt_copies=1
done
echo done
