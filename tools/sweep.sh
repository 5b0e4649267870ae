#!/bin/bash
# A/B sweep of opt-in paths: one short bench per configuration (each arg = space-separated --set items,
# "-" = defaults).  Stops at the first crash/timeout.  Usage: tools/sweep.sh "-" "engine.skinny_encoder=1" ...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
for cfg in "$@"; do
  sets=()
  if [ "$cfg" != "-" ]; then for s in $cfg; do sets+=(--set "$s"); done; fi
  echo "=== $cfg" | tee -a gpurun_out/sweep.log
  timeout -k 10 180 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-secondary ${EXTRA_BENCH_ARGS} "${sets[@]}" > gpurun_out/sweep_one.log 2>&1
  rc=$?
  grep '^{' gpurun_out/sweep_one.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline'] and d['roofline']['kernel'], d['roofline'] and d['roofline']['avg_us'])" | tee -a gpurun_out/sweep.log
  if [ $rc -ne 0 ]; then tail -20 gpurun_out/sweep_one.log | tee -a gpurun_out/sweep.log; echo "rc=$rc"; exit $rc; fi
done
