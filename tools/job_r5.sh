#!/bin/bash
# Round-5 GPU job steps (run through gpurun from the repo root).  Each step under its own time
# limit; the script stops at the first failing step.
set -eo pipefail
O=gpurun_out/${JOB:-r5}
mkdir -p "$O"
export PYTHONUNBUFFERED=1
PT=(python -u -m pytest -x -q --timeout 300 --timeout-method thread)
run() { local name=$1 t=$2; shift 2; echo "[job] $name: $*"; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1 || { echo "[job] $name FAILED rc=$?"; tail -30 "$O/$name.log"; exit 1; }; tail -3 "$O/$name.log"; }
for step in "$@"; do
  case $step in
    r5) run r5 300 "${PT[@]}" tests/test_gpu_x_round5.py -v ;;
    gpu) run gpu 600 "${PT[@]}" tests -m gpu ;;
    bench) run bench 420 python bench.py --steps 20 --warmup 5 ;;
    c2) run c2 300 python bench.py --steps 20 --warmup 5 --no-secondary ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
