#!/bin/bash
# Same-box A/B of library builds: alternates bench runs between libalignn_hip.so builds (paths as
# arguments; "-" = the in-tree build), ROUNDS times each.  Usage: tools/ab_libs.sh ROUNDS LIB...
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
rounds=$1; shift
for r in $(seq "$rounds"); do
  for lib in "$@"; do
    if [ "$lib" = "-" ]; then unset ALIGNN_HIP_LIB; else export ALIGNN_HIP_LIB="$lib"; fi
    timeout -k 10 180 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-secondary --no-roofline --e2e 0 > gpurun_out/ab_one.log 2>&1
    rc=$?
    v=$(grep '^{' gpurun_out/ab_one.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")
    echo "round $r lib $lib: $v" | tee -a gpurun_out/ab.log
    if [ $rc -ne 0 ]; then tail -20 gpurun_out/ab_one.log; exit $rc; fi
  done
done
