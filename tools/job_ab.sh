#!/bin/bash
# Same-box A/B with per-kernel times: for each library (path, or "-" = in-tree build) one rocprofv3
# kernel-trace pass (its kernel stats -> gpurun_out/ab_<i>_stats.csv), then ROUNDS alternating
# bench runs.  Usage: tools/job_ab.sh ROUNDS LIB... (extra bench flags in $BENCH_EXTRA)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
rounds=$1; shift
export TMPDIR=/tmp
i=0
for lib in "$@"; do
  if [ "$lib" = "-" ]; then unset ALIGNN_HIP_LIB; else export ALIGNN_HIP_LIB="$lib"; fi
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/abprof_$i -o run --output-format csv -- \
    python bench.py --steps 8 --warmup 2 --no-cpu-baseline --no-secondary --no-roofline $BENCH_EXTRA > gpurun_out/abprof_$i.log 2>&1
  rc=$?; [ $rc -eq 0 ] || { tail -20 gpurun_out/abprof_$i.log; exit $rc; }
  cp gpurun_out/abprof_$i/*/run_kernel_stats.csv gpurun_out/ab_${i}_stats.csv 2>/dev/null || cp gpurun_out/abprof_$i/run_kernel_stats.csv gpurun_out/ab_${i}_stats.csv
  echo "lib $i = $lib" | tee -a gpurun_out/ab.log
  i=$((i+1))
done
for r in $(seq "$rounds"); do
  i=0
  for lib in "$@"; do
    if [ "$lib" = "-" ]; then unset ALIGNN_HIP_LIB; else export ALIGNN_HIP_LIB="$lib"; fi
    timeout -k 10 180 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-secondary $BENCH_EXTRA > gpurun_out/ab_one.log 2>&1
    rc=$?
    v=$(grep '^{' gpurun_out/ab_one.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(d['value'], d['ms_per_step'], r['kernel'], r['avg_us'])")
    echo "round $r lib $i: $v" | tee -a gpurun_out/ab.log
    [ $rc -eq 0 ] || { tail -20 gpurun_out/ab_one.log; exit $rc; }
    i=$((i+1))
  done
done
