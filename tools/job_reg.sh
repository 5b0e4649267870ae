#!/bin/bash
# Register-direct fp32 GEMM A/B (gemm_reg.hip): its tests, the per-product sweep under each forced
# mode, then the C2 step with the automatic rule in each mode (ALIGNN_GEMM_REG_MODE), with and
# without K-contiguous weight copies for the dX products.  usage: bash tools/job_reg.sh OUTDIR
O=${1:?outdir}
mkdir -p "$O"
run() {
  local name=$1 lim=$2; shift 2
  echo "=== $name: $*" | tee -a "$O/run.log"
  timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a "$O/run.log"
  tail -3 "$O/$name.log" | cut -c1-300
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stop after $name (rc=$rc)"; exit $rc; fi
}
Q=(bench.py --no-secondary --no-cpu-baseline --e2e 0 --steps 20 --warmup 5)
run regtest 300 python -u -m pytest -m gpu -v --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gpu_x_gemm_reg.py
for f in 16384 32768 49152; do
  run "sweep_$f" 300 python -u tools/gemm_bench.py --quick --reps 10 --flag $f
done
for m in 0 1 2 3; do
  ALIGNN_GEMM_REG_MODE=$m run "c2_m$m" 300 python "${Q[@]}"
  ALIGNN_GEMM_REG_MODE=$m run "c2_m${m}_wt" 300 python "${Q[@]}" --set engine.wt_copies=1
done
ALIGNN_GEMM_REG_MODE=0 run c2_m0_b 300 python "${Q[@]}"
