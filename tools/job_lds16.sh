#!/bin/bash
# bf16 LDS images for the bf16 tiled GEMM (arithmetic 2) A/B: its bitwise tests, the C3 per-product
# sweep with it forced (--flag 16384), the C3 step with the environment default off / on (twice),
# and the whole GPU suite with it on.  usage: bash tools/job_lds16.sh OUTDIR [all|default]
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
PT=(python -u -m pytest -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider)
C3=(bench.py --no-secondary --no-cpu-baseline --e2e 0 --batch 256 --precision bf16 --steps 10 --warmup 3)
MODE=${2:-all}
if [ "$MODE" = all ]; then   # first pass: forced on everywhere
  run t_lds16 300 "${PT[@]}" tests/test_gpu_x_gemm_lds16.py
  run sweep 300 python -u tools/gemm_bench.py --precision bf16 --batch 256 --quick --reps 5 --flag 16384
  for i in 1 2; do
    ALIGNN_GEMM_LDS16=0 run "c3_off_$i" 300 python "${C3[@]}"
    ALIGNN_GEMM_LDS16=1 run "c3_on_$i" 300 python "${C3[@]}"
  done
  ALIGNN_GEMM_LDS16=1 run suite_on 600 "${PT[@]}" tests
else                         # second pass: the default rule (A k-contiguous) against off
  for i in 1 2; do
    ALIGNN_GEMM_LDS16=0 run "c3_off_$i" 300 python "${C3[@]}"
    run "c3_def_$i" 300 python "${C3[@]}"
  done
  run suite 600 "${PT[@]}" tests
  run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
  run bench 600 python bench.py
fi
