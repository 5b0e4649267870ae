#!/bin/bash
# Round-4 GPU job: named steps in order, each under its own time limit; stops at the first step that
# crashed or timed out (exit codes other than 0 = ok and 1 = test failures).
#   usage: bash tools/job_r4.sh OUTDIR STEP...
#   STEP: new | lgm | tests | smoke | bench | quick | c3 | probes | rocprof-c2 | rocprof-c3 | pmc-c2 | pmc-c3
O=${1:?outdir}; shift
mkdir -p "$O"
PT=(python -u -m pytest -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider)
Q=(bench.py --no-secondary --no-cpu-baseline --e2e 0)
C3=(bench.py --no-secondary --no-cpu-baseline --e2e 0 --batch 256 --precision bf16)
run() {
  local name=$1 lim=$2; shift 2
  echo "=== $name: $*" | tee -a "$O/run.log"
  timeout -k 10 "$lim" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a "$O/run.log"
  tail -4 "$O/$name.log" | cut -c1-400
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stop after $name (rc=$rc)"; exit $rc; fi
}
pmc() {   # pmc NAME COUNTERS BENCHARGS...
  local name=$1 ctr=$2; shift 2
  echo "=== $name" | tee -a "$O/run.log"
  timeout -s KILL 300 rocprofv3 --pmc $ctr --kernel-trace -d "$O/$name" -o run --output-format csv -- python "$@" \
    --steps 3 --warmup 1 --no-roofline > "$O/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a "$O/run.log"
  [ $rc -eq 0 ] || { tail -5 "$O/$name.log"; exit $rc; }
}
for st in "$@"; do
  case "$st" in
    new) run new 600 "${PT[@]}" tests/test_gpu_x_round4.py tests/test_gpu_x_bf16_io.py tests/test_gpu_x_lgmma.py tests/test_gpu_x_bf16_stream.py ;;
    sched) run sched 600 "${PT[@]}" tests/test_gpu_x_round4.py tests/test_gpu_x_store.py tests/test_gpu_x_capacity.py tests/test_gpu_x_configs.py ;;
    lgm) run lgm 300 python tools/lgm_bench.py --reps 20 ;;
    lgmv) for v in gnn-elasticity-predictor_amd/alignn_mi355x/variants/*.so; do
            ALIGNN_HIP_LIB=$v run "lgm_$(basename $v .so)" 300 python tools/lgm_bench.py --reps 20
          done ;;
    lgmt) run lgmt 300 "${PT[@]}" tests/test_gpu_x_lgmma.py tests/test_gpu_x_bf16_io.py ;;
    tests) run tests 1000 "${PT[@]}" tests ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) run bench 600 python bench.py ;;
    quick) run quick 300 python "${Q[@]}" --steps 20 --warmup 5 --dump-probes "$O/probes_c2.json" ;;
    c3) run c3 300 python "${C3[@]}" --steps 10 --warmup 3 --dump-probes "$O/probes_c3.json" ;;
    hostprof) run hostprof 300 python -u tools/host_prep_profile.py --graphs 2000 --steps 30 ;;
    gemmbf) run gemmbf 300 python -u tools/gemm_bench.py --quick --reps 10 --flag 64 ;;
    ab) for i in 1 2; do
          run "ab_r3_$i" 300 bash -c "cd _r3ab && python bench.py --no-secondary --no-cpu-baseline --e2e 0 --steps 20 --warmup 5"
          run "ab_r4_$i" 300 python "${Q[@]}" --steps 20 --warmup 5
        done ;;
    ab3) run ab3_r3 300 bash -c "cd _r3ab && python bench.py --no-secondary --no-cpu-baseline --e2e 0 --batch 256 --precision bf16 --steps 10 --warmup 3"
         run ab3_r4 300 python "${C3[@]}" --steps 10 --warmup 3 ;;
    tcb) run tcb 300 python -u tools/tconv_bench.py --batch 256 --reps 10 ;;
    rpab) run rpab_r3 400 rocprofv3 --kernel-trace --stats -d "$O/rp_ab_r3" -o run --output-format csv -- \
            python _r3ab/bench.py --no-secondary --no-cpu-baseline --e2e 0 --steps 10 --warmup 3 --no-roofline
          run rpab_r4 400 rocprofv3 --kernel-trace --stats -d "$O/rp_ab_r4" -o run --output-format csv -- \
            python "${Q[@]}" --steps 10 --warmup 3 --no-roofline ;;
    rpe2e) run rpe2e 400 rocprofv3 --kernel-trace --stats -d "$O/rp_e2e" -o run --output-format csv -- \
             python bench.py --no-secondary --no-cpu-baseline --e2e 2000 --steps 10 --warmup 3 --no-roofline ;;
    e2eab) run e2eab_r3 400 python _r3ab/bench.py --no-secondary --no-cpu-baseline --e2e 2000 --steps 20 --warmup 5 --no-roofline
           run e2eab_r4 400 python bench.py --no-secondary --no-cpu-baseline --e2e 2000 --steps 20 --warmup 5 --no-roofline ;;
    e2ep) P=(--set stream_priority=-1 --set main_priority=-1 --set loader_priority=0)
          E=(bench.py --no-secondary --no-cpu-baseline --e2e 2000 --no-roofline)
          run e2ep_b32_base 400 python "${E[@]}" --steps 20 --warmup 5
          run e2ep_b32_prio 400 python "${E[@]}" --steps 20 --warmup 5 "${P[@]}"
          run e2ep_b32_prio_pf2 400 python "${E[@]}" --steps 20 --warmup 5 "${P[@]}" --set prefetch=2
          run e2ep_c5_base 400 python "${E[@]}" --batch 256 --precision bf16 --steps 10 --warmup 3
          run e2ep_c5_prio_pf2 400 python "${E[@]}" --batch 256 --precision bf16 --steps 10 --warmup 3 "${P[@]}" --set prefetch=2 ;;
    pre) run pre_off 300 python "${Q[@]}" --steps 20 --warmup 5 --set engine.preamble_aux=0
         run pre_on 300 python "${Q[@]}" --steps 20 --warmup 5
         run pre_off3 300 python "${C3[@]}" --steps 10 --warmup 3 --set engine.preamble_aux=0
         run pre_on3 300 python "${C3[@]}" --steps 10 --warmup 3 ;;
    ptest) run ptest 600 "${PT[@]}" tests/test_gpu_x_pending.py tests/test_gpu_x_round4.py -k "neutral or aux or validator or capture" ;;
    gsweep) run gsweep 600 python -u tools/gemm_bench.py --reps 8 --json "$O/gemm_sweep_c2.json" ;;
    rpvar) run rpvar 500 rocprofv3 --kernel-trace --stats -d "$O/rp_var" -o run --output-format csv -- \
             python bench.py --no-secondary --no-cpu-baseline --e2e 2000 --steps 10 --warmup 3 --no-roofline \
             --set stream_priority=-1 --set main_priority=-1 --set loader_priority=0 ;;
    lp) run lp_m1 500 python bench.py --no-cpu-baseline --set loader_priority=-1
        run lp_def 500 python bench.py --no-cpu-baseline ;;
    lp2) run lp2_a 500 python bench.py --no-cpu-baseline
         run lp2_b 500 python bench.py --no-cpu-baseline --set prefetch=2 ;;
    hwq) run hwq4 500 python bench.py --no-cpu-baseline
         GPU_MAX_HW_QUEUES=8 run hwq8 500 python bench.py --no-cpu-baseline
         GPU_MAX_HW_QUEUES=8 run hwq8b 500 python bench.py --no-cpu-baseline ;;
    src) run src_off 300 python "${C3[@]}" --steps 10 --warmup 3 --set engine.bf16_src=0
         run src_on 300 python "${C3[@]}" --steps 10 --warmup 3
         run src_off2 300 python "${C3[@]}" --steps 10 --warmup 3 --set engine.bf16_src=0
         run src_on2 300 python "${C3[@]}" --steps 10 --warmup 3 ;;
    smm) ALIGNN_GEMM_STREAM_MIN_M=4096 run smm_4k 300 python "${C3[@]}" --steps 10 --warmup 3
         run smm_32k 300 python "${C3[@]}" --steps 10 --warmup 3
         ALIGNN_GEMM_STREAM_MIN_M=4096 run smm_4k2 300 python "${C3[@]}" --steps 10 --warmup 3
         run smm_32k2 300 python "${C3[@]}" --steps 10 --warmup 3 ;;
    lgx) run lgx_tests 300 "${PT[@]}" tests/test_gpu_x_lg3.py tests/test_gpu_x_bf16.py
         ALIGNN_HIP_LIB=$PWD/gnn-elasticity-predictor_amd/alignn_mi355x/variants/base.so run lgx_lgm_base 300 python tools/lgm_bench.py --reps 20
         run lgx_lgm_new 300 python tools/lgm_bench.py --reps 20
         ALIGNN_HIP_LIB=$PWD/gnn-elasticity-predictor_amd/alignn_mi355x/variants/base.so run lgx_c2_base 300 python "${Q[@]}" --steps 20 --warmup 5
         run lgx_c2_new 300 python "${Q[@]}" --steps 20 --warmup 5
         ALIGNN_HIP_LIB=$PWD/gnn-elasticity-predictor_amd/alignn_mi355x/variants/base.so run lgx_c3_base 300 python "${C3[@]}" --steps 10 --warmup 3
         run lgx_c3_new 300 python "${C3[@]}" --steps 10 --warmup 3 ;;
    lgy) VD=$PWD/gnn-elasticity-predictor_amd/alignn_mi355x/variants
         run lgy_tests 300 "${PT[@]}" tests/test_gpu_x_lg3.py tests/test_gpu_x_bf16.py tests/test_gpu_x_round4.py
         run lgy_lgm_new 300 python tools/lgm_bench.py --reps 20
         ALIGNN_HIP_LIB=$VD/base.so run lgy_lgm_base 300 python tools/lgm_bench.py --reps 20
         for r in 1 2; do
           for v in base nosrc3 s3pf8; do
             ALIGNN_HIP_LIB=$VD/$v.so run lgy_c3_${v}_$r 300 python "${C3[@]}" --steps 10 --warmup 3 --dump-probes "$O/probes_${v}_$r.json"
           done
           run lgy_c3_new_$r 300 python "${C3[@]}" --steps 10 --warmup 3 --dump-probes "$O/probes_new_$r.json"
         done ;;
    lgz) VD=$PWD/gnn-elasticity-predictor_amd/alignn_mi355x/variants
         run lgz_diff 200 python tools/lg_diff.py
         run lgz_tests 300 "${PT[@]}" tests/test_gpu_x_round4.py tests/test_gpu_x_lg3.py tests/test_gpu_parity.py
         for r in 1 2; do
           for v in noxcd_nosrc3 src3pf8; do
             ALIGNN_HIP_LIB=$VD/$v.so run lgz_c3_${v}_$r 300 python "${C3[@]}" --steps 10 --warmup 3 --dump-probes "$O/probes_${v}_$r.json"
           done
           run lgz_c3_new_$r 300 python "${C3[@]}" --steps 10 --warmup 3 --dump-probes "$O/probes_new_$r.json"
           ALIGNN_HIP_LIB=$VD/noxcd_nosrc3.so run lgz_c2_noxcd_$r 300 python "${Q[@]}" --steps 20 --warmup 5
           run lgz_c2_new_$r 300 python "${Q[@]}" --steps 20 --warmup 5
         done ;;
    e2ed) run e2ed_tests 300 "${PT[@]}" tests/test_gpu_x_bf16.py tests/test_gpu_x_configs.py tests/test_gpu_x_round4.py
          run e2ed_on 400 python bench.py --no-cpu-baseline
          run e2ed_off 400 python bench.py --no-cpu-baseline --set loader_dedicated=0
          run e2ed_on2 400 python bench.py --no-cpu-baseline ;;
    sdx) run sdx_tests 300 "${PT[@]}" tests/test_gpu_x_pending.py tests/test_gpu_x_round4.py
         for r in 1 2; do
           run sdx_c2_0_$r 300 python "${Q[@]}" --steps 20 --warmup 5
           run sdx_c2_1_$r 300 python "${Q[@]}" --steps 20 --warmup 5 --set engine.skip_dx=1
           run sdx_c2_2_$r 300 python "${Q[@]}" --steps 20 --warmup 5 --set engine.skip_dx=2
           run sdx_c3_0_$r 300 python "${C3[@]}" --steps 10 --warmup 3
           run sdx_c3_2_$r 300 python "${C3[@]}" --steps 10 --warmup 3 --set engine.skip_dx=2
         done ;;
    bst) run bst 300 "${PT[@]}" tests/test_gpu_x_bf16_stream.py ;;
    gbst) run gbst 600 python -u tools/gemm_bench.py --quick --reps 5 --batch 256 --precision bf16 --flag 512 ;;
    c3m) run c3m 300 python "${C3[@]}" --steps 10 --warmup 3 --set engine.attn_mfma=1 --dump-probes "$O/probes_c3m.json" ;;
    rocprof-c2) run rocprof-c2 400 rocprofv3 --kernel-trace --stats -d "$O/rp_c2" -o run --output-format csv -- \
                  python "${Q[@]}" --steps 10 --warmup 3 --no-roofline ;;
    rocprof-c3) run rocprof-c3 400 rocprofv3 --kernel-trace --stats -d "$O/rp_c3" -o run --output-format csv -- \
                  python "${C3[@]}" --steps 5 --warmup 2 --no-roofline ;;
    pmc-c2) pmc pmc_c2_fetch FETCH_SIZE "${Q[@]}"; pmc pmc_c2_write WRITE_SIZE "${Q[@]}"
            pmc pmc_c2_mfma "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" "${Q[@]}" ;;
    pmc-c3) pmc pmc_c3_fetch FETCH_SIZE "${C3[@]}"; pmc pmc_c3_write WRITE_SIZE "${C3[@]}"
            pmc pmc_c3_mfma "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" "${C3[@]}" ;;
    *) echo "unknown step $st"; exit 2 ;;
  esac
done
echo done
