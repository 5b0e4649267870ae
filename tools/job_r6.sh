#!/bin/bash
# Round-6 GPU job steps (run through gpurun from the repo root).  Each step under its own time
# limit; the script stops at the first failing step.
set -eo pipefail
O=$PWD/gpurun_out/${JOB:-r6}
mkdir -p "$O"
export PYTHONUNBUFFERED=1
PT=(python -u -m pytest -x -q --timeout 300 --timeout-method thread)
run() { local name=$1 t=$2; shift 2; echo "[job] $name: $*"; timeout -k 10 "$t" "$@" > "$O/$name.log" 2>&1 || { echo "[job] $name FAILED rc=$?"; tail -30 "$O/$name.log"; exit 1; }; tail -3 "$O/$name.log"; }
val() { for f in "$@"; do echo "$(basename "$f") $(grep -o '"value": [0-9.]*' "$f" | head -1) e2e=$(python -c "import json,sys;d=json.loads([l for l in open('$f') if l.startswith('{')][-1]);e=d.get('e2e') or {};print(e.get('value'),e.get('ms_per_step'),e.get('host_ms_per_step'),e.get('stream_priorities'))" 2>/dev/null)"; done; }
E2E=(python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-secondary --no-roofline --e2e 3000)
for step in "$@"; do
  case $step in
    gpu) run gpu 900 "${PT[@]}" tests -m gpu ;;
    gpuall) run gpuall 1100 python -u -m pytest -q --maxfail 20 --timeout 300 --timeout-method thread tests -m gpu ;;
    bench) run bench 600 python bench.py --steps 20 --warmup 5 ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    c2) run c2 300 python bench.py --steps 20 --warmup 5 --no-secondary --e2e 0 --no-cpu-baseline ;;
    c3) run c3 300 python bench.py --steps 10 --warmup 3 --batch 256 --precision bf16 --no-secondary --e2e 0 --no-cpu-baseline ;;
    e2e) for i in 1 2; do
           run e2e_def_$i 300 "${E2E[@]}"
           run e2e_pool0_$i 300 "${E2E[@]}" --set loader_dedicated=0
           run e2e_poolhi_$i 300 "${E2E[@]}" --set loader_priority=-1
           run e2e_poolhi_pf2_$i 300 "${E2E[@]}" --set loader_priority=-1 --set prefetch=2
           run e2e_allnorm_$i 300 "${E2E[@]}" --set main_priority=0
         done
         val "$O"/e2e_*.log ;;
    lgmx) run lgmx 600 "${PT[@]}" tests/test_gpu_x_lgmx.py tests/test_gpu_x_recompute.py -v ;;
    newt) run newt 900 "${PT[@]}" tests/test_gpu_x_lgmx.py tests/test_gpu_x_recompute.py tests/test_gpu_x_infer.py tests/test_gpu_x_round6.py -v ;;
    lgmxb) ALIGNN_LGM_PERSIST=1 run lgmx_bench_p1 300 python tools/lgx_bench.py --batch 256
           ALIGNN_LGM_PERSIST=0 run lgmx_bench_p0 300 python tools/lgx_bench.py --batch 256
           for f in $O/lgmx_bench_p*.log; do echo "$(basename $f) $(grep -o '"fwd_bf16_x_us": [0-9.]*\|"bwd_bf16_x_us": [0-9.]*\|"enc_bwd_bf16_x_us": [0-9.]*' $f | tr '\n' ' ')"; done ;;
    c3ab) for i in 1 2; do for v in 1 0; do
            ALIGNN_LGM_PERSIST=$v run c3_p${v}_$i 300 python bench.py --steps 10 --warmup 3 --batch 256 --precision bf16 --no-secondary --e2e 0 --no-cpu-baseline; done; done
          for f in $O/c3_p*.log; do echo "$(basename $f) $(grep -o '"value": [0-9.]*' $f | head -1)"; done ;;
    c3rx) for i in 1 2; do for v in 1 0; do
            run c3_rx${v}_$i 300 python bench.py --steps 10 --warmup 3 --batch 256 --precision bf16 --no-secondary --e2e 0 --no-cpu-baseline --set engine.recompute_angle_bf16=$v; done; done
          for f in $O/c3_rx*.log; do echo "$(basename $f) $(grep -o '"value": [0-9.]*' $f | head -1)"; done ;;
    lin) run lin 300 python tools/lgx_bench.py --batch 256 --only linear_smallk_bf16 enc_bwd_bf16_rows enc_bwd_bf16_x fwd_bf16_rows bwd_bf16_rows ;;
    linab) for nt in 0 1; do for wg in 2 4 8; do ALIGNN_SK_NT=$nt ALIGNN_SK_WG=$wg run lin_nt${nt}_wg$wg 300 python tools/lgx_bench.py --batch 256 --only linear_smallk_bf16; done; done
           for f in $O/lin_nt*.log; do echo "$(basename $f) $(grep -o '"linear_smallk_bf16_us": [0-9.]*' $f)"; done ;;
    hwq) for q in 4 8 16; do GPU_MAX_HW_QUEUES=$q run hwq_$q 600 python bench.py --steps 20 --warmup 5 --no-cpu-baseline; done
         val "$O"/hwq_*.log
         for f in $O/hwq_*.log; do python -c "
import json,sys
d=json.loads([l for l in open('$f') if l.startswith('{')][-1]); s=d.get('secondary') or {}
print('$f'.split('/')[-1], d['value'], 'e2e', (d.get('e2e') or {}).get('value'), 'var', (d.get('e2e_variable') or {}).get('value'), 'c3', (s.get('c3_b256_bf16') or {}).get('value'), 'c5', (s.get('c5_e2e_b256_bf16') or {}).get('value'), 'cw', (s.get('corrected_wiring') or {}).get('value'), 'c4p', (s.get('c4_ensemble_predict_b256') or {}).get('plan_graphs_per_s'))"; done ;;
    e2es) for sc in cw c3 c3,c5; do run e2es_$sc 600 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --e2e 3000 --secondaries $sc; done
          val "$O"/e2es_*.log ;;
    e2ep) cd /tmp && export TMPDIR=/tmp
          for sc in none cw; do
            timeout -s KILL 400 rocprofv3 --kernel-trace -d $O/rp_e2e_$sc -o run --output-format csv -- python $OLDPWD/bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-roofline --e2e 3000 --secondaries $sc > $O/rp_e2e_$sc.log 2>&1 || exit 1
          done
          cd $OLDPWD
          for sc in none cw; do for st in 2 5; do python tools/timeline.py $O/rp_e2e_$sc/run_kernel_trace.csv --top 12 --step $st > $O/rp_e2e_${sc}_s$st.txt; python tools/timeline.py $O/rp_e2e_$sc/run_kernel_trace.csv --by-kernel --step $st > $O/rp_e2e_${sc}_s${st}_k.txt; done; head -6 $O/rp_e2e_${sc}_s2.txt; done ;;
    e2ef) for st in "prefetch=1" "prefetch=2" "prefetch=3" "loader_priority=0"; do run "e2ef_$st" 600 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-roofline --e2e 3000 --secondaries cw --set $st; done
          val "$O"/e2ef_*.log ;;
    e2eo) for i in 1 2; do
            run e2eo_last_$i 600 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --e2e 3000
            run e2eo_first_$i 600 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --e2e 3000 --secondaries cw,c1,c3,c5,c4,var,e2e_first
          done
          for f in $O/e2eo_*.log; do python -c "
import json,sys
d=json.loads([l for l in open('$f') if l.startswith('{')][-1]); s=d.get('secondary') or {}
print('$f'.split('/')[-1], d['value'], 'e2e', (d.get('e2e') or {}).get('value'), 'var', (d.get('e2e_variable') or {}).get('value'), 'c3', (s.get('c3_b256_bf16') or {}).get('value'), 'c5', (s.get('c5_e2e_b256_bf16') or {}).get('value'), 'cw', (s.get('corrected_wiring') or {}).get('value'))"; done ;;
    pdump) run pdump 300 python tools/plan_dump.py --batch 32 ;;
    e2er) for rp in ${RPARTS:-none probe stamps stamps,serial probe,stamps,serial}; do run "e2er_$rp" 600 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-secondary --e2e 3000 --secondaries none --roofline-parts $rp; done
          val "$O"/e2er_*.log ;;
    e2ev) for n in 0 500; do ALIGNN_DIAG_EVENTS=$n run "e2ev_$n" 600 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-secondary --e2e 3000 --secondaries none --roofline-parts none; done
          val "$O"/e2ev_*.log ;;
    e2eq) E=(python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-secondary --e2e 3000 --secondaries none --roofline-parts probe)
          ALIGNN_DIAG_PROBE_STEPS=0 run e2eq_stamps_nosteps 600 "${E[@]}"
          ALIGNN_DIAG_PROBE_STAMPS=0 ALIGNN_DIAG_PROBE_SERIAL=1 run e2eq_nostamps_serial 600 "${E[@]}"
          ALIGNN_DIAG_PROBE_STAMPS=1 ALIGNN_DIAG_PROBE_SERIAL=0 run e2eq_stamps_concurrent 600 "${E[@]}"
          ALIGNN_DIAG_PROBE_STAMPS=0 ALIGNN_DIAG_PROBE_SERIAL=0 run e2eq_nostamps_concurrent 600 "${E[@]}"
          val "$O"/e2eq_*.log ;;
    e2et) run e2et_store_first 600 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-secondary --e2e 3000 --secondaries store_first,e2e_first
          run e2et_default_nosec 600 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-secondary --e2e 3000 --secondaries e2e_first
          run e2et_store_first_full 600 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --e2e 3000 --secondaries store_first,e2e_first,cw,c3,c5,var
          val "$O"/e2et_*.log ;;
    ab) # generic same-box A/B of one engine switch: AB_KEY=engine.x AB_VALS="1 0" AB_CFG="c2|c3"
        for i in 1 2; do for v in $AB_VALS; do
          if [ "$AB_CFG" = c3 ]; then run ab_${v}_$i 300 python bench.py --steps 10 --warmup 3 --batch 256 --precision bf16 --no-secondary --e2e 0 --no-cpu-baseline --set $AB_KEY=$v
          else run ab_${v}_$i 300 python bench.py --steps 20 --warmup 5 --no-secondary --e2e 0 --no-cpu-baseline --set $AB_KEY=$v; fi
        done; done
        for f in $O/ab_*.log; do echo "$(basename $f) $(grep -o '"value": [0-9.]*' $f | head -1)"; done ;;
    lgxab) for i in 1 2; do for lib in $ABL_LIBS; do
             if [ "$lib" = "-" ]; then unset ALIGNN_HIP_LIB; t=tree; else export ALIGNN_HIP_LIB=$PWD/$lib; t=$(basename ${lib%.so}); fi
             run lgxab_${t}_$i 300 python tools/lgx_bench.py --batch 32 --only fwd_f32_x bwd_f32_x
             run lgxab3_${t}_$i 300 python tools/lgx_bench.py --batch 256 --only fwd_bf16_rows bwd_bf16_rows
           done; done; unset ALIGNN_HIP_LIB
           for f in $O/lgxab*.log; do echo "$(basename $f) $(grep -o '"fwd_[a-z0-9_]*_us": [0-9.]*\|"bwd_[a-z0-9_]*_us": [0-9.]*' $f | tr '\n' ' ')"; done ;;
    e2ec) B=(python bench.py --steps 20 --warmup 5)   # the default line, twice (e2e after the C1 forward)
          run e2ec_default_1 600 "${B[@]}"
          run e2ec_default_2 600 "${B[@]}"
          val "$O"/e2ec_*.log ;;
    ti) run ti 600 "${PT[@]}" tests/test_gpu_x_infer.py -v ;;
    tl) run tl 900 "${PT[@]}" tests/test_gpu_x_lg3.py tests/test_gpu_x_recompute.py tests/test_gpu_parity.py tests/test_gpu_x_configs.py ;;
    tg) run tg 900 "${PT[@]}" tests/test_gpu_x_gemm_pipe.py tests/test_gpu_x_gemm_rows.py tests/test_gpu_x_splitk.py tests/test_gpu_x_gemm_lds16.py tests/test_gpu_x_gemm_wgrad.py tests/test_gpu_kernels.py ;;
    gb3) run gb3 600 python tools/gemm_bench.py --batch 256 --precision bf16 --min-m 15000 --quick --reps 10 ;;
    tc) run tc 900 "${PT[@]}" tests/test_gpu_kernels.py tests/test_gpu_parity.py tests/test_gpu_x_bf16.py tests/test_gpu_x_configs.py tests/test_gpu_x_round4.py tests/test_gpu_x_round5.py ;;
    ablm) # multi-library A/B: ABL_LIBS="ab/libH.so - ab/libF3.so" ("-": the in-tree build); C2 + C3
          # bench values, then one C3 and one C2 kernel trace per library (per-kernel averages)
          for i in $(seq 1 ${ABL_ROUNDS:-2}); do for lib in $ABL_LIBS; do
            if [ "$lib" = "-" ]; then unset ALIGNN_HIP_LIB; t=tree; else export ALIGNN_HIP_LIB=$PWD/$lib; t=$(basename ${lib%.so}); fi
            run ablm_c2_${t}_$i 300 python bench.py --steps 20 --warmup 5 --no-secondary --e2e 0 --no-cpu-baseline
            run ablm_c3_${t}_$i 300 python bench.py --steps 10 --warmup 3 --batch 256 --precision bf16 --no-secondary --e2e 0 --no-cpu-baseline
          done; done
          unset ALIGNN_HIP_LIB
          for f in $O/ablm_c*.log; do echo "$(basename $f) $(grep -o '"value": [0-9.]*' $f | head -1)"; done
          cd /tmp && export TMPDIR=/tmp
          for lib in $ABL_LIBS; do
            if [ "$lib" = "-" ]; then unset ALIGNN_HIP_LIB; t=tree; else export ALIGNN_HIP_LIB=$OLDPWD/$lib; t=$(basename ${lib%.so}); fi
            timeout -s KILL 300 rocprofv3 --kernel-trace -d $O/rpab3_$t -o run --output-format csv -- python $OLDPWD/bench.py --steps 5 --warmup 2 --batch 256 --precision bf16 --no-secondary --e2e 0 --no-cpu-baseline --no-roofline > $O/rpab3_$t.log 2>&1 || exit 1
            timeout -s KILL 300 rocprofv3 --kernel-trace -d $O/rpab2_$t -o run --output-format csv -- python $OLDPWD/bench.py --steps 10 --warmup 2 --no-secondary --e2e 0 --no-cpu-baseline --no-roofline > $O/rpab2_$t.log 2>&1 || exit 1
          done
          unset ALIGNN_HIP_LIB; cd $OLDPWD
          for lib in $ABL_LIBS; do t=tree; [ "$lib" = "-" ] || t=$(basename ${lib%.so})
            for c in 3 2; do python tools/trace_by_grid.py $O/rpab${c}_$t/run_kernel_trace.csv > $O/rpab${c}_$t.txt 2>&1
              echo "C$c $t: $(grep -E "${ABL_PAT:-tconv_(fwd2|bwd_dst2|bwd_src)}" $O/rpab${c}_$t.txt | awk '{n=$0; sub(/.*alignn::/, "", n); printf "%s %s | ", $1, n}')"; done; done ;;
    abl) # library A/B (C2 bench + lgx_bench fp32 kernels): ab/libA.so vs the in-tree build
         for i in 1 2; do for lib in ab/libA.so -; do
           if [ "$lib" = "-" ]; then unset ALIGNN_HIP_LIB; t=B; else export ALIGNN_HIP_LIB=$PWD/$lib; t=A; fi
           run abl_${t}_$i 300 python bench.py --steps 20 --warmup 5 --no-secondary --e2e 0 --no-cpu-baseline ${ABL_ARGS:-}
         done; done
         unset ALIGNN_HIP_LIB
         ALIGNN_HIP_LIB=$PWD/ab/libA.so run abl_lgx_A 300 python tools/lgx_bench.py --batch 32 --only fwd_f32_x bwd_f32_x
         run abl_lgx_B 300 python tools/lgx_bench.py --batch 32 --only fwd_f32_x bwd_f32_x
         for f in $O/abl_*.log; do echo "$(basename $f) $(grep -o '"value": [0-9.]*\|"fwd_f32_x_us": [0-9.]*\|"bwd_f32_x_us": [0-9.]*' $f | head -2 | tr '\n' ' ')"; done ;;
    pmc) cd /tmp && export TMPDIR=/tmp
         B2="--steps 5 --warmup 2 --no-secondary --e2e 0 --no-cpu-baseline"
         B3="--steps 3 --warmup 2 --batch 256 --precision bf16 --no-secondary --e2e 0 --no-cpu-baseline"
         for c in FETCH_SIZE WRITE_SIZE; do
           timeout -s KILL 420 rocprofv3 --pmc $c --kernel-trace -d $O/pmc_c3_$c -o run --output-format csv -- python $OLDPWD/bench.py $B3 > $O/pmc_c3_$c.log 2>&1 || exit 1
           timeout -s KILL 420 rocprofv3 --pmc $c --kernel-trace -d $O/pmc_c2_$c -o run --output-format csv -- python $OLDPWD/bench.py $B2 > $O/pmc_c2_$c.log 2>&1 || exit 1
         done
         timeout -s KILL 420 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d $O/pmc_c3_mf -o run --output-format csv -- python $OLDPWD/bench.py $B3 > $O/pmc_c3_mf.log 2>&1 || exit 1
         timeout -s KILL 420 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d $O/pmc_c2_mf -o run --output-format csv -- python $OLDPWD/bench.py $B2 > $O/pmc_c2_mf.log 2>&1 || exit 1
         cd $OLDPWD
         for c in c2 c3; do
           python tools/pmc_traffic.py $O/pmc_${c}_FETCH_SIZE $O/pmc_${c}_WRITE_SIZE --json $O/pmc_${c}_traffic.json --top 40 > $O/pmc_${c}_traffic.txt
           python tools/pmc_mfma.py $O/pmc_${c}_mf > $O/pmc_${c}_mfma.txt; done
         head -12 $O/pmc_c3_traffic.txt; head -12 $O/pmc_c2_traffic.txt ;;
    e2ed) run e2ed_ns3k 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-secondary --no-roofline --e2e 3000
          run e2ed_ns10k 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-secondary --no-roofline --e2e 10000
          run e2ed_sec3k 600 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --e2e 3000
          val "$O"/e2ed_*.log ;;
    bf16t) run bf16t 900 "${PT[@]}" tests/test_gpu_x_bf16.py tests/test_gpu_x_configs.py tests/test_gpu_x_round5.py tests/test_gpu_x_round4.py tests/test_gpu_x_encbwd.py -v ;;
    rpc2) cd /tmp && export TMPDIR=/tmp
          timeout -s KILL 400 rocprofv3 --kernel-trace --stats -d $O/rp_c2 -o run --output-format csv -- python $OLDPWD/bench.py --steps 20 --warmup 5 --no-secondary --e2e 0 --no-cpu-baseline > $O/rp_c2.log 2>&1 || exit 1
          cd $OLDPWD; python tools/timeline.py $O/rp_c2/run_kernel_trace.csv --top 25 > $O/rp_c2_timeline.txt; python tools/timeline.py $O/rp_c2/run_kernel_trace.csv --by-kernel --step 5 > $O/rp_c2_timeline_bykernel.txt; python tools/trace_by_grid.py $O/rp_c2/run_kernel_trace.csv > $O/rp_c2_by_grid.txt 2>&1; head -20 $O/rp_c2_timeline.txt ;;
    rpc3) cd /tmp && export TMPDIR=/tmp
          timeout -s KILL 400 rocprofv3 --kernel-trace --stats -d $O/rp_c3 -o run --output-format csv -- python $OLDPWD/bench.py --steps 10 --warmup 3 --batch 256 --precision bf16 --no-secondary --e2e 0 --no-cpu-baseline > $O/rp_c3.log 2>&1 || exit 1
          cd $OLDPWD; python tools/timeline.py $O/rp_c3/run_kernel_trace.csv --top 25 > $O/rp_c3_timeline.txt; python tools/timeline.py $O/rp_c3/run_kernel_trace.csv --by-kernel --step 5 > $O/rp_c3_timeline_bykernel.txt; python tools/trace_by_grid.py $O/rp_c3/run_kernel_trace.csv > $O/rp_c3_by_grid.txt 2>&1; head -20 $O/rp_c3_timeline.txt ;;
    pmcx) cd /tmp && export TMPDIR=/tmp
          for c in FETCH_SIZE WRITE_SIZE; do
            timeout -s KILL 300 rocprofv3 --pmc $c --kernel-trace -d $O/pmcx_$c -o run --output-format csv -- python $OLDPWD/tools/lgx_bench.py --batch 256 --reps 3 > $O/pmcx_$c.log 2>&1 || exit 1
          done
          timeout -s KILL 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU --kernel-trace -d $O/pmcx_sq -o run --output-format csv -- python $OLDPWD/tools/lgx_bench.py --batch 256 --reps 3 > $O/pmcx_sq.log 2>&1 || exit 1
          timeout -s KILL 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d $O/pmcx_mf -o run --output-format csv -- python $OLDPWD/tools/lgx_bench.py --batch 256 --reps 3 > $O/pmcx_mf.log 2>&1 || exit 1
          cd $OLDPWD
          python tools/pmc_traffic.py $O/pmcx_FETCH_SIZE $O/pmcx_WRITE_SIZE --top 20 > $O/pmcx_traffic.txt
          python tools/pmc_sq.py $O/pmcx_sq > $O/pmcx_sq.txt; python tools/pmc_mfma.py $O/pmcx_mf > $O/pmcx_mfma.txt
          cat $O/pmcx_traffic.txt $O/pmcx_sq.txt | head -40 ;;
    pmcl) cd /tmp && export TMPDIR=/tmp
          LB=(python $OLDPWD/tools/lgx_bench.py --batch 256 --reps 3 --only fwd_bf16_x bwd_bf16_x fwd_bf16_rows bwd_bf16_rows)
          i=0
          for cs in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU" \
                    "SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD" \
                    "SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES GRBM_GUI_ACTIVE" "FETCH_SIZE" "WRITE_SIZE"; do
            i=$((i+1))
            timeout -s KILL 120 rocprofv3 --pmc $cs --kernel-trace -d $O/pmcl_$i -o run --output-format csv -- "${LB[@]}" > $O/pmcl_$i.log 2>&1 || { echo "pass $i failed"; tail -5 $O/pmcl_$i.log; cd $OLDPWD; exit 1; }
          done
          cd $OLDPWD
          for j in $(seq 1 $i); do python tools/pmc_dump.py $O/pmcl_$j --match lg; done > $O/pmcl.txt; cat $O/pmcl.txt ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
