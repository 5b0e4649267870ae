#!/bin/bash
# Round-5 GPU job steps (run through gpurun from the repo root).  Each step under its own time
# limit; the script stops at the first failing step.  The A/B steps expect their comparison build
# where they name it (abl/wt: a git worktree of the base commit with its library built; abl/lib*.so:
# alternative builds of the library) — set up by hand before the call, removed after.
set -eo pipefail
O=$PWD/gpurun_out/${JOB:-r5}
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
    xf) run xf 300 "${PT[@]}" tests/test_gpu_x_recompute.py tests/test_gpu_x_round5.py tests/test_gpu_x_round4.py ;;
    r5t) run r5t 300 "${PT[@]}" tests/test_gpu_x_round5.py ;;
    lgx) run lgx 300 python tools/lgx_bench.py ;;
    c3) run c3 300 python bench.py --steps 10 --warmup 3 --batch 256 --precision bf16 --no-secondary --e2e 0 --no-cpu-baseline ;;
    abx) for i in 1 2; do
           run c2_xf_$i 300 python bench.py --steps 30 --warmup 5 --no-secondary --e2e 0 --no-cpu-baseline
           run c2_rows_$i 300 python bench.py --steps 30 --warmup 5 --no-secondary --e2e 0 --no-cpu-baseline --set engine.recompute_angle=0
         done ;;
    gemmt) run gemmt 400 "${PT[@]}" tests/test_gpu_kernels.py tests/test_gpu_x_gemm_pipe.py tests/test_gpu_x_gemm_lds16.py tests/test_gpu_x_splitk.py tests/test_gpu_parity.py ;;
    abl) for i in 1 2; do
           run c2_new_$i 300 python bench.py --steps 30 --warmup 5 --no-secondary --e2e 0 --no-cpu-baseline
           (cd abl/wt && run c2_base_$i 300 python bench.py --steps 30 --warmup 5 --no-secondary --e2e 0 --no-cpu-baseline)
         done
         run c3_new 300 python bench.py --steps 10 --warmup 3 --batch 256 --precision bf16 --no-secondary --e2e 0 --no-cpu-baseline
         (cd abl/wt && run c3_base 300 python bench.py --steps 10 --warmup 3 --batch 256 --precision bf16 --no-secondary --e2e 0 --no-cpu-baseline) ;;
    gprobe) for t in 0 1 17 2 3 20 129 145; do run gprobe_$t 120 python tools/gemm_probe.py --tile $t; done ;;
    gbf) for sh in "16020 768 256" "15360 1024 256" "16020 256 768" "15360 256 1024"; do set -- $sh
           for t in 0 128 16 129 130 131; do run gbf_$1_$2_$3_$t 120 python tools/gemm_probe.py --bf16 --M $1 --N $2 --K $3 --tile $t; done; done
         for t in 0 512 640 528 641 642; do run gbf_184320_$t 120 python tools/gemm_probe.py --bf16 --M 184320 --tile $t; done
         grep -h '^{' $O/gbf_*.log ;;
    gbs) for sh in "184320 256 256" "16020 768 256" "15360 1024 256" "16020 256 768"; do set -- $sh
           for t in 0 8192; do for io in "" --io16; do
             run gbs_$1_$2_$3_$t$io 120 python tools/gemm_probe.py --bf16 --M $1 --N $2 --K $3 --tile $t $io; done; done; done
         grep -h '^{' $O/gbs_*.log ;;
    grows) run t_rows 300 "${PT[@]}" tests/test_gpu_x_gemm_rows.py
           for sh in "184320 256 256" "184320 256 36" "16020 768 256" "15360 1024 256"; do set -- $sh
             for t in 0 131072 65536; do for io in "" --io16; do
               run grows_$1_$2_$3_$t$io 120 python tools/gemm_probe.py --bf16 --M $1 --N $2 --K $3 --tile $t $io; done; done; done
           grep -h '^{' $O/grows_*.log ;;
    rowsab) run t_rows 300 "${PT[@]}" tests/test_gpu_x_gemm_rows.py
           for io in "" --io16; do run grows_184320$io 120 python tools/gemm_probe.py --bf16 --M 184320 $io; done
           for io in "" --io16; do run grows_16020$io 120 python tools/gemm_probe.py --bf16 --M 16020 --N 768 --tile 65536 $io; done
           grep -h '^{' $O/grows_*.log
           for m in 32768 4096 999999999 32768 4096 999999999; do
             ALIGNN_GEMM_ROWS_MIN_M=$m run c3_m$m 300 python bench.py --steps 10 --warmup 3 --batch 256 --precision bf16 --no-secondary --e2e 0 --no-cpu-baseline; done ;;
    rowsf) run t_rows 300 "${PT[@]}" tests/test_gpu_x_gemm_rows.py
           for t in 0 131072; do run growsf_$t 120 python tools/gemm_probe.py --M 23040 --tile $t; done
           run growsf_2003 120 python tools/gemm_probe.py --M 2003 --N 768 --tile 65536
           run growsf_2003n 120 python tools/gemm_probe.py --M 2003 --N 768 --tile 131072
           grep -h '^{' $O/growsf_*.log
           for m in 4096 999999999 4096 999999999; do
             ALIGNN_GEMM_ROWS_MIN_M_F32=$m run c2_m$m 300 python bench.py --steps 20 --warmup 5 --no-secondary --e2e 0 --no-cpu-baseline; grep -o '"value": [0-9.]*' $O/c2_m$m.log; done ;;
    npf) for L in in-tree abl/libnpf2.so; do tag=$(basename $L .so)
           for sh in "2580 768 256" "1920 1024 256" "23040 256 256" "2580 256 256"; do set -- $sh
             if [ $L = in-tree ]; then run gnpf_${tag}_$1_$2 120 python tools/gemm_probe.py --M $1 --N $2 --K $3 --no-lib
             else ALIGNN_HIP_LIB=$PWD/$L run gnpf_${tag}_$1_$2 120 python tools/gemm_probe.py --M $1 --N $2 --K $3 --no-lib; fi; done; done
         for f in $O/gnpf_*.log; do echo "$(basename $f) $(grep '^{' $f)"; done
         for i in 1 2; do run c2_new$i 300 python bench.py --steps 20 --warmup 5 --no-secondary --e2e 0 --no-cpu-baseline
           ALIGNN_HIP_LIB=$PWD/abl/libnpf2.so run c2_npf2_$i 300 python bench.py --steps 20 --warmup 5 --no-secondary --e2e 0 --no-cpu-baseline; done
         for f in $O/c2_*.log; do echo "$(basename $f) $(grep -o '"value": [0-9.]*' $f)"; done ;;
    gtrace) run gtrace_c3 300 python tools/gemm_trace.py --batch 256 --precision bf16 --time
           run gtrace_c2 300 python tools/gemm_trace.py --batch 32 --precision fp32 --time
           head -30 $O/gtrace_c3.log; head -30 $O/gtrace_c2.log ;;
    wgrad) run t_wgrad 300 "${PT[@]}" tests/test_gpu_x_gemm_wgrad.py tests/test_gpu_x_round5.py -k "wgrad or rowsum"
           run gtrace_c3 300 python tools/gemm_trace.py --batch 256 --precision bf16 --time
           head -16 $O/gtrace_c3.log | cut -c1-200
           for i in 1 2; do run c3_w$i 300 python bench.py --steps 10 --warmup 3 --batch 256 --precision bf16 --no-secondary --e2e 0 --no-cpu-baseline
             ALIGNN_GEMM_WGRAD=0 run c3_nw$i 300 python bench.py --steps 10 --warmup 3 --batch 256 --precision bf16 --no-secondary --e2e 0 --no-cpu-baseline; done
           for f in $O/c3_*.log; do echo "$(basename $f) $(grep -o '"value": [0-9.]*' $f)"; done ;;
    wgradab) for i in 1 2; do for w in 256 128 64 off; do
             if [ $w = off ]; then ALIGNN_GEMM_WGRAD=0 run c3_w${w}_$i 300 python bench.py --steps 10 --warmup 3 --batch 256 --precision bf16 --no-secondary --e2e 0 --no-cpu-baseline
             else ALIGNN_WGRAD_WGS=$w run c3_w${w}_$i 300 python bench.py --steps 10 --warmup 3 --batch 256 --precision bf16 --no-secondary --e2e 0 --no-cpu-baseline; fi; done; done
           for f in $O/c3_*.log; do echo "$(basename $f) $(grep -o '"value": [0-9.]*' $f)"; done ;;
    sw) run t_sw 400 "${PT[@]}" tests/test_gpu_x_lg3.py tests/test_gpu_x_recompute.py tests/test_gpu_parity.py
        run lgx_sw 300 python tools/lgx_bench.py --batch 32
        ALIGNN_LG3_SW=1 run lgx_sw1 300 python tools/lgx_bench.py --batch 32
        grep -h '^{' $O/lgx_sw.log $O/lgx_sw1.log | cut -c1-400
        for i in 1 2; do for w in 4 2 1; do
          ALIGNN_LG3_SW=$w run c2_sw${w}_$i 300 python bench.py --steps 20 --warmup 5 --no-secondary --e2e 0 --no-cpu-baseline; done; done
        for f in $O/c2_*.log; do echo "$(basename $f) $(grep -o '"value": [0-9.]*' $f)"; done ;;
    batched) run t_batched 400 "${PT[@]}" tests/test_gpu_x_gemm_rows.py tests/test_gpu_x_gemm_wgrad.py tests/test_gpu_x_round5.py
           run gtrace_c3 300 python tools/gemm_trace.py --batch 256 --precision bf16 --time
           head -3 $O/gtrace_c3.log | cut -c1-120
           for i in 1 2; do run c3_new$i 300 python bench.py --steps 10 --warmup 3 --batch 256 --precision bf16 --no-secondary --e2e 0 --no-cpu-baseline
             ALIGNN_HIP_LIB=$PWD/abl/libprev.so run c3_prev$i 300 python bench.py --steps 10 --warmup 3 --batch 256 --precision bf16 --no-secondary --e2e 0 --no-cpu-baseline; done
           for f in $O/c3_*.log; do echo "$(basename $f) $(grep -o '"value": [0-9.]*' $f)"; done ;;
    batched2) run t_b2 400 "${PT[@]}" tests/test_gpu_x_gemm_rows.py tests/test_gpu_x_gemm_wgrad.py
           for i in 1 2; do run c3_new$i 300 python bench.py --steps 10 --warmup 3 --batch 256 --precision bf16 --no-secondary --e2e 0 --no-cpu-baseline
             ALIGNN_HIP_LIB=$PWD/abl/libprev.so run c3_prev$i 300 python bench.py --steps 10 --warmup 3 --batch 256 --precision bf16 --no-secondary --e2e 0 --no-cpu-baseline; done
           for f in $O/c3_*.log; do echo "$(basename $f) $(grep -o '"value": [0-9.]*' $f)"; done
           run bench 600 python bench.py
           tail -1 $O/bench.log ;;
    evid) cd /tmp && export TMPDIR=/tmp
          B3="--steps 3 --warmup 2 --batch 256 --precision bf16 --no-secondary --e2e 0 --no-cpu-baseline"
          B2="--steps 5 --warmup 2 --no-secondary --e2e 0 --no-cpu-baseline"
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
    heads) run t_heads 400 "${PT[@]}" tests/test_gpu_x_gemm_rows.py tests/test_gpu_x_pending.py tests/test_gpu_x_round5.py
           run gtrace_c3 300 python tools/gemm_trace.py --batch 256 --precision bf16 --time
           head -1 $O/gtrace_c3.log; grep -E "B\(4, 256, 64\)" $O/gtrace_c3.log | head -4 | cut -c1-110
           for i in 1 2; do run c3_new$i 300 python bench.py --steps 10 --warmup 3 --batch 256 --precision bf16 --no-secondary --e2e 0 --no-cpu-baseline
             ALIGNN_HIP_LIB=$PWD/abl/libprev.so run c3_prev$i 300 python bench.py --steps 10 --warmup 3 --batch 256 --precision bf16 --no-secondary --e2e 0 --no-cpu-baseline; done
           for f in $O/c3_*.log; do echo "$(basename $f) $(grep -o '"value": [0-9.]*' $f)"; done ;;
    gpmc) cd /tmp && export TMPDIR=/tmp
          timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU --kernel-trace -d $O/gpmc_sq -o run --output-format csv -- python $OLDPWD/tools/gemm_probe.py --iters 10 --no-lib > $O/gpmc_sq.log 2>&1 || exit 1
          timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --kernel-trace -d $O/gpmc_mf -o run --output-format csv -- python $OLDPWD/tools/gemm_probe.py --iters 10 --no-lib > $O/gpmc_mf.log 2>&1 || exit 1
          cd $OLDPWD; python tools/pmc_sq.py $O/gpmc_sq > $O/gpmc_sq.txt; python tools/pmc_mfma.py $O/gpmc_mf > $O/gpmc_mf.txt; cat $O/gpmc_sq.txt $O/gpmc_mf.txt ;;
    rpc2) cd /tmp && export TMPDIR=/tmp
          timeout -s KILL 400 rocprofv3 --kernel-trace --stats -d $O/rp_c2 -o run --output-format csv -- python $OLDPWD/bench.py --steps 20 --warmup 5 --no-secondary --e2e 0 --no-cpu-baseline > $O/rp_c2.log 2>&1 || exit 1
          cd $OLDPWD; python tools/timeline.py $O/rp_c2/run_kernel_trace.csv --top 25 > $O/rp_c2_timeline.txt; python tools/trace_by_grid.py $O/rp_c2/run_kernel_trace.csv > $O/rp_c2_by_grid.txt 2>&1; head -40 $O/rp_c2_timeline.txt ;;
    rpc3) cd /tmp && export TMPDIR=/tmp
          timeout -s KILL 400 rocprofv3 --kernel-trace --stats -d $O/rp_c3 -o run --output-format csv -- python $OLDPWD/bench.py --steps 10 --warmup 3 --batch 256 --precision bf16 --no-secondary --e2e 0 --no-cpu-baseline > $O/rp_c3.log 2>&1 || exit 1
          cd $OLDPWD; python tools/timeline.py $O/rp_c3/run_kernel_trace.csv --top 25 > $O/rp_c3_timeline.txt; python tools/trace_by_grid.py $O/rp_c3/run_kernel_trace.csv > $O/rp_c3_by_grid.txt 2>&1; head -20 $O/rp_c3_timeline.txt ;;
    esweep) B2="--steps 30 --warmup 5 --no-secondary --e2e 0 --no-cpu-baseline $EXTRA"
            for i in 1 2; do for v in base ${VARIANTS:-engine.enc_bwd_aux=1 engine.wgrad_early=1}; do
              if [ $v = base ]; then run c2_${v}_$i 300 python bench.py $B2
              else run c2_${v}_$i 300 python bench.py $B2 --set ${v//+/ --set }; fi; done; done
            for f in $O/c2_*.log; do echo "$(basename $f) $(grep -o '"value": [0-9.]*' $f)"; done ;;
    esweep3) B3="--steps 10 --warmup 3 --batch 256 --precision bf16 --no-secondary --e2e 0 --no-cpu-baseline"
            for i in 1 2; do for v in base ${VARIANTS:-engine.wgrad_early=2 engine.wgrad_early=0}; do
              if [ $v = base ]; then run c3_${v}_$i 300 python bench.py $B3
              else run c3_${v}_$i 300 python bench.py $B3 --set ${v//+/ --set }; fi; done; done
            for f in $O/c3_*.log; do echo "$(basename $f) $(grep -o '"value": [0-9.]*' $f)"; done ;;
    libab) B2="--steps 30 --warmup 5 --no-secondary --e2e 0 --no-cpu-baseline $EXTRA"
           for i in 1 2; do run c2_base_$i 300 python bench.py $B2
             for L in $LIBS; do ALIGNN_HIP_LIB=$PWD/abl/lib$L.so run c2_${L}_$i 300 python bench.py $B2; done; done
           for f in $O/c2_*.log; do echo "$(basename $f) $(grep -o '"value": [0-9.]*' $f)"; done ;;
    envab) B2="--steps 30 --warmup 5 --no-secondary --e2e 0 --no-cpu-baseline"
           B3="--steps 10 --warmup 3 --batch 256 --precision bf16 --no-secondary --e2e 0 --no-cpu-baseline"
           for i in 1 2; do run c2_base_$i 300 python bench.py $B2
             for v in $ENVS; do (export $v; run c2_${v}_$i 300 python bench.py $B2); done; done
           if [ -n "$C3" ]; then for i in 1 2; do run c3_base_$i 300 python bench.py $B3
             for v in $ENVS; do (export $v; run c3_${v}_$i 300 python bench.py $B3); done; done; fi
           for f in $O/c[23]_*.log; do echo "$(basename $f) $(grep -o '"value": [0-9.]*' $f)"; done ;;
    libab3) B3="--steps 10 --warmup 3 --batch 256 --precision bf16 --no-secondary --e2e 0 --no-cpu-baseline"
           for i in 1 2; do run c3_base_$i 300 python bench.py $B3
             for L in $LIBS; do ALIGNN_HIP_LIB=$PWD/abl/lib$L.so run c3_${L}_$i 300 python bench.py $B3; done; done
           for f in $O/c3_*.log; do echo "$(basename $f) $(grep -o '"value": [0-9.]*' $f)"; done ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
