mkdir -p gpurun_out/j7
timeout -k 10 400 python -u -m pytest tests/test_gpu_x_gemm_pipe.py tests/test_gpu_kernels.py tests/test_gpu_x_bf16.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/j7/t.log 2>&1; rc=$?; tail -3 gpurun_out/j7/t.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python tools/gemm_bench.py --quick --reps 10 > gpurun_out/j7/gemm_pipe.log 2>&1; tail -4 gpurun_out/j7/gemm_pipe.log
ALIGNN_HIP_LIB=$PWD/gnn-elasticity-predictor_amd/alignn_mi355x/variants/libalignn_hip_nopipe.so timeout -k 10 300 python tools/gemm_bench.py --quick --reps 10 > gpurun_out/j7/gemm_nopipe.log 2>&1; tail -4 gpurun_out/j7/gemm_nopipe.log
for r in 1 2; do for lib in - $PWD/gnn-elasticity-predictor_amd/alignn_mi355x/variants/libalignn_hip_nopipe.so; do
  if [ "$lib" = "-" ]; then unset ALIGNN_HIP_LIB; else export ALIGNN_HIP_LIB=$lib; fi
  timeout -k 10 180 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-secondary > gpurun_out/j7/b.log 2>&1 || { tail -20 gpurun_out/j7/b.log; exit 3; }
  echo "round $r lib $(basename $lib): $(grep '^{' gpurun_out/j7/b.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(d['value'], d['ms_per_step'], r['kernel'], r['avg_us'], r['frac'])")" | tee -a gpurun_out/j7/ab.log
done; done
