set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_x_lg3.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/t_lg3.log 2>&1 || { tail -30 gpurun_out/t_lg3.log; exit 1; }
tail -3 gpurun_out/t_lg3.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/t_all.log 2>&1; rc=$?
tail -3 gpurun_out/t_all.log
[ $rc -le 1 ] || exit $rc
for r in 1 2; do
  for arm in new old nr1; do
    case $arm in
      new) unset ALIGNN_HIP_LIB; extra="";;
      old) unset ALIGNN_HIP_LIB; extra="--set wave_items=0";;
      nr1) export ALIGNN_HIP_LIB=$PWD/gnn-elasticity-predictor_amd/alignn_mi355x/variants/libalignn_hip_nr1.so; extra="";;
    esac
    timeout -k 10 180 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-secondary $extra > gpurun_out/b_$arm.log 2>&1 || { tail -20 gpurun_out/b_$arm.log; exit 3; }
    echo "round $r $arm: $(grep '^{' gpurun_out/b_$arm.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(d['value'], d['ms_per_step'], r['kernel'], r['avg_us'], r['frac'])")" | tee -a gpurun_out/ab.log
  done
done
unset ALIGNN_HIP_LIB
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-secondary > gpurun_out/prof.log 2>&1; echo "rocprof rc $?"
