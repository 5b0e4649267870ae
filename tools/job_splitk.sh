#!/bin/bash
# split-K in-launch combine: kernel tests, A/B of the step (combine on/off), then every GPU test.
O=${1:-gpurun_out/sk}
mkdir -p "$O"
ok() { local rc=$1; [ "$rc" -le 1 ] || { echo "stop rc=$rc"; exit "$rc"; }; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_x_splitk.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > "$O/t_sk.log" 2>&1; rc=$?; tail -3 "$O/t_sk.log"; ok $rc
[ $rc -eq 0 ] || exit 1
for r in 1 2; do for c in 2 4 0; do
  timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-secondary --e2e 0 --set splitk_combine=$c > "$O/b.log" 2>&1; ok $?
  echo "round $r combine=$c: $(tail -1 "$O/b.log" | cut -c1-200)" | tee -a "$O/ab.log"
done; done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > "$O/t_all.log" 2>&1; ok $?; tail -3 "$O/t_all.log"
