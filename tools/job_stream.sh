#!/bin/bash
O=${1:-gpurun_out/st}
mkdir -p "$O"
ok() { local rc=$1; [ "$rc" -le 1 ] || { echo "stop rc=$rc"; exit "$rc"; }; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_x_bf16_stream.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > "$O/t.log" 2>&1; rc=$?; tail -3 "$O/t.log"; ok $rc
[ $rc -eq 0 ] || exit 1
timeout -k 10 300 python tools/gemm_bench.py --quick --reps 5 --batch 256 --precision bf16 > "$O/gq.log" 2>&1; ok $?; grep "M184320\|M 15360 N 1024\|M 16020 N  768\|total" "$O/gq.log"
for r in 1 2; do for c in 1 0; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --batch 256 --precision bf16 --no-cpu-baseline --no-secondary --e2e 0 --set bf16_stream=$c > "$O/b.log" 2>&1; ok $?
  echo "round $r bf16_stream=$c: $(tail -1 "$O/b.log" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")" | tee -a "$O/ab.log"
done; done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > "$O/t_all.log" 2>&1; ok $?; tail -1 "$O/t_all.log"
