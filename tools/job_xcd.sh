#!/bin/bash
O=${1:-gpurun_out/xcd}
mkdir -p "$O"
ok() { local rc=$1; [ "$rc" -le 1 ] || { echo "stop rc=$rc"; exit "$rc"; }; }
for r in 1 2; do for c in 1 0; do
  timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-secondary --e2e 0 --set xcd_items=$c > "$O/b.log" 2>&1; ok $?
  echo "round $r xcd_items=$c: $(tail -1 "$O/b.log" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")" | tee -a "$O/ab.log"
done; done
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-secondary --e2e 0 --set xcd_items=1 --dump-probes "$O/probes_xcd.json" > "$O/bp.log" 2>&1; ok $?
timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$O/fetch" -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-secondary --no-roofline --e2e 0 --set xcd_items=1 > "$O/fetch.log" 2>&1; ok $?
echo done
