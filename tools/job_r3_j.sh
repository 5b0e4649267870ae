#!/bin/bash
# (1) A/B of the step stream at high priority (e2e: the loader's kernels fill in behind the step's),
# (2) per-launch HBM traffic of config C3's dominant bf16 product (FETCH / WRITE passes, own runs).
# Usage: bash tools/job_r3_j.sh OUTDIR
O=${1:-gpurun_out/r3_j}
mkdir -p "$O"
ok() { local rc=$1; [ "$rc" -le 1 ] || { echo "stop rc=$rc"; exit "$rc"; }; }
for r in 1 2; do
  timeout -k 10 300 python bench.py --no-secondary --no-cpu-baseline > "$O/ab_default_$r.json" 2> "$O/ab_default_$r.err"; ok $?
  timeout -k 10 300 python bench.py --no-secondary --no-cpu-baseline --set main_priority=-1 > "$O/ab_mainprio_$r.json" 2> "$O/ab_mainprio_$r.err"; ok $?
done
for f in "$O"/ab_*.json; do python -c "
import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1])
print('$f', d['value'], d['e2e']['value'], d['e2e_variable']['value'])"; done
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$O/pmc_fetch" -o run --output-format csv -- python tools/gemm_one.py --bf16 > "$O/pmc_fetch.log" 2>&1; ok $?
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$O/pmc_write" -o run --output-format csv -- python tools/gemm_one.py --bf16 > "$O/pmc_write.log" 2>&1; ok $?
python tools/pmc_traffic.py "$O/pmc_fetch" "$O/pmc_write" --json "$O/pmc_traffic.json" > "$O/pmc_traffic.txt" 2>&1
head -5 "$O/pmc_traffic.txt"
echo done
