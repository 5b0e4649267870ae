#!/bin/bash
O=${1:-gpurun_out/r3_e}
mkdir -p "$O"
ok() { local rc=$1; [ "$rc" -le 1 ] || { echo "stop rc=$rc"; exit "$rc"; }; }
bash tools/job_tests_all.sh "$O"; ok $?
timeout -k 10 600 python bench.py --gpus 2 --dist-backend gloo --share-device --steps 5 --warmup 2 --e2e 600 > "$O/bench_2rank_rehearsal.log" 2>&1; ok $?
grep '^{' "$O/bench_2rank_rehearsal.log" | cut -c1-300
