#!/bin/bash
# Multi-stream configurations at HEAD: C4 (five B = 256 bf16 members on one GPU, each with its own
# main/side/aux streams, atom blocks on aux) and a 2-rank bucketed-DP rehearsal at B = 256 bf16 on
# one GPU (gloo), both under time limits.  Usage: tools/job_r3_ac.sh OUT
O=${1:-gpurun_out/r3_ac}
mkdir -p "$O"
ok() { local rc=$1; [ "$rc" -le 1 ] || { echo "stop rc=$rc"; exit "$rc"; }; }
timeout -k 10 400 python bench.py --ensemble 5 --batch 256 --precision bf16 --steps 6 --warmup 2 --e2e 0 --no-cpu-baseline > "$O/c4.json" 2> "$O/c4.err"; ok $?
tail -1 "$O/c4.json" | cut -c1-260
timeout -k 10 500 python bench.py --gpus 2 --dist-backend gloo --share-device --batch 256 --precision bf16 --steps 4 --warmup 2 --e2e 0 --no-cpu-baseline --no-secondary > "$O/dp2_b256.log" 2>&1; ok $?
grep '^{' "$O/dp2_b256.log" | cut -c1-260
echo done
