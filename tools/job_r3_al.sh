#!/bin/bash
# Intermittent bucketed-DP plan-vs-eager mismatch: repeat the test under option overrides.
O=${1:-gpurun_out/r3_al}
mkdir -p "$O"
for cfg in "" "wgrad_early=0" "skip_early=0 angle_side=0" "gate_reduce_side=0"; do
  timeout -k 10 240 python -u tools/dp_race_probe.py 12 $cfg 2>&1 | grep -v amdgpu.ids | tee -a "$O/probe.log" || exit 3
done
echo done
