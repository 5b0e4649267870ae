#!/bin/bash
# HEAD defaults: the stream-option tests, bench quick line, kernel trace of the C2 step (timeline +
# sequence) and of the C3 step.  Usage: tools/job_r3_z.sh OUT
O=${1:-gpurun_out/r3_z}
mkdir -p "$O"
ok() { local rc=$1; [ "$rc" -le 1 ] || { echo "stop rc=$rc"; exit "$rc"; }; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_x_pending.py -m gpu -x -q -k third_stream --timeout 120 --timeout-method thread -p no:cacheprovider > "$O/tests.log" 2>&1
rc=$?; tail -1 "$O/tests.log"; [ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" "$O/tests.log" | head; exit $rc; }
one() {
  local tag=$1; shift
  timeout -k 10 240 python bench.py --no-cpu-baseline --no-secondary --no-roofline --e2e 0 "$@" > "$O/one.json" 2>&1 || { tail -20 "$O/one.json"; exit 3; }
  echo "$tag: $(grep '^{' "$O/one.json" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")" | tee -a "$O/ab.log"
}
for r in 1 2; do
  one "c2 base r$r" --steps 30 --warmup 5
  one "c2 skip_dx_aux r$r" --steps 30 --warmup 5 --set engine.skip_dx_aux=1
done
for r in 1 2; do
  one "c3 base r$r" --steps 15 --warmup 3 --batch 256 --precision bf16
  one "c3 skip_dx_aux r$r" --steps 15 --warmup 3 --batch 256 --precision bf16 --set engine.skip_dx_aux=1
done
timeout -k 10 240 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-secondary --e2e 0 > "$O/bench_c2.json" 2>&1; ok $?
tail -1 "$O/bench_c2.json" | cut -c1-200
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$O/rocprof" -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-secondary --no-roofline --e2e 0 > "$O/rocprof.log" 2>&1; ok $?
f=$(find "$O/rocprof" -name "run_kernel_trace.csv" | head -1)
python tools/timeline.py "$f" --by-kernel --sequence > "$O/timeline_c2.txt" 2>&1
s=$(find "$O/rocprof" -name "run_kernel_stats.csv" | head -1); cp "$s" "$O/c2_kernel_stats.csv"
rm -rf "$O/rocprof"
timeout -k 10 400 rocprofv3 --kernel-trace -d "$O/rocprof3" -o run --output-format csv -- python bench.py --steps 6 --warmup 2 --batch 256 --precision bf16 --no-cpu-baseline --no-secondary --no-roofline --e2e 0 > "$O/rocprof3.log" 2>&1; ok $?
f=$(find "$O/rocprof3" -name "run_kernel_trace.csv" | head -1)
python tools/timeline.py "$f" --by-kernel --sequence > "$O/timeline_c3.txt" 2>&1
rm -rf "$O/rocprof3"
echo done
