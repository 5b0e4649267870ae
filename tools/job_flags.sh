#!/bin/bash
# Same-box A/B of engine flags against the default: tools/job_flags.sh OUTDIR FLAG...
O=$1; shift
mkdir -p "$O"
ok() { local rc=$1; [ "$rc" -le 1 ] || { echo "stop rc=$rc"; exit "$rc"; }; }
run() {
  timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-secondary --e2e 0 --no-roofline "$@" > "$O/b.log" 2>&1; ok $?
  tail -1 "$O/b.log" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])"
}
for r in 1 2; do
  echo "round $r default: $(run)" | tee -a "$O/ab.log"
  for f in "$@"; do echo "round $r $f: $(run --set $f)" | tee -a "$O/ab.log"; done
done
