#!/bin/bash
# Same-box A/B of one bench --set KEY over values: tools/job_ab_set.sh OUTDIR KEY V1 V2 [TESTS...]
O=$1; K=$2; A=$3; B=$4; shift 4
mkdir -p "$O"
ok() { local rc=$1; [ "$rc" -le 1 ] || { echo "stop rc=$rc"; exit "$rc"; }; }
if [ $# -gt 0 ]; then
  timeout -k 10 300 python -u -m pytest "$@" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > "$O/t.log" 2>&1; rc=$?; tail -1 "$O/t.log"; ok $rc
  [ $rc -eq 0 ] || exit 1
fi
for r in 1 2; do for c in $A $B; do
  timeout -k 10 200 python bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-secondary --e2e 0 --set $K=$c > "$O/b.log" 2>&1; ok $?
  echo "round $r $K=$c: $(tail -1 "$O/b.log" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")" | tee -a "$O/ab.log"
done; done
