#!/bin/bash
# Every -m gpu test (one pytest process), then smoke.  Usage: bash tools/job_tests_all.sh OUTDIR
O=${1:-gpurun_out/all}
mkdir -p "$O"
ok() { local rc=$1; [ "$rc" -le 1 ] || { echo "stop rc=$rc"; exit "$rc"; }; }
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > "$O/tests.log" 2>&1; ok $?
grep -E "FAIL|ERROR" "$O/tests.log" | head -20; tail -3 "$O/tests.log"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1; ok $?
tail -2 "$O/smoke.log"
