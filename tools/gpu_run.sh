#!/bin/bash
# Runs GPU steps in order; stops at the first step whose exit code signals a crash/timeout
# (anything other than 0 = ok and 1 = ordinary test failure).  Usage: tools/gpu_run.sh STEP...
# STEP is one of: tests tests-all smoke bench bench-quick probes rocprof pmc-fetch pmc-write
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out
for step in "$@"; do
  case "$step" in
    tests) cmd=(timeout -k 10 900 python -u -m pytest tests -m gpu -v -x --timeout 120 --timeout-method thread -p no:cacheprovider) ;;
    tests-core) cmd=(timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread -p no:cacheprovider --ignore-glob=tests/test_gpu_x_*) ;;
    tests-x) cmd=(timeout -k 10 600 python -u -m pytest -m gpu -v --timeout 120 --timeout-method thread -p no:cacheprovider tests/test_gpu_x_*.py) ;;
    tests-enc) cmd=(timeout -k 10 300 python -u -m pytest tests/test_gpu_x_encbwd.py -m gpu -v --timeout 120 --timeout-method thread -p no:cacheprovider) ;;
    tests-all) cmd=(timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider) ;;
    smoke) cmd=(timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()") ;;
    bench) cmd=(timeout -k 10 600 python bench.py --steps 20 --warmup 5) ;;
    bench-quick) cmd=(timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-secondary --e2e 0) ;;
    bench-bf16) cmd=(timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-secondary --precision bf16 --e2e 0) ;;
    bench-b256) cmd=(timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-secondary --batch 256 --precision bf16 --e2e 0) ;;
    bench-e2e) cmd=(timeout -k 10 600 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-secondary --e2e 10000) ;;
    probes) cmd=(timeout -k 10 300 python bench.py --steps 5 --warmup 3 --no-cpu-baseline --no-secondary --dump-probes gpurun_out/probes.json --e2e 0) ;;
    rocprof) cmd=(timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/rocprof -o run --output-format csv -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-secondary --e2e 0) ;;
    pmc-fetch) cmd=(timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d gpurun_out/pmc_fetch -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-secondary --no-roofline --e2e 0) ;;
    pmc-write) cmd=(timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d gpurun_out/pmc_write -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-secondary --no-roofline --e2e 0) ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
  echo "=== $step: ${cmd[*]}" | tee -a gpurun_out/run.log
  "${cmd[@]}" > "gpurun_out/$step.log" 2>&1
  rc=$?
  echo "=== $step rc=$rc" | tee -a gpurun_out/run.log
  tail -5 "gpurun_out/$step.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $step (rc=$rc)"; exit $rc; fi
done
