#!/bin/bash
# Round-3 GPU call: new parity tests first (fast fail), the whole -m gpu suite, smoke, the default
# bench (headline C2 + every other config), then PMC traffic passes per config (pmc_run.py between
# markers).  Each GPU step has its own limit; the first failure ends the script.
#   TESTS="tests/x.py ..."  only these test files (skips the full suite)
#   NO_BENCH=1 / NO_PMC=1 / PMC_CONFIGS="2 4 5"
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
step() { echo "[$(date +%T)] $*"; }
if [ -n "$TESTS" ]; then
  step "pytest $TESTS"
  timeout -k 10 900 python -u -m pytest $TESTS -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_sel.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_sel.log; exit 1; }
  tail -3 gpurun_out/pytest_sel.log
elif [ -z "$SKIP_TESTS" ]; then
  step pytest
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
  tail -3 gpurun_out/pytest_gpu.log
  step smoke
  timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -30 gpurun_out/smoke.log; exit 1; }
  cat gpurun_out/smoke.log
fi
if [ -z "$NO_BENCH" ]; then
  step bench
  timeout -k 10 600 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed"; tail -30 gpurun_out/bench.err; exit 1; }
  cut -c1-600 gpurun_out/bench.json
fi
if [ -z "$NO_PMC" ]; then
  for c in ${PMC_CONFIGS:-2 1 3 4 5}; do
    st=3; [ "$c" = 2 ] && st=10
    step "pmc fetch c$c"
    timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_c$c -o fetch --output-format csv -- python3 scripts/pmc_run.py --config $c --steps $st > gpurun_out/pmc_fetch_c$c.log 2>&1 || { echo "pmc fetch failed"; tail -5 gpurun_out/pmc_fetch_c$c.log; exit 1; }
    step "pmc write c$c"
    timeout -s KILL 180 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_c$c -o write --output-format csv -- python3 scripts/pmc_run.py --config $c --steps $st > gpurun_out/pmc_write_c$c.log 2>&1 || { echo "pmc write failed"; tail -5 gpurun_out/pmc_write_c$c.log; exit 1; }
  done
fi
if [ -n "$KTRACE" ]; then
  for c in $KTRACE; do
    step "kernel trace c$c"
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c$c -o c$c --output-format csv -- python3 -u bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --extra-configs none > gpurun_out/bench_c$c.json 2> gpurun_out/bench_c$c.err || { echo "config $c failed"; tail -20 gpurun_out/bench_c$c.err; exit 1; }
  done
fi
step done
