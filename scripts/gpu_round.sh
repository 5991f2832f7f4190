#!/bin/bash
# One GPU call covering a round checkpoint: parity tests, smoke, default bench (C2 + CPU baseline),
# rocprofv3 kernel-trace stats for every config, and PMC traffic passes for C2.
# Every GPU step has its own time limit; the first failure ends the script.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
step() { echo "[$(date +%T)] $*"; }
if [ -z "$SKIP_TESTS" ]; then
  step pytest
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
  tail -3 gpurun_out/pytest_gpu.log
  step smoke
  timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -30 gpurun_out/smoke.log; exit 1; }
  cat gpurun_out/smoke.log
fi
step bench
timeout -k 10 300 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { echo "bench failed"; tail -30 gpurun_out/bench.err; exit 1; }
cat gpurun_out/bench.json
for c in ${CONFIGS:-2 1 3 4 5}; do
  step "rocprof config $c"
  st=20; [ "$c" != 2 ] && st=${STEPS:-3}
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c$c -o c$c --output-format csv -- python3 -u bench.py --config $c --steps $st --warmup ${CWARM:-2} --no-cpu-baseline > gpurun_out/bench_c$c.json 2> gpurun_out/bench_c$c.err || { echo "config $c failed"; tail -20 gpurun_out/bench_c$c.err; exit 1; }
  grep '"metric"' gpurun_out/bench_c$c.json | cut -c1-300
done
if [ -z "$NO_PMC" ]; then
  for c in ${PMC_CONFIGS:-2}; do
    st=10; [ "$c" != 2 ] && st=2
    step "pmc fetch c$c"
    timeout -s KILL 150 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_c$c -o fetch --output-format csv -- python3 bench.py --config $c --steps $st --warmup 1 --no-cpu-baseline > gpurun_out/pmc_fetch_c$c.log 2>&1 || { echo "pmc fetch failed"; tail -5 gpurun_out/pmc_fetch_c$c.log; exit 1; }
    step "pmc write c$c"
    timeout -s KILL 150 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_c$c -o write --output-format csv -- python3 bench.py --config $c --steps $st --warmup 1 --no-cpu-baseline > gpurun_out/pmc_write_c$c.log 2>&1 || { echo "pmc write failed"; tail -5 gpurun_out/pmc_write_c$c.log; exit 1; }
  done
fi
step done
