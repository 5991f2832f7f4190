#!/bin/bash
# Checkpoint: bench.py per config (no profiler), smoke, then the GPU test suite (or $PYTEST_FILES).
# Every GPU step has its own time limit; the first failure ends the script.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for c in ${CONFIGS-2 1 3 4 5}; do
  timeout -k 10 300 python -u bench.py --config $c --steps ${STEPS:-10} --warmup 3 --no-cpu-baseline > gpurun_out/bench_c$c.json 2> gpurun_out/bench_c$c.err || { echo "bench $c failed"; tail -20 gpurun_out/bench_c$c.err; exit 1; }
  python3 -c "
import json;d=json.loads(open('gpurun_out/bench_c$c.json').read().strip().splitlines()[-1])
print('c$c', 'ms/step=%.4f'%d['ms_per_step'], 'rows/s=%.3e'%d['value'], 'frac=%.3f'%d['roofline']['frac'], {k:round(v*1e3,1) for k,v in d['kernels_ms_per_step'].items()})"
done
if [ "${SMOKE:-1}" = 1 ]; then
  timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -30 gpurun_out/smoke.log; exit 1; }
  tail -1 gpurun_out/smoke.log
fi
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 ${PYT_TMO:-1000} python -u -m pytest ${PYTEST_FILES:-tests} -m gpu --maxfail=${MAXFAIL:-5} -v --timeout 150 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_gpu.log 2>&1
  rc=$?
  grep -E "PASSED|FAILED|ERROR" gpurun_out/pytest_gpu.log | grep -v PASSED | head -20
  tail -3 gpurun_out/pytest_gpu.log
  exit $rc
fi
