#!/bin/bash
# pytest -m gpu (optional: TESTS=0 skips), then bench.py for each config in $CONFIGS (default 2).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 ${PYT_TMO:-900} python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
  tail -2 gpurun_out/pytest_gpu.log
fi
for c in ${CONFIGS:-2}; do
  timeout -k 10 300 python -u bench.py --config $c --steps ${STEPS:-20} --warmup 3 ${BENCH_ARGS:---no-cpu-baseline} > gpurun_out/bench_c$c.json 2> gpurun_out/bench_c$c.err || { echo "bench $c failed"; tail -20 gpurun_out/bench_c$c.err; exit 1; }
  python3 -c "
import json;d=json.loads(open('gpurun_out/bench_c$c.json').read().strip().splitlines()[-1])
print('c$c', 'ms/step=%.4f'%d['ms_per_step'], 'rows/s=%.3e'%d['value'], 'kernel_us=%.2f'%(d['roofline']['kernel_avg_ms']*1e3), 'frac=%.3f'%d['roofline']['frac'], {k:round(v*1e3,1) for k,v in d['kernels_ms_per_step'].items()})"
done
