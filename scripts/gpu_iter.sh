#!/bin/bash
# Iteration loop on the GPU box: parity tests, then C2 A/B, then the other configs' step time.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
  tail -2 gpurun_out/pytest_gpu.log
fi
CFG=2 bash scripts/gpu_ab.sh ${AB:-base:} || exit 1
for c in ${CONFIGS:-1 3 4 5}; do
  timeout -k 10 300 python -u bench.py --config $c --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline > gpurun_out/it_c$c.json 2> gpurun_out/it_c$c.err || { echo "config $c failed"; tail -20 gpurun_out/it_c$c.err; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/it_c$c.json').read().strip().splitlines()[-1]);print('c$c', round(d['ms_per_step'],3),'ms/step', round(d['roofline']['kernel_avg_ms'],3),'ms insert', round(d['roofline']['frac'],3), {k: round(v,3) for k,v in d['kernels_ms_per_step'].items()})"
done
if [ -n "$PROF" ]; then
  timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_it -o it --output-format csv -- python3 bench.py --config ${PROF_CFG:-2} --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/prof_it.log 2>&1 || { echo "rocprof failed"; tail -20 gpurun_out/prof_it.log; exit 1; }
  cut -d, -f1-4 gpurun_out/prof_it/it_kernel_stats.csv | cut -c1-160
fi
