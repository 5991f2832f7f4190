#!/bin/bash
# Round checkpoint as the driver runs it: the whole GPU suite, smoke, the default bench line.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAILED|Error" gpurun_out/pytest_gpu.log | head; tail -5 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/smoke.log; exit 1; }
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python -u bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err || { echo "bench failed"; tail -20 gpurun_out/bench_default.err; exit 1; }
tail -1 gpurun_out/bench_default.json | cut -c1-400
