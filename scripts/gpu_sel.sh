#!/bin/bash
# Selected GPU test files (TESTS), then optionally the C2 trace and the full gpu_r3 run (FULL=1).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_sel.log 2>&1 || { echo "selected tests failed"; tail -60 gpurun_out/pytest_sel.log; exit 1; }
tail -3 gpurun_out/pytest_sel.log
if [ -n "$FULL" ]; then
  bash scripts/gpu_trace_c2.sh && NO_PMC=1 bash scripts/gpu_r3.sh
fi
