#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
timeout -k 10 180 rocprofv3 --runtime-trace -d gpurun_out/trace_c2 -o c2 --output-format csv -- python3 bench.py --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/trace_c2.log 2>&1
