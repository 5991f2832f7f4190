#!/bin/bash
# round 4 (i): specialised pp aggregation with LDS-only barriers and batched staging: parity, C4 step, phase trace
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r4i; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_pp.py > $O/pytest_pp.log 2>&1 || { tail -40 $O/pytest_pp.log; exit 1; }
tail -2 $O/pytest_pp.log
timeout -k 10 240 python -u scripts/step_timing_cfg.py 4 4 > $O/steps_c4.json 2> $O/steps_c4.err || { tail -5 $O/steps_c4.err; exit 1; }
cat $O/steps_c4.json
true
true
echo done
