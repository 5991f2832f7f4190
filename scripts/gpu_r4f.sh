#!/bin/bash
# round 4 (f): specialised pp aggregation, records in registers: parity + C4 step
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r4f; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_pp.py > $O/pytest_pp.log 2>&1 || { tail -40 $O/pytest_pp.log; exit 1; }
tail -2 $O/pytest_pp.log
for v in 1 0; do
  DBG_X_PPSPEC=$v timeout -k 10 240 python -u scripts/step_timing_cfg.py 4 4 > $O/steps_c4_spec$v.json 2> $O/steps_c4_spec$v.err || { tail -5 $O/steps_c4_spec$v.err; exit 1; }
  echo "spec=$v $(cat $O/steps_c4_spec$v.json)"
done
echo done
