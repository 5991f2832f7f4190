#!/bin/bash
# round 4 (l): generic insert without the selection queue (C1: 97 % selected) A/B, C5 beside it
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r4l; mkdir -p $O
for v in 0 1; do
  for c in 1 5; do
    DBG_X_NOQUEUE=$v timeout -k 10 240 python -u scripts/step_timing_cfg.py $c 6 > $O/steps_c${c}_nq$v.json 2> $O/steps_c${c}_nq$v.err || { tail -5 $O/steps_c${c}_nq$v.err; exit 1; }
    echo "noqueue=$v $(cat $O/steps_c${c}_nq$v.json)"
  done
done
DBG_X_NOQUEUE=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "bench or filter or pred" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
echo done
