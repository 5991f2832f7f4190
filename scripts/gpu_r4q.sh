#!/bin/bash
# round 4 (q): C1 short-key insert ablations: LDS-slot replicas, no aggregate atomics (timing only)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r4q; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_short_keys.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for cfg in "1 0" "1 2" "1 4" "1 8" "1 16" "2 0"; do
  set -- $cfg
  DBG_X_SHORT=$1 DBG_X_SHORT_REP=$2 timeout -k 10 240 python -u scripts/step_timing_cfg.py 1 6 > $O/c1_$1_$2.json 2> $O/c1_$1_$2.err || { tail -5 $O/c1_$1_$2.err; exit 1; }
  echo "short=$1 rep=$2 $(cat $O/c1_$1_$2.json)"
done
for r in 2 4; do
  DBG_X_SHORT_REP=$r timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_short_keys.py > $O/pytest_rep$r.log 2>&1 || { tail -30 $O/pytest_rep$r.log; exit 1; }
  echo "rep=$r $(tail -1 $O/pytest_rep$r.log)"
done
echo done
