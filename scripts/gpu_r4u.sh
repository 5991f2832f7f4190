#!/bin/bash
# round 4 (u): C1 finalize ablations (timing only) + short-key parity with the defaults
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r4u; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_short_keys.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
run() { env $1 timeout -k 10 240 python -u scripts/step_timing_cfg.py 1 6 > $O/c1_$2.json 2> $O/c1_$2.err || { tail -5 $O/c1_$2.err; exit 1; }; echo "$2 $(cat $O/c1_$2.json)"; }
run DBG_X_FIN=0 base
run DBG_X_FIN=1 nowrite
run DBG_X_FIN=2 nobits
run DBG_X_FIN=8 empty
run DBG_X_FIN=3 nowrite_nobits
echo done
