#!/bin/bash
# round 4 (t): short-key insert with narrow Decimal sums and the merge-tree flush: parity + C1 A/B
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r4t; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_short_keys.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
run() { env $1 timeout -k 10 240 python -u scripts/step_timing_cfg.py 1 6 > $O/c1_$2.json 2> $O/c1_$2.err || { tail -5 $O/c1_$2.err; exit 1; }; echo "$2 $(cat $O/c1_$2.json)"; }
run DBG_X_SHORT=1 base
run DBG_X_TREE=0 notree
run DBG_X_NARROW=0 nonarrow
run DBG_X_SHORT=3 noflush
for v in "DBG_X_TREE=0" "DBG_X_NARROW=0"; do
  env $v timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_short_keys.py > $O/pytest_$v.log 2>&1 || { tail -30 $O/pytest_$v.log; exit 1; }
  echo "$v $(tail -1 $O/pytest_$v.log)"
done
echo done
