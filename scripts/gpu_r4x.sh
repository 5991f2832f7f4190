#!/bin/bash
# round 4 (x): short-key insert limited to small tables: parity + C1 / C5 steps
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r4x; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_short_keys.py tests/test_gpu_parity.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for c in 1 5; do
  timeout -k 10 300 python -u scripts/step_timing_cfg.py $c 4 > $O/c$c.json 2> $O/c$c.err || { tail -5 $O/c$c.err; exit 1; }
  echo "c$c $(cat $O/c$c.json)"
done
echo done
