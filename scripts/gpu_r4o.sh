#!/bin/bash
# round 4 (o): short-key specialised insert: parity + C1 A/B
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r4o; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_short_keys.py "tests/test_gpu_parity.py::test_benchmark_configs_match_oracle" tests/test_gpu_parity.py -k "short or bench or string or str" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for v in 1 0; do
  DBG_X_SHORT=$v timeout -k 10 240 python -u scripts/step_timing_cfg.py 1 6 > $O/steps_c1_short$v.json 2> $O/steps_c1_short$v.err || { tail -5 $O/steps_c1_short$v.err; exit 1; }
  echo "short=$v $(cat $O/steps_c1_short$v.json)"
done
echo done
