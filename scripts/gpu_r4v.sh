#!/bin/bash
# round 4 (v): decimal-avg divide fast path: parity of every aggregate test + C1 step, then the bench line and rocprof summary
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r4v; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_short_keys.py tests/test_gpu_parity.py tests/test_gpu_fused_dense.py tests/test_gpu_pipeline.py tests/test_gpu_distinct.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 240 python -u scripts/step_timing_cfg.py 1 6 > $O/c1.json 2> $O/c1.err || { tail -5 $O/c1.err; exit 1; }
echo "c1 $(cat $O/c1.json)"
echo done
