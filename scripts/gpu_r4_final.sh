#!/bin/bash
# round 4: the whole GPU test suite, then the default bench line and its rocprofv3 kernel summary
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r4final; mkdir -p $O
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests -m gpu > $O/pytest_gpu.log 2>&1 || { tail -40 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
echo done
