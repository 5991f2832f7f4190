set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/s13


CFG=4 OUT=gpurun_out/s13/c4 NO_PROF=1 bash scripts/gpu_cfg.sh
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_pp.py tests/test_abi.py > gpurun_out/s13/pytest.log 2>&1 || { tail -40 gpurun_out/s13/pytest.log; exit 1; }
tail -2 gpurun_out/s13/pytest.log
