set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/s9
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_pp.py tests/test_gpu_payload.py > gpurun_out/s9/pytest.log 2>&1 || { tail -40 gpurun_out/s9/pytest.log; exit 1; }
tail -2 gpurun_out/s9/pytest.log
CFG=4 OUT=gpurun_out/s9/c4 NO_PROF=1 bash scripts/gpu_cfg.sh
CONFIGS="3 5" bash scripts/gpu_pmc.sh
