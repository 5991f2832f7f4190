set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/s14
CFG=5 OUT=gpurun_out/s14/c5 bash scripts/gpu_cfg.sh
CFG=3 OUT=gpurun_out/s14/c3 NO_PROF=1 bash scripts/gpu_cfg.sh
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_str1.py tests/test_gpu_parity.py -k "str1 or growth or overflow" > gpurun_out/s14/pytest.log 2>&1 || { tail -40 gpurun_out/s14/pytest.log; exit 1; }
tail -2 gpurun_out/s14/pytest.log
CONFIGS="5" bash scripts/gpu_pmc.sh
