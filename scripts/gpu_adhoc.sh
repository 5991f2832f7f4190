set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/s5
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_str1.py tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_pipeline.py tests/test_gpu_short_keys.py > gpurun_out/s5/pytest.log 2>&1 || { tail -40 gpurun_out/s5/pytest.log; exit 1; }
tail -2 gpurun_out/s5/pytest.log
CFG=5 OUT=gpurun_out/s5/c5 bash scripts/gpu_cfg.sh
