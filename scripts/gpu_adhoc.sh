set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/s7
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_str1.py tests/test_gpu_fullsize.py -k "str1 or c5" > gpurun_out/s7/pytest.log 2>&1 || { tail -40 gpurun_out/s7/pytest.log; exit 1; }
tail -2 gpurun_out/s7/pytest.log
for l in 84 112; do
DBGPU_LIB=$GRAFT_REPO_ROOT/databend_amd/libdbgpu_agg_exp.so DBG_X_STR1_LDS=$l CFG=5 NO_PROF=1 OUT=gpurun_out/s7/l$l bash scripts/gpu_cfg.sh 2>&1 | grep cfg
done
CFG=5 OUT=gpurun_out/s7/c5 bash scripts/gpu_cfg.sh
