set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/s8
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_fused_dense.py tests/test_gpu_parity.py -k "fast or fused or golden or c2 or config" > gpurun_out/s8/pytest.log 2>&1 || { tail -40 gpurun_out/s8/pytest.log; exit 1; }
tail -2 gpurun_out/s8/pytest.log
for r in 1 2 3; do
timeout -k 10 300 python -u bench.py --no-cpu-baseline --extra-configs none --steps 200 --warmup 10 > gpurun_out/s8/b$r.json 2> gpurun_out/s8/b$r.err || exit 1
python3 -c "import json; d=json.loads(open('gpurun_out/s8/b$r.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['roofline']['kernel_avg_ms'], d['roofline']['frac'])"
done
bash scripts/gpu_trace_c2.sh
