#!/bin/bash
# Compaction tests, then C1 / C2 with SCR_GROUP 4 / 16 / 64 builds (DBGPU_LIB).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_compact.py tests/test_gpu_pipeline.py tests/test_gpu_serialized.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_cmp.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/pytest_cmp.log; exit 1; }
tail -2 gpurun_out/pytest_cmp.log
for lib in libdbgpu_agg.so libdbgpu_agg_g4.so libdbgpu_agg_g64.so; do
  for c in 1 2; do
    st=5; [ $c = 2 ] && st=200
    DBGPU_LIB=$GRAFT_REPO_ROOT/databend_amd/$lib timeout -k 10 200 python3 -u bench.py --config $c --steps $st --warmup 3 --no-cpu-baseline --extra-configs none > gpurun_out/sg_${lib}_$c.json 2> gpurun_out/sg_${lib}_$c.err || { echo "failed $lib $c"; tail -20 gpurun_out/sg_${lib}_$c.err; exit 1; }
    python3 -c "import json;d=json.load(open('gpurun_out/sg_${lib}_$c.json'));print('$lib c$c', round(d['ms_per_step']*1000,2), 'us', d['roofline'].get('kernel_avg_ms'))"
  done
done
