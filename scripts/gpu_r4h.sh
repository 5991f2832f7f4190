#!/bin/bash
# round 4 (h): fused dense hand-off (C2) parity + A/B + grid sweep + phase traces; DISTINCT processors; C4 pp trace
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r4h; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_fused_dense.py tests/test_gpu_distinct.py "tests/test_gpu_parity.py" -k "dense or distinct or fast or bench or recycl or c2" > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
TL=$GRAFT_REPO_ROOT/scripts/micro/libdbgpu_agg_trace.so
DBGPU_LIB=$TL DBG_X_PPTRACE=1 timeout -k 10 240 python -u scripts/step_timing_cfg.py 4 2 > $O/steps_c4_trace.json 2> $O/steps_c4_trace.err || { tail -5 $O/steps_c4_trace.err; exit 1; }
grep pptrace $O/steps_c4_trace.err || true
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 300 python -u bench.py --steps 100 --warmup 20 --extra-configs none --no-cpu-baseline > $O/bench_c2_$name.json 2> $O/bench_c2_$name.err || { tail -5 $O/bench_c2_$name.err; return 1; }
  python -c "import json; d=json.load(open('$O/bench_c2_$name.json')); print('$name', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['kernel_avg_ms'], d['config']['groups'])"
}
for r in 1 2; do
  run dense$r DBG_X_DENSE=1 && run chain$r DBG_X_DENSE=0 && run dense512_$r DBG_X_FAST_GRID=512 && run dense1024_$r DBG_X_FAST_GRID=1024 || exit 1
done
DBGPU_LIB=$TL DBG_X_TRACE=1 timeout -k 10 300 python -u bench.py --steps 200 --warmup 20 --extra-configs none --no-cpu-baseline > $O/trace_dense.json 2> $O/trace_dense.err || { tail -5 $O/trace_dense.err; exit 1; }
grep "^trace" $O/trace_dense.err || true
DBGPU_LIB=$TL DBG_X_TRACE=1 DBG_X_DENSE=0 timeout -k 10 300 python -u bench.py --steps 200 --warmup 20 --extra-configs none --no-cpu-baseline > $O/trace_chain.json 2> $O/trace_chain.err || { tail -5 $O/trace_chain.err; exit 1; }
grep "^trace" $O/trace_chain.err || true
echo done
