#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r4d
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py -k "filter or fused or pred or fast or partitioned_insert or bench" "tests/test_gpu_fullsize.py::test_c3_full_1b" "tests/test_gpu_fullsize.py::test_c2_full_100m" > gpurun_out/r4d/pytest.log 2>&1 || { tail -30 gpurun_out/r4d/pytest.log; exit 1; }
tail -2 gpurun_out/r4d/pytest.log
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parquet.py tests/test_gpu_legacy_buckets.py tests/test_legacy_hash.py -m gpu > gpurun_out/r4d/pytest2.log 2>&1 || { tail -30 gpurun_out/r4d/pytest2.log; exit 1; }
tail -2 gpurun_out/r4d/pytest2.log
for nt in 512 1024; do
  DBG_X_SLICE_NT=$nt timeout -k 10 180 python -u scripts/step_timing_cfg.py 3 4 > gpurun_out/r4d/steps_c3_$nt.json 2>&1 || { tail -5 gpurun_out/r4d/steps_c3_$nt.json; exit 1; }
  echo "slice $nt $(tail -1 gpurun_out/r4d/steps_c3_$nt.json)"
done
for c in 1 5; do
  timeout -k 10 180 python -u scripts/step_timing_cfg.py $c 6 > gpurun_out/r4d/steps_c$c.json 2> gpurun_out/r4d/steps_c$c.err || { tail -5 gpurun_out/r4d/steps_c$c.err; exit 1; }
  cat gpurun_out/r4d/steps_c$c.json
done
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum -d gpurun_out/r4d/calib_rdreq -o rdreq --output-format csv -- ./scripts/micro/fetch_calib > gpurun_out/r4d/calib_known.json 2> gpurun_out/r4d/calib_rdreq.err || { tail -5 gpurun_out/r4d/calib_rdreq.err; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum -d gpurun_out/r4d/calib_wrreq -o wrreq --output-format csv -- ./scripts/micro/fetch_calib > /dev/null 2> gpurun_out/r4d/calib_wrreq.err || { tail -5 gpurun_out/r4d/calib_wrreq.err; exit 1; }
for r in 1 2; do
  for v in tail notail; do
    if [ $v = notail ]; then export DBGPU_LIB=$GRAFT_REPO_ROOT/scripts/micro/libdbgpu_agg_notail.so; else unset DBGPU_LIB; fi
    timeout -k 10 300 python -u bench.py --steps 50 --warmup 10 --extra-configs none --no-cpu-baseline > gpurun_out/r4d/bench_c2_$v$r.json 2> gpurun_out/r4d/bench_c2_$v$r.err || { tail -5 gpurun_out/r4d/bench_c2_$v$r.err; exit 1; }
    python -c "import json; d=json.load(open('gpurun_out/r4d/bench_c2_$v$r.json')); print('$v', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['kernel_avg_ms'], d['config']['groups'])"
  done
done
unset DBGPU_LIB
echo done
