#!/bin/bash
# round 4, first GPU call: the ADVICE fixes' tests, host-side step timing per config
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r4a
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_parquet.py tests/test_gpu_compact.py tests/test_gpu_legacy_buckets.py "tests/test_gpu_parity.py::test_partitioned_insert" "tests/test_gpu_fullsize.py::test_c3_full_1b" > gpurun_out/r4a/pytest.log 2>&1 || { tail -30 gpurun_out/r4a/pytest.log; exit 1; }
tail -3 gpurun_out/r4a/pytest.log
for c in 3 1 5 4; do
  timeout -k 10 180 python -u scripts/step_timing_cfg.py $c 4 > gpurun_out/r4a/steps_c$c.json 2> gpurun_out/r4a/steps_c$c.err || { tail -5 gpurun_out/r4a/steps_c$c.err; exit 1; }
  cat gpurun_out/r4a/steps_c$c.json
done
timeout -k 10 240 rocprofv3 --kernel-trace --hip-trace -d gpurun_out/r4a/trace_c3 -o c3 --output-format csv -- python3 -u scripts/step_timing_cfg.py 3 3 > gpurun_out/r4a/trace_c3.log 2>&1 || { tail -5 gpurun_out/r4a/trace_c3.log; exit 1; }

# FETCH_SIZE / WRITE_SIZE calibration microbenchmark (separate --pmc passes)
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/r4a/calib_fetch -o fetch --output-format csv -- ./scripts/micro/fetch_calib > gpurun_out/r4a/calib_known.json 2> gpurun_out/r4a/calib_fetch.err || { tail -5 gpurun_out/r4a/calib_fetch.err; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d gpurun_out/r4a/calib_write -o write --output-format csv -- ./scripts/micro/fetch_calib > gpurun_out/r4a/calib_known2.json 2> gpurun_out/r4a/calib_write.err || { tail -5 gpurun_out/r4a/calib_write.err; exit 1; }
echo calib-done
