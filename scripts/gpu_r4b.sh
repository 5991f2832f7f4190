#!/bin/bash
# round 4: record-centric pp_agg + radix tile-shape sweep
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r4b
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_pp.py "tests/test_gpu_fullsize.py::test_c4_full_1b" "tests/test_gpu_fullsize.py::test_c5_full_1b" > gpurun_out/r4b/pytest.log 2>&1 || { tail -30 gpurun_out/r4b/pytest.log; exit 1; }
tail -3 gpurun_out/r4b/pytest.log
for c in 4 1 5; do
  timeout -k 10 180 python -u scripts/step_timing_cfg.py $c 4 > gpurun_out/r4b/steps_c$c.json 2> gpurun_out/r4b/steps_c$c.err || { tail -5 gpurun_out/r4b/steps_c$c.err; exit 1; }
  cat gpurun_out/r4b/steps_c$c.json
done
DBG_X_PPRC=0 timeout -k 10 180 python -u scripts/step_timing_cfg.py 4 3 > gpurun_out/r4b/steps_c4_oldagg.json 2>&1 && cat gpurun_out/r4b/steps_c4_oldagg.json
for sh in 512,16 1024,8 256,16 512,8 256,32; do
  DBG_X_RP=$sh timeout -k 10 180 python -u scripts/step_timing_cfg.py 3 3 > gpurun_out/r4b/steps_c3_$sh.json 2>&1 || { tail -5 gpurun_out/r4b/steps_c3_$sh.json; exit 1; }
  echo "$sh $(cat gpurun_out/r4b/steps_c3_$sh.json)"
done
