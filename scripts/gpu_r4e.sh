#!/bin/bash
# round 4 (e): pp specialised kernel parity + C4 A/B, Zstd/legacy parity, C2 tail A/B, C3 slice NT, PMC calibration
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r4e
O=gpurun_out/r4e
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_pp.py > $O/pytest_pp.log 2>&1 || { tail -40 $O/pytest_pp.log; exit 1; }
tail -2 $O/pytest_pp.log
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parquet.py tests/test_gpu_legacy_buckets.py tests/test_legacy_hash.py -m gpu > $O/pytest2.log 2>&1 || { tail -40 $O/pytest2.log; exit 1; }
tail -2 $O/pytest2.log
for v in 1 0; do
  DBG_X_PPSPEC=$v timeout -k 10 240 python -u scripts/step_timing_cfg.py 4 4 > $O/steps_c4_spec$v.json 2> $O/steps_c4_spec$v.err || { tail -5 $O/steps_c4_spec$v.err; exit 1; }
  echo "spec=$v $(cat $O/steps_c4_spec$v.json)"
done
for nt in 512 1024; do
  DBG_X_SLICE_NT=$nt timeout -k 10 180 python -u scripts/step_timing_cfg.py 3 4 > $O/steps_c3_$nt.json 2>&1 || { tail -5 $O/steps_c3_$nt.json; exit 1; }
  echo "slice $nt $(tail -1 $O/steps_c3_$nt.json)"
done
for c in 1 5; do
  timeout -k 10 180 python -u scripts/step_timing_cfg.py $c 6 > $O/steps_c$c.json 2> $O/steps_c$c.err || { tail -5 $O/steps_c$c.err; exit 1; }
  cat $O/steps_c$c.json
done
for r in 1 2; do
  for v in tail notail; do
    if [ $v = notail ]; then export DBGPU_LIB=$GRAFT_REPO_ROOT/scripts/micro/libdbgpu_agg_notail.so; else unset DBGPU_LIB; fi
    timeout -k 10 300 python -u bench.py --steps 50 --warmup 10 --extra-configs none --no-cpu-baseline > $O/bench_c2_$v$r.json 2> $O/bench_c2_$v$r.err || { tail -5 $O/bench_c2_$v$r.err; exit 1; }
    python -c "import json; d=json.load(open('$O/bench_c2_$v$r.json')); print('$v', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['kernel_avg_ms'], d['config']['groups'])"
  done
done
unset DBGPU_LIB
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc TCC_EA0_RDREQ_32B_sum TCC_EA0_RDREQ_64B_sum TCC_EA0_RDREQ_128B_sum -d $O/calib_rdreq -o rdreq --output-format csv -- ./scripts/micro/fetch_calib > $O/calib_known.json 2> $O/calib_rdreq.err || { tail -5 $O/calib_rdreq.err; exit 1; }
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum -d $O/calib_wrreq -o wrreq --output-format csv -- ./scripts/micro/fetch_calib > /dev/null 2> $O/calib_wrreq.err || { tail -5 $O/calib_wrreq.err; exit 1; }
echo done
