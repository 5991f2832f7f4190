#!/bin/bash
# round 4: predicate loop restructure (C1, C5), C2 bench, counters list
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/r4c
for c in 1 5; do
  timeout -k 10 180 python -u scripts/step_timing_cfg.py $c 6 > gpurun_out/r4c/steps_c$c.json 2> gpurun_out/r4c/steps_c$c.err || { tail -5 gpurun_out/r4c/steps_c$c.err; exit 1; }
  cat gpurun_out/r4c/steps_c$c.json
done
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --extra-configs none --no-cpu-baseline > gpurun_out/r4c/bench_c2.json 2> gpurun_out/r4c/bench_c2.err || { tail -5 gpurun_out/r4c/bench_c2.err; exit 1; }
python -c "import json; d=json.load(open('gpurun_out/r4c/bench_c2.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['kernel_avg_ms'])"
timeout -k 10 60 rocprofv3 -L > gpurun_out/r4c/counters.txt 2>&1 || true
