#!/bin/bash
# bench.py for each config in $CONFIGS (default "4 3 5"), short runs, one summary line each.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for c in ${CONFIGS:-4 3 5}; do
  timeout -k 10 300 python -u bench.py --config $c --steps ${STEPS:-3} --warmup ${WARM:-1} --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/bench_c$c.json 2> gpurun_out/bench_c$c.err || { echo "bench $c failed"; tail -20 gpurun_out/bench_c$c.err; exit 1; }
  python3 - "$c" <<'PY'
import json, sys
c = sys.argv[1]
d = json.loads(open(f"gpurun_out/bench_c{c}.json").read().strip().splitlines()[-1])
print(f"c{c} ms/step={d['ms_per_step']:.3f} rows/s={d['value']:.3e} frac={d['roofline']['frac']:.3f}",
      {k: round(v, 3) for k, v in d["kernels_ms_per_step"].items()})
PY
done
