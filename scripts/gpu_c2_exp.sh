#!/bin/bash
# C2 experiments: bench.py C2 under knobs (DBG_X_*), phase trace of the fused kernel.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
run() {  # label, env...
  local label=$1; shift
  env "$@" timeout -k 10 120 python -u bench.py --config 2 --steps 200 --warmup 20 --no-cpu-baseline > gpurun_out/c2_$label.json 2> gpurun_out/c2_$label.err || { echo "bench $label failed"; tail -5 gpurun_out/c2_$label.err; exit 1; }
  python3 -c "
import json;d=json.loads(open('gpurun_out/c2_$label.json').read().strip().splitlines()[-1])
print('$label', 'ms/step=%.4f'%d['ms_per_step'], 'frac=%.3f'%d['roofline']['frac'], {k:round(v*1e3,2) for k,v in d['kernels_ms_per_step'].items()})"
  grep trace gpurun_out/c2_$label.err || true
}
for spec in ${RUNS:-"base"}; do
  label=${spec%%:*}; envs=${spec#*:}; [ "$envs" = "$spec" ] && envs=""
  run $label $(echo $envs | tr ',' ' ')
done
