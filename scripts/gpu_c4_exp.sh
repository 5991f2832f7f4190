#!/bin/bash
# C4 experiments: bench.py C4 under knobs (RUNS="label:ENV=1,ENV2=1 label2"), pp_agg phase trace
# with the label "trace" (DBG_X_PPTRACE).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for spec in ${RUNS:-"base"}; do
  label=${spec%%:*}; envs=${spec#*:}; [ "$envs" = "$spec" ] && envs=""
  env $(echo $envs | tr ',' ' ') timeout -k 10 240 python -u bench.py --config ${CFG:-4} --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline > gpurun_out/c4_$label.json 2> gpurun_out/c4_$label.err || { echo "bench $label failed"; tail -5 gpurun_out/c4_$label.err; exit 1; }
  grep pptrace gpurun_out/c4_$label.err || true
  python3 -c "
import json;d=json.loads(open('gpurun_out/c4_$label.json').read().strip().splitlines()[-1])
print('$label', 'ms/step=%.3f'%d['ms_per_step'], d.get('parity_vs_cpu'), {k:round(v,2) for k,v in d['kernels_ms_per_step'].items()})"
done
