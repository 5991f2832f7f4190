#!/bin/bash
# A/B of env knobs on one config: each argument is "label:VAR=val,VAR2=val" (empty env allowed).
#   CFG=2 STEPS=50 bash scripts/gpu_ab.sh base: pf0:DBG_FAST_PF=0
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for spec in "$@"; do
  label=${spec%%:*}; envs=${spec#*:}
  ( IFS=','; for kv in $envs; do [ -n "$kv" ] && export "$kv"; done
    timeout -k 10 ${TMO:-120} python -u bench.py --config ${CFG:-2} --steps ${STEPS:-50} --warmup ${WARM:-3} --no-cpu-baseline > gpurun_out/ab_$label.json 2>gpurun_out/ab_$label.err ) || { echo "$label failed"; tail -5 gpurun_out/ab_$label.err; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/ab_$label.json').read().strip().splitlines()[-1]);print('$label', round(d['roofline']['kernel_avg_ms']*1000,2),'us/insert', round(d['ms_per_step']*1000,1),'us/step', round(d['roofline']['frac'],3), {k: round(v*1000,1) for k,v in d['kernels_ms_per_step'].items()})"
done
