#!/bin/bash
# A/B sweep of the generic insert's LDS partial-table budget (DBG_LDS_BYTES) on C5 and C1.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for b in ${BUDGETS:-16384 32768 65536}; do
  for c in ${CONFIGS:-5 1}; do
    DBG_LDS_BYTES=$b timeout -k 10 300 python -u bench.py --config $c --steps ${STEPS:-3} --warmup 2 --no-cpu-baseline > gpurun_out/lds_${b}_c$c.json 2> gpurun_out/lds_${b}_c$c.err || { echo "bench $b $c failed"; tail -20 gpurun_out/lds_${b}_c$c.err; exit 1; }
    python3 -c "
import json;d=json.loads(open('gpurun_out/lds_${b}_c$c.json').read().strip().splitlines()[-1])
print('lds=$b c$c', 'ms/step=%.4f'%d['ms_per_step'], {k:round(v*1e3,1) for k,v in d['kernels_ms_per_step'].items()})"
  done
done
