#!/bin/bash
# Timing experiments on the filtered generic insert (DBG_GEN_XMODE; results are NOT valid
# aggregates in modes 1-5): 1 scan+queue only, 2 + string hash, 3 + LDS probe (no flush, LDS
# misses dropped), 4 LDS probe then the normal HBM path, 5 normal without periodic LDS flushes.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for m in ${MODES:-0 1 2 3 4 5}; do
  for c in ${CONFIGS:-5}; do
    DBG_GEN_XMODE=$m timeout -k 10 300 python -u bench.py --config $c --steps ${STEPS:-3} --warmup 2 --no-cpu-baseline > gpurun_out/xm_${m}_c$c.json 2> gpurun_out/xm_${m}_c$c.err || { echo "bench $m $c failed"; tail -5 gpurun_out/xm_${m}_c$c.err; continue; }
    python3 -c "
import json;d=json.loads(open('gpurun_out/xm_${m}_c$c.json').read().strip().splitlines()[-1])
print('xmode=$m c$c', 'ms/step=%.4f'%d['ms_per_step'], {k:round(v*1e3,1) for k,v in d['kernels_ms_per_step'].items()})"
  done
done
