#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for cfg in "DBG_FAST_MAXBLOCKS=256" "DBG_FAST_MINB=2 DBG_FAST_MAXBLOCKS=512" "DBG_FAST_MINB=2 DBG_FAST_MAXBLOCKS=256" "DBG_FAST_MAXBLOCKS=256"; do
  env $cfg timeout -k 10 120 python -u bench.py --steps 50 --warmup 3 --no-cpu-baseline > gpurun_out/sel.json 2>gpurun_out/sel.err || { tail gpurun_out/sel.err; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/sel.json').read().strip().splitlines()[-1]);print('$cfg', round(d['roofline']['kernel_avg_ms']*1000,2),'us', round(d['ms_per_step']*1000,1),'us/step')"
done
