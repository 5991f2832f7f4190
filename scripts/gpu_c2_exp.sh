#!/bin/bash
# C2 fast-kernel experiments: xmode (0 full, 1 predicate only, 2 loads only) x grid size; no-flush timing.
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for x in 2 1 0; do
 for b in 256 512 1024 2048; do
  DBG_FAST_XMODE=$x DBG_FAST_MAXBLOCKS=$b timeout -k 10 120 python -u bench.py --steps 50 --warmup 3 --no-cpu-baseline > gpurun_out/exp_x${x}_$b.json 2>gpurun_out/exp.err || exit 1
  python3 -c "import json;d=json.loads(open('gpurun_out/exp_x${x}_$b.json').read().strip().splitlines()[-1]);print('x=$x b=$b', round(d['roofline']['kernel_avg_ms']*1000,2),'us', round(d['ms_per_step']*1000,1),'us/step')"
 done
done
DBG_FAST_NOFLUSH=1 timeout -k 10 120 python -u bench.py --steps 50 --warmup 3 --no-cpu-baseline > gpurun_out/exp_noflush.json 2>>gpurun_out/exp.err || exit 1
python3 -c "import json;d=json.loads(open('gpurun_out/exp_noflush.json').read().strip().splitlines()[-1]);print('noflush', round(d['roofline']['kernel_avg_ms']*1000,2),'us')"
