#!/bin/bash
# C4 experiments: bench.py C4 with the pp_agg phase trace (DBG_X_PPTRACE).
set -o pipefail
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
DBG_X_PPTRACE=1 timeout -k 10 240 python -u bench.py --config 4 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/c4_trace.json 2> gpurun_out/c4_trace.err || { echo "bench failed"; tail -5 gpurun_out/c4_trace.err; exit 1; }
grep pptrace gpurun_out/c4_trace.err
python3 -c "
import json;d=json.loads(open('gpurun_out/c4_trace.json').read().strip().splitlines()[-1])
print('ms/step=%.3f'%d['ms_per_step'], {k:round(v,2) for k,v in d['kernels_ms_per_step'].items()})"
