#!/bin/bash
# C2 A/B: the shipped library against the EXP library (built with a different compile-time
# variant), alternating, REPS rounds of bench.py --config 2 --steps 200.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; O=${OUT:-gpurun_out/c2ab}; mkdir -p $O
for rep in $(seq ${REPS:-3}); do
  for lib in shipped exp; do
    if [ $lib = exp ]; then export DBGPU_LIB=$PWD/databend_amd/libdbgpu_agg_exp.so; else unset DBGPU_LIB; fi
    timeout -k 10 200 python -u bench.py --config 2 --steps ${STEPS:-200} --warmup 20 --no-cpu-baseline > $O/c2.json 2> $O/c2.err || { tail -20 $O/c2.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/c2.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$lib', round(d['ms_per_step']*1e3,2), 'us/step kernel', round(r['kernel_avg_ms']*1e3,2), 'us frac', round(r['frac'],4))"
  done
done
echo done
