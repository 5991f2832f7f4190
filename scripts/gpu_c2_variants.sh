#!/bin/bash
# C2 kernel time: the shipped library against in-tree experiment builds (LIBS="name ..." ->
# databend_amd/libdbgpu_x_<name>.so), alternating, REPS rounds of bench.py --config 2 --steps 200.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; O=${OUT:-gpurun_out/c2var}; mkdir -p $O
for rep in $(seq ${REPS:-2}); do
  for lib in shipped ${LIBS}; do
    if [ $lib = shipped ]; then unset DBGPU_LIB; else export DBGPU_LIB=$PWD/databend_amd/libdbgpu_x_$lib.so; fi
    timeout -k 10 200 python -u bench.py --config 2 --steps ${STEPS:-200} --warmup 20 --no-cpu-baseline --extra-configs none > $O/c2.json 2> $O/c2.err || { tail -20 $O/c2.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/c2.json').read().strip().splitlines()[-1]); r=d['roofline']; print('$lib', round(d['ms_per_step']*1e3,2), 'us/step kernel', round(r['kernel_avg_ms']*1e3,2), 'us frac', round(r['frac'],4))"
  done
done
echo done
