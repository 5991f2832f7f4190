#!/bin/bash
# One config's step and kernel times: the shipped library against in-tree experiment builds
# (LIBS="name ..." -> databend_amd/libdbgpu_x_<name>.so), alternating, REPS rounds.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; O=${OUT:-gpurun_out/cfgvar}; mkdir -p $O
for rep in $(seq ${REPS:-2}); do
  for lib in shipped ${LIBS}; do
    if [ $lib = shipped ]; then unset DBGPU_LIB; else export DBGPU_LIB=$PWD/databend_amd/libdbgpu_x_$lib.so; fi
    timeout -k 10 300 python -u bench.py --config ${CFG:-4} --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline --extra-configs none > $O/c.json 2> $O/c.err || { tail -20 $O/c.err; exit 1; }
    python3 -c "import json; d=json.loads(open('$O/c.json').read().strip().splitlines()[-1]); print('$lib', round(d['ms_per_step'],3), 'ms', {k: round(v,3) for k,v in d.get('kernels_ms_per_step',{}).items()})"
  done
done
echo done
