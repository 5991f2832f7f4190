#!/bin/bash
# A/B timing of one config across experiment settings (the EXP=1 library, DBG_X_* knobs):
#   CFG=3 VARIANTS="DBG_X_RP=512,16 DBG_X_RP=1024,8" bash scripts/gpu_ab.sh
# Each variant: bench.py --config CFG, its ms_per_step and kernel split.  Results are timing only.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; O=${OUT:-gpurun_out/ab}; mkdir -p $O
export DBGPU_LIB=$PWD/databend_amd/libdbgpu_agg_exp.so
for rep in ${REPS:-1}; do
for v in $VARIANTS; do
  echo "[$(date +%T)] $v"
  env $(echo $v | tr ';' ' ') timeout -k 10 300 python -u bench.py --config $CFG --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline > $O/ab.json 2> $O/ab.err || { tail -20 $O/ab.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/ab.json').read().strip().splitlines()[-1]); print('  $v', round(d['ms_per_step'],4), 'ms frac', round(d['roofline']['frac'],4), {k: round(v,3) for k,v in d.get('kernels_ms_per_step',{}).items()})"
done
done
echo done
