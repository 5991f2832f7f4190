#!/bin/bash
# C1 insert ablations (experiment build): DBG_X_SHORT 1 = full, 3 = no flush, 4 = no adds / flush,
# 5 = loads + predicate only; DBG_X_SHORT_RC 0 = no register slot cache.
export DBGPU_LIB=$PWD/databend_amd/libdbgpu_agg_exp.so
for v in ${VARIANTS:-"1 1" "3 1" "4 1" "5 1" "1 0" "3 0"}; do set -- $v
  DBG_X_SHORT=$1 DBG_X_SHORT_RC=$2 CFG=1 STEPS=200 WARM=20 NO_PROF=1 OUT=gpurun_out/c1x$1_$2 bash scripts/gpu_cfg.sh | grep cfg | sed "s/^/short=$1 rc=$2 /" || exit 1
done
