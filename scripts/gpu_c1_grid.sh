#!/bin/bash
# C1 insert vs the short kernel's grid size (DBG_X_SHORT_BLOCKS; experiment build).
export DBGPU_LIB=$PWD/databend_amd/libdbgpu_agg_exp.so
for b in ${GRIDS:-1280 1465 1536 2048 1024}; do
  DBG_X_SHORT_BLOCKS=$b CFG=1 STEPS=200 WARM=20 NO_PROF=1 OUT=gpurun_out/c1g$b bash scripts/gpu_cfg.sh | grep cfg | sed "s/^/blocks=$b /" || exit 1
done
