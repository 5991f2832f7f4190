#!/bin/bash
# Uncompressed Parquet decode vs the y-piece size of required PLAIN pages (DBG_X_PQ_PIECE; experiment build).
export DBGPU_LIB=$PWD/databend_amd/libdbgpu_agg_exp.so
for v in ${PIECES:-8192 4096 2048 1024}; do
  DBG_X_PQ_PIECE=$v timeout -k 10 120 python3 scripts/scan_run.py --codec NONE --steps 50 --time | grep "ms per" | sed "s/^/piece=$v /" || exit 1
done
