#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
for x in 0 1 2; do
 for b in 256 512; do
  DBG_FAST_XMODE=$x DBG_FAST_MAXBLOCKS=$b timeout -k 10 120 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/exp_x${x}_$b.log 2>&1 || exit 1
 done
done
