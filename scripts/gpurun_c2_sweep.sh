#!/bin/bash
# C2 insert-kernel sweep: grid size knob + rocprof kernel trace
set -o pipefail
cd /tmp && export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT"
for b in 256 512 1024 2048 4096; do
  DBG_FAST_MAXBLOCKS=$b timeout -k 10 120 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/sweep_$b.log 2>&1 || exit 1
done
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c2 -o c2 --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/prof_c2.log 2>&1
