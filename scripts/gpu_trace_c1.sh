#!/bin/bash
# C1 phase trace: the short-key insert's timestamps (DBG_X_TRACE_SHORT, medians over launches),
# with the block_flush groups (DBG_X_TREE=0, shipped) and the merge tree (DBG_X_TREE=1).
# Needs the trace build (here, before the GPU call): make -C databend_amd/csrc TRACE=1
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for ch in ${TREES:-0 1}; do
  DBG_X_TREE=$ch DBG_X_TRACE_SHORT=1 DBGPU_LIB=$GRAFT_REPO_ROOT/databend_amd/libdbgpu_agg_exp.so timeout -k 10 120 python -u bench.py --config 1 --steps 200 --warmup 10 --no-cpu-baseline --extra-configs none \
    > gpurun_out/trace_c1_ch$ch.json 2> gpurun_out/trace_c1_ch$ch.err || { echo "trace failed"; tail -20 gpurun_out/trace_c1_ch$ch.err; exit 1; }
  echo "tree=$ch"; grep "short trace" gpurun_out/trace_c1_ch$ch.err
  python3 -c "import json; d=json.loads(open('gpurun_out/trace_c1_ch$ch.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d.get('kernels_ms_per_step'))"
done
