#!/bin/bash
# C2 phase trace: the fused insert+finalize launch's timestamps (DBG_X_TRACE, medians over launches).
# Needs a library built with phase tracing (here, before the GPU call):
#   make -C databend_amd/csrc clean && make -C databend_amd/csrc TRACE=1
# (it builds databend_amd/libdbgpu_agg_exp.so; the shipped library is untouched).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
DBG_X_TRACE=1 DBGPU_LIB=$GRAFT_REPO_ROOT/databend_amd/libdbgpu_agg_exp.so timeout -k 10 120 python -u bench.py --config 2 --steps 200 --warmup 10 --no-cpu-baseline --extra-configs none \
  > gpurun_out/trace_c2.json 2> gpurun_out/trace_c2.err || { echo "trace failed"; tail -20 gpurun_out/trace_c2.err; exit 1; }
grep trace gpurun_out/trace_c2.err
cut -c1-300 gpurun_out/trace_c2.json
