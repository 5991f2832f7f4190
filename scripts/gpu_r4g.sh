#!/bin/bash
# round 4 (g): phase trace of the specialised pp aggregation (C4)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r4g; mkdir -p $O
DBGPU_LIB=$GRAFT_REPO_ROOT/scripts/micro/libdbgpu_agg_trace.so DBG_X_PPTRACE=1 timeout -k 10 240 python -u scripts/step_timing_cfg.py 4 2 > $O/steps_c4_trace.json 2> $O/steps_c4_trace.err || { tail -5 $O/steps_c4_trace.err; exit 1; }
cat $O/steps_c4_trace.json; grep pptrace $O/steps_c4_trace.err
