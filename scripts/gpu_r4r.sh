#!/bin/bash
# round 4 (r): C1 short-key insert ablations: where the time goes (no flush / no atomics)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r4r; mkdir -p $O
for cfg in "1 0" "3 0" "2 0" "4 0"; do
  set -- $cfg
  DBG_X_SHORT=$1 DBG_X_SHORT_REP=$2 timeout -k 10 240 python -u scripts/step_timing_cfg.py 1 6 > $O/c1_$1_$2.json 2> $O/c1_$1_$2.err || { tail -5 $O/c1_$1_$2.err; exit 1; }
  echo "short=$1 rep=$2 $(cat $O/c1_$1_$2.json)"
done
echo done
