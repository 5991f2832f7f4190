#!/bin/bash
# Inputs of the multi-GPU projections: C3 at one GPU's share of the 8-GPU strong
# scaling run (1.25e8 rows) under both strategies, and at full size partitioned; C5 at its share.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; O=gpurun_out/proj; mkdir -p $O
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline --extra-configs none "$@" > $O/$n.json 2> $O/$n.err || { tail -20 $O/$n.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/$n.json').read().strip().splitlines()[-1]); print('$n', round(d['ms_per_step'],3), 'ms', d['config'].get('groups'), {k: round(v,3) for k,v in d.get('kernels_ms_per_step',{}).items()})"
}
run c3_125m_auto --config 3 --rows 125000000
run c3_125m_part --config 3 --rows 125000000 --strategy partitioned
run c3_1b_part --config 3 --strategy partitioned
run c5_125m --config 5 --rows 125000000
run c4_125m --config 4 --rows 125000000
echo done
