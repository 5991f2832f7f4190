#!/bin/bash
# One config's bench line (and, unless NO_PROF, its rocprofv3 kernel summary).
#   CFG=5 ARGS="--strategy partitioned" OUT=gpurun_out/c5pp bash scripts/gpu_cfg.sh
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; O=${OUT:-gpurun_out/cfg$CFG}; mkdir -p $O
timeout -k 10 ${TLIM:-300} python -u bench.py --config $CFG --steps ${STEPS:-5} --warmup ${WARM:-2} --no-cpu-baseline --extra-configs none ${ARGS} > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "
import json,sys; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1])
print('cfg $CFG', d['ms_per_step'], d['roofline'].get('frac'), json.dumps(d.get('kernels_ms_per_step')))"
if [ -z "$NO_PROF" ]; then
  timeout -k 10 ${TLIM:-300} rocprofv3 --kernel-trace --stats -d $O/prof -o k --output-format csv -- python3 -u bench.py --config $CFG --steps ${STEPS:-5} --warmup ${WARM:-2} --no-cpu-baseline --extra-configs none ${ARGS} > $O/prof.json 2> $O/prof.err || { tail -20 $O/prof.err; exit 1; }
  find $O/prof -name "*kernel_stats.csv" | head -1 | xargs head -12 | cut -c1-200
fi
echo done
