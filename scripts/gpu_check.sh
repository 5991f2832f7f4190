#!/bin/bash
# A focused GPU check: the given pytest selection, then bench.py for the given configs
# (TESTS="..." CONFIGS="3 4").  Every GPU step has its own time limit; the first failure ends it.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; O=${OUT:-gpurun_out/check}; mkdir -p $O
if [ -n "$TESTS" ]; then
  echo "[$(date +%T)] pytest $TESTS"
  timeout -k 10 ${TEST_LIMIT:-900} python -u -m pytest -x -v --timeout 300 --timeout-method thread $TESTS > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
  tail -3 $O/pytest.log
fi
for c in $CONFIGS; do
  echo "[$(date +%T)] bench config $c"
  timeout -k 10 300 python -u bench.py --config $c --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline > $O/bench_c$c.json 2> $O/bench_c$c.err || { tail -20 $O/bench_c$c.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$O/bench_c$c.json').read().strip().splitlines()[-1]); r=d['roofline']; print('c$c', round(d['ms_per_step'],3), 'ms', '%.3g rows/s'%d['value'], 'frac', round(r['frac'],4), r['kernel'][:60], {k: round(v,3) for k,v in d.get('kernels_ms_per_step',{}).items()})"
done
echo "[$(date +%T)] done"
