#!/bin/bash
# All five configs under rocprofv3 kernel-trace (bench JSON + per-kernel stats), then a PMC pass for C2.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for c in ${CONFIGS:-1 3 4 5}; do
  echo "config $c"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c$c -o c$c --output-format csv -- python3 -u bench.py --config $c --steps ${STEPS:-3} --warmup 1 --no-cpu-baseline > gpurun_out/bench_c$c.json 2> gpurun_out/bench_c$c.err || { echo "config $c failed"; tail -20 gpurun_out/bench_c$c.err; exit 1; }
  grep '"metric"' gpurun_out/bench_c$c.json | cut -c1-400
done
if [ -n "$PMC" ]; then
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_c2 -o fetch --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_fetch.log 2>&1 || { echo "pmc fetch failed"; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_c2 -o write --output-format csv -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline > gpurun_out/pmc_write.log 2>&1 || { echo "pmc write failed"; exit 1; }
fi
echo done
