#!/bin/bash
# The default bench line and the rocprofv3 kernel summary of the same command.
# OUT (default gpurun_out/bench) receives the line, the logs and the rocprofv3 output.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; O=${OUT:-gpurun_out/bench}; mkdir -p $O
timeout -k 10 900 python -u bench.py ${BENCH_ARGS} > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
cut -c1-600 $O/bench_default.json
if [ -z "$NO_PROF" ]; then
  timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $O/prof -o bench --output-format csv -- python3 -u bench.py ${BENCH_ARGS} > $O/bench_prof.json 2> $O/bench_prof.err || { tail -20 $O/bench_prof.err; exit 1; }
  find $O/prof -name "*kernel_stats.csv" | head -1 | xargs head -14 | cut -c1-160
fi
echo done
