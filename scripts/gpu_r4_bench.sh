#!/bin/bash
# round 4: the default bench line and the rocprofv3 kernel summary of the same command
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r4bench; mkdir -p $O
timeout -k 10 900 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
cat $O/bench_default.json | cut -c1-600
timeout -k 10 900 rocprofv3 --kernel-trace --stats -d $O/prof -o bench --output-format csv -- python3 -u bench.py > $O/bench_prof.json 2> $O/bench_prof.err || { tail -20 $O/bench_prof.err; exit 1; }
find $O/prof -name "*kernel_stats.csv" | head -1 | xargs head -12 | cut -c1-160
echo done
