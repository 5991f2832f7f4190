#!/bin/bash
# round 4 (k): inflate from an LDS window: parquet parity + scan leg + its kernel trace
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r4k; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parquet.py > $O/pytest_pq.log 2>&1 || { tail -40 $O/pytest_pq.log; exit 1; }
tail -2 $O/pytest_pq.log
timeout -k 10 300 python -u scripts/scan_prof.py 10 > $O/scan.json 2> $O/scan.err || { tail -5 $O/scan.err; exit 1; }
cat $O/scan.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o scan --output-format csv -- python3 -u scripts/scan_prof.py 10 > $O/scan_prof.json 2> $O/scan_prof.err || { tail -5 $O/scan_prof.err; exit 1; }
find $O/prof -name "*kernel_stats.csv" | head -1 | xargs cat | cut -c1-200 | head -20
echo done
