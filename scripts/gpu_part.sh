#!/bin/bash
# Full GPU parity suite (or -k $PYTEST_K), then C3 A/B (streaming vs partitioned insert), other configs, rocprof of C3.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/pytest_part.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_part.log; exit 1; }
tail -3 gpurun_out/pytest_part.log
CFG=3 STEPS=${STEPS:-4} WARM=1 TMO=240 bash scripts/gpu_ab.sh part: stream:DBG_PART=0 || exit 1
for c in ${MORE:-4 5}; do CFG=$c STEPS=3 WARM=1 TMO=240 bash scripts/gpu_ab.sh c$c: || exit 1; done
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_part -o c3 --output-format csv -- python3 -u bench.py --config 3 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof_part.json 2> gpurun_out/prof_part.err || { echo "rocprof failed"; tail -20 gpurun_out/prof_part.err; exit 1; }
python3 scripts/kstats.py gpurun_out/prof_part/c3_kernel_stats.csv
