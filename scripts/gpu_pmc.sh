#!/bin/bash
# FETCH_SIZE / WRITE_SIZE passes over marker-delimited steps of C1, C3, C4, C5 (kernels changed
# this round) -> profiles/pmc_traffic_c*.json via scripts/pmc_step_traffic.py
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
declare -A ALG=([1]=603864258 [2]=200000320 [3]=10146238128 [4]=52000000000 [5]=10673805104)
for c in ${CONFIGS:-1 3 4 5}; do
  st=2; [ "$c" = 2 ] && st=10
  rm -rf gpurun_out/pmc4_c$c
  for pass in fetch write; do
    case $pass in fetch) ctr="FETCH_SIZE";; write) ctr="WRITE_SIZE";; esac
    echo "[$(date +%T)] c$c $pass"
    timeout -s KILL 300 rocprofv3 --kernel-trace --pmc $ctr -d gpurun_out/pmc4_c$c/$pass -o $pass --output-format csv -- python3 -u scripts/pmc_run.py --config $c --steps $st > gpurun_out/pmc4_c${c}_$pass.log 2>&1 || { echo "pmc $pass c$c failed"; tail -5 gpurun_out/pmc4_c${c}_$pass.log; exit 1; }
  done
  python3 scripts/pmc_step_traffic.py gpurun_out/pmc4_c$c $st gpurun_out/pmc_traffic_c$c.json ${ALG[$c]} || exit 1
  python3 -c "import json; d=json.load(open('gpurun_out/pmc_traffic_c$c.json')); print('c$c', d['hbm_bytes_per_launch'], d['traffic_over_algorithmic'])"
done
echo done
