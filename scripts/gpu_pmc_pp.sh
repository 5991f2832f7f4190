#!/bin/bash
# PMC passes over one bench step of the given configs (default "3 4"): SQ instruction / LDS
# counters, then FETCH_SIZE and WRITE_SIZE in runs of their own.  CSVs under gpurun_out/pmc_pp_c*.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
SQ="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_WAIT_ANY"
for c in ${CONFIGS:-3 4}; do
  for pass in sq fetch write; do
    case $pass in sq) ctr="$SQ";; fetch) ctr="FETCH_SIZE";; write) ctr="WRITE_SIZE";; esac
    echo "[$(date +%T)] c$c $pass"
    timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $ctr -d gpurun_out/pmc_pp_c$c -o $pass --output-format csv -- python3 -u bench.py --config $c --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/pmc_pp_c${c}_$pass.log 2>&1 || { echo "pmc $pass c$c failed"; tail -5 gpurun_out/pmc_pp_c${c}_$pass.log; exit 1; }
  done
done
find gpurun_out/pmc_pp_c* -name "*.csv" | head -20
