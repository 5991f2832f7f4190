#!/bin/bash
# LDS / atomic / occupancy counter passes over one marker-delimited step of each config
# (scripts/pmc_run.py), one counter group per rocprofv3 run, then scripts/pmc_lds_summary.py ->
# gpurun_out/pmc_lds_atomics_c<cfg>.json (copied into profiles/ when judged).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
SQ1="SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU"
SQ2="SQ_WAVES SQ_LDS_ATOMIC_RETURN SQ_INSTS_SALU SQ_INSTS_VMEM SQ_LDS_ADDR_CONFLICT SQ_LDS_UNALIGNED_STALL"
ATOM="TCC_ATOMIC_sum TCC_EA0_ATOMIC_sum"
for c in ${CONFIGS:-4 5 3 1 2}; do
  O=gpurun_out/pmclds_c$c; rm -rf $O; mkdir -p $O
  for pass in sq1 sq2 atom; do
    case $pass in sq1) ctr="$SQ1";; sq2) ctr="$SQ2";; atom) ctr="$ATOM";; esac
    echo "[$(date +%T)] c$c $pass"
    timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $ctr -d $O/$pass -o $pass --output-format csv -- python3 -u scripts/pmc_run.py --config $c --steps 1 > $O/$pass.log 2>&1 || { echo "pmc $pass c$c failed"; tail -5 $O/$pass.log; exit 1; }
  done
  python3 scripts/pmc_lds_summary.py $O 1 gpurun_out/pmc_lds_atomics_c$c.json || exit 1
done
echo done
