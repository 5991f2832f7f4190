#!/bin/bash
# SQ counter passes over the scan kernels of one codec (scripts/scan_run.py), one counter group per
# rocprofv3 run -> gpurun_out/pmc_scan_<codec>/<pass>/...counter_collection.csv
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
SQ1="SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_SALU"
SQ2="SQ_WAVES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD"
for codec in ${CODECS:-SNAPPY LZ4}; do
  O=gpurun_out/pmc_scan_$codec; rm -rf $O; mkdir -p $O
  for pass in sq1 sq2; do
    case $pass in sq1) ctr="$SQ1";; sq2) ctr="$SQ2";; esac
    echo "[$(date +%T)] $codec $pass"
    timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $ctr -d $O/$pass -o $pass --output-format csv -- python3 -u scripts/scan_run.py --codec $codec --steps 1 > $O/$pass.log 2>&1 || { echo "pmc $pass $codec failed"; tail -5 $O/$pass.log; exit 1; }
  done
done
echo done
