#!/bin/bash
# Round profile: rocprofv3 kernel-trace stats of bench.py for every config, then PMC passes
# (one counter group per run, as MI355X_MICROARCH.md prescribes): SQ instruction / LDS counters,
# FETCH_SIZE, WRITE_SIZE, L2 atomics.  Outputs under gpurun_out/prof/c<cfg>/<pass>/.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/prof
SQ="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_LDS_ATOMIC_RETURN"
for c in ${CONFIGS:-2 1 3 4 5}; do
  st=20; [ "$c" != 2 ] && st=${STEPS:-3}
  [ "$c" = 1 ] && st=10
  echo "[$(date +%T)] c$c stats"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof/c$c/stats -o c$c --output-format csv -- python3 -u bench.py --config $c --steps $st --warmup 2 --no-cpu-baseline > gpurun_out/prof/c${c}_bench.json 2> gpurun_out/prof/c${c}_bench.err || { echo "stats c$c failed"; tail -5 gpurun_out/prof/c${c}_bench.err; exit 1; }
  [ "${NO_PMC:-0}" = 1 ] && continue
  for pass in sq fetch write atom; do
    case $pass in sq) ctr="$SQ";; fetch) ctr="FETCH_SIZE";; write) ctr="WRITE_SIZE";; atom) ctr="TCC_ATOMIC_sum TCC_EA0_ATOMIC_sum";; esac
    echo "[$(date +%T)] c$c $pass"
    timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $ctr -d gpurun_out/prof/c$c/$pass -o $pass --output-format csv -- python3 -u bench.py --config $c --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/prof/c${c}_$pass.log 2>&1 || { echo "pmc $pass c$c failed"; tail -5 gpurun_out/prof/c${c}_$pass.log; exit 1; }
  done
done
echo "[$(date +%T)] done"
