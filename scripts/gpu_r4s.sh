#!/bin/bash
# round 4 (s): SQ counters of the C1 short-key insert (full, and without atomics + flush)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r4s; rm -rf $O; mkdir -p $O
CT="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY"
for m in 1 4; do
  DBG_X_SHORT=$m timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $CT -d $O/m$m -o sq --output-format csv -- python3 -u scripts/pmc_run.py --config 1 --steps 2 > $O/m$m.log 2>&1 || { echo "pmc m$m failed"; tail -5 $O/m$m.log; exit 1; }
  f=$(find $O/m$m -name "*counter_collection.csv" | head -1)
  python3 - "$f" <<'PY'
import csv, sys, collections
acc = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    if "agg_insert_short" in r["Kernel_Name"]:
        acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
print({k: v[-1] for k, v in sorted(acc.items())})
PY
done
echo done
