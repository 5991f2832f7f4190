#!/bin/bash
# round 4 (m): why the required-PLAIN decode runs at ~1 TB/s: SQ / fetch counters of pq_decode_kernel
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r4m; mkdir -p $O
timeout -k 10 300 python -u scripts/scan_prof.py 4 > $O/scan.json 2> $O/scan.err || { tail -5 $O/scan.err; exit 1; }
cut -c1-300 $O/scan.json
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY -d $O/sq -o sq --output-format csv -- python3 -u scripts/scan_prof.py 2 > $O/sq.log 2>&1 || { tail -5 $O/sq.log; exit 1; }
timeout -s KILL 200 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/fetch -o fetch --output-format csv -- python3 -u scripts/scan_prof.py 2 > $O/fetch.log 2>&1 || { tail -5 $O/fetch.log; exit 1; }
python3 - <<'PY'
import csv, glob, collections
for stem in ("sq", "fetch"):
    f = glob.glob(f"gpurun_out/r4m/{stem}/**/*counter_collection.csv", recursive=True)[0]
    agg = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
    for r in csv.DictReader(open(f)):
        if "pq_decode" not in r["Kernel_Name"]: continue
        agg[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
    ids = sorted(agg, key=int)
    for i in ids[:2]: print(stem, i, dict(agg[i]))
PY
echo done
