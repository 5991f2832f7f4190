#!/bin/bash
# round 4 (j): parquet parity (vectorised required PLAIN decode, Zstd) + the default bench line
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r4j; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parquet.py > $O/pytest_pq.log 2>&1 || { tail -40 $O/pytest_pq.log; exit 1; }
tail -2 $O/pytest_pq.log
timeout -k 10 900 python -u bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -20 $O/bench_default.err; exit 1; }
python - <<'PY'
import json
d=json.load(open("gpurun_out/r4j/bench_default.json"))
print("C2", d["value"], d["ms_per_step"], d["roofline"]["frac"])
for k,v in d.get("configs",{}).items(): print(k, v.get("ms_per_step"), v.get("roofline",{}).get("frac"))
print("scan", json.dumps(d.get("scan"))[:800])
PY
echo done
