#!/bin/bash
# round 4 (n): first-batch table pre-sizing (C3 / C5 first steps) + parity; scan numbers
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r4n; mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_compact.py tests/test_gpu_pipeline.py > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python -u - > $O/first.json 2> $O/first.err <<'PY' || { tail -5 $O/first.err; exit 1; }
import json, time, torch
from databend_amd import ffi
from databend_amd.workloads import DEFAULT_ROWS, ConfigRunner
out = {}
for cfg in (3, 5):
    r = ConfigRunner(cfg, DEFAULT_ROWS[cfg], copies=1)
    torch.cuda.synchronize()
    ts = []
    for k in range(3):
        t0 = time.perf_counter(); r.step(0); torch.cuda.synchronize(); ts.append((time.perf_counter() - t0) * 1e3)
    out[f"C{cfg}"] = {"first_steps_ms": ts, "groups": r.n_groups}
    r.close() if hasattr(r, "close") else None
    del r
print(json.dumps(out))
PY
cat $O/first.json
timeout -k 10 300 python -u scripts/scan_prof.py 10 > $O/scan.json 2> $O/scan.err || { tail -5 $O/scan.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/scan.json'))
for k in ['none','snappy','zstd']: print(k, {x:d[k][x] for x in ['pages','ms_per_chunk','frac','kernel_ms_per_chunk','kernel_frac']})"
echo done
