"""Host-side timing of one step's C-ABI calls (reset / add_groups / finalize_into) for any config,
beside the HIP-event kernel sum of the same steps: where a step's host gaps come from.

    python scripts/step_timing_cfg.py <cfg> [steps]
"""
import ctypes as C
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

from databend_amd import ffi  # noqa: E402
from databend_amd.ffi import check, lib  # noqa: E402
from databend_amd.workloads import DEFAULT_ROWS, ConfigRunner  # noqa: E402

cfg = int(sys.argv[1])
K = int(sys.argv[2]) if len(sys.argv) > 2 else 5
r = ConfigRunner(cfg, DEFAULT_ROWS[cfg], copies=1)
L = lib()
h = r.table.h
for k in range(2):
    r.step(k)
torch.cuda.synchronize()
T = {"reset": 0.0, "add": 0.0, "fin": 0.0}
t00 = time.perf_counter()
for k in range(K):
    keys, args, fp = r._prepared(0)
    t0 = time.perf_counter()
    check(L.dbg_agg_reset(h))
    t1 = time.perf_counter()
    check(L.dbg_agg_add_groups(h, keys, args, fp, r.rows, 1))
    t2 = time.perf_counter()
    r.finalize_into(h)
    t3 = time.perf_counter()
    T["reset"] += t1 - t0
    T["add"] += t2 - t1
    T["fin"] += t3 - t2
torch.cuda.synchronize()
tot = time.perf_counter() - t00
ffi.prof_reset()
ffi.prof_enable(True)
for k in range(K):
    r.step(k)
torch.cuda.synchronize()
ffi.prof_enable(False)
prof = ffi.prof_read()
print(json.dumps({"cfg": cfg, "host_ms_per_call": {k: round(v / K * 1e3, 3) for k, v in T.items()},
                  "ms_per_step": round(tot / K * 1e3, 3),
                  "kernel_ms_per_step": {k: round(v[0] / K, 3) for k, v in prof.items()},
                  "kernel_sum_ms": round(sum(v[0] for v in prof.values()) / K, 3)}))
r.close()
