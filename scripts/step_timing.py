"""Host-side timing of one C2 step's C-ABI calls (reset / add_groups / finalize_into)."""
import os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import ctypes as C
import torch
from databend_amd.workloads import ConfigRunner
from databend_amd.ffi import lib, check
from databend_amd import abi

r = ConfigRunner(2, 100_000_000, copies=4)
L = lib(); h = r.table.h
for k in range(10): r.step(k)
torch.cuda.synchronize()
T = {"reset": 0.0, "add": 0.0, "fin": 0.0}
n = C.c_uint64(); sb = (C.c_uint64 * 1)()
K = 200
t00 = time.perf_counter()
for k in range(K):
    keys, args, fp = r._prepared(k % 4)
    t0 = time.perf_counter(); check(L.dbg_agg_reset(h)); t1 = time.perf_counter()
    check(L.dbg_agg_add_groups(h, keys, args, fp, r.rows, 1)); t2 = time.perf_counter()
    oa, ok, cap, scap = r._out_structs
    check(L.dbg_agg_finalize_into(h, oa, ok, cap, scap, C.byref(n), sb)); t3 = time.perf_counter()
    T["reset"] += t1 - t0; T["add"] += t2 - t1; T["fin"] += t3 - t2
tot = time.perf_counter() - t00
print({k: round(v / K * 1e6, 1) for k, v in T.items()}, "us/step total", round(tot / K * 1e6, 1))
