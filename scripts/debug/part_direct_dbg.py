"""Diagnostics for the direct table stage: which scopes each call launches."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np
from databend_amd import ffi, abi
from databend_amd.ffi import check, lib
from tests.test_gpu_part_direct import _Table, _keys
from databend_amd.column import Column
from databend_amd.device import DeviceColumn
import ctypes as C

t, vals = _keys("i64", 600_000, 3_000_000, 600_000)
tab = _Table(t, 1 << 20)
dev = DeviceColumn.from_host(Column.from_numbers(t, vals))
exp = len(np.unique(vals))
cap = C.c_uint64()
def run(label, fn):
    ffi.prof_reset(); ffi.prof_enable(True)
    r = fn()
    ffi.prof_enable(False)
    check(lib().dbg_agg_capacity(tab.ht.h, C.byref(cap)))
    print(label, r, "cap", cap.value, {k: v[1] for k, v in ffi.prof_read().items()}, flush=True)
run("reset", lambda: lib().dbg_agg_reset(tab.ht.h))
run("add", lambda: tab.add(dev))
run("fin1024", lambda: tab.finalize(1024))
run("fin", lambda: tab.finalize(exp + 10))
for s in range(2):
    run("reset", lambda: lib().dbg_agg_reset(tab.ht.h))
    run("add", lambda: tab.add(dev))
    run("fin", lambda: tab.finalize(exp + 10))
    run("fin-again", lambda: tab.finalize(exp + 10))
