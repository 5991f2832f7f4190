"""The direct table stage of the radix-partitioned COUNT(*) insert (part.hip
part_slice_direct_kernel): in recycle mode, reset -> add_groups(on device) -> finalize_into writes
every slice's groups straight into the result columns (the HBM table is never written).  Checked
against numpy's unique counts (the same GROUP BY key, COUNT(*) the oracle restates), for every key
width, the all-ones key (the table's sentinel slot), a slice holding more keys than its slots and
result columns too short (both replay the table path from the same sorted keys), a second batch
before the finalize (the held-back stage runs as the regular slices) and an abandoned batch."""
import ctypes as C

import numpy as np
import pytest

from databend_amd import abi, ffi
from databend_amd import column as col
from databend_amd.aggregates import AggregateFunctionFactory
from databend_amd.aggregator import AggregateHashTable, AggregatorParams, HashTableConfig
from databend_amd.column import Column
from databend_amd.device import DeviceColumn
from databend_amd.ffi import check, lib
from databend_amd.workloads import _dev_to_host, _OutSet

pytestmark = pytest.mark.gpu
F = AggregateFunctionFactory.instance()
M64 = (1 << 64) - 1


def slot_unmix(y: int) -> int:
    """agg.hpp slot_unmix: the inverse of slot_mix (the slot placement of inline keys)."""
    ci = pow(0xD6E8FEB86659FD93, -1, 1 << 64)
    y ^= y >> 32
    y = (y * ci) & M64
    y ^= y >> 32
    y = (y * ci) & M64
    y ^= y >> 32
    return y ^ 0x9E3779B97F4A7C15


class _Table:
    def __init__(self, t, hint):
        self.params = AggregatorParams([t], [F.get("count", [], [])])
        self.result_types = [f.return_type() for f in self.params.aggregate_functions]
        self.ht = AggregateHashTable(self.params, HashTableConfig(True, hint))
        check(lib().dbg_agg_set_recycle(self.ht.h, 1))
        self.out = None

    def add(self, key_col):
        check(lib().dbg_agg_add_groups(self.ht.h, (abi.dbg_column * 1)(key_col.to_abi()), None, None, len(key_col), 1))

    def finalize(self, cap):
        if self.out is None or self.out.cap != cap:
            self.out = _OutSet(self, cap, [1 << 16])
        n = C.c_uint64()
        sb = (C.c_uint64 * 1)()
        rc = lib().dbg_agg_finalize_into(self.ht.h, self.out.oa, self.out.ok, self.out.cap, self.out.scap, C.byref(n), sb)
        return rc, n.value

    def result(self, n):
        k = _dev_to_host(self.out.keys[0], n).data
        c = _dev_to_host(self.out.aggs[0], n).data
        return k, c


def _expect(vals):
    u, c = np.unique(vals, return_counts=True)
    return dict(zip(u.tolist(), c.tolist()))


def _check(tab, n, vals):
    k, c = tab.result(n)
    got = dict(zip(k.tolist(), c.tolist()))
    assert len(got) == n, "duplicate groups in the result"
    assert got == _expect(vals)


def _keys(kind, distinct, n, seed):
    rng = np.random.default_rng(seed)
    t = {"i64": col.Int64, "i32": col.Int32, "i16": col.Int16, "u8": col.UInt8}[kind]
    if kind == "i64":
        pool = rng.integers(-2**63, 2**63 - 1, distinct, dtype=np.int64)
        pool[0] = -1  # packs to the EMPTY entry: the sentinel group
    elif kind == "i32":
        pool = rng.integers(-2**31, 2**31 - 1, distinct, dtype=np.int64)
        pool[0] = -1
    elif kind == "i16":
        pool = np.arange(-2**15, 2**15, dtype=np.int64)
    else:
        pool = np.arange(0, 256, dtype=np.int64)
    vals = pool[rng.integers(0, len(pool), n)].astype(t.np_dtype)
    return t, vals


@pytest.mark.parametrize("kind,distinct,n,hint", [("i64", 600_000, 3_000_000, 1 << 20), ("i32", 400_000, 2_500_000, 1 << 20),
                                                  ("i16", 65_536, 2_000_000, 1 << 20), ("u8", 256, 1_200_000, 1 << 20),
                                                  ("i64", 700_000, 2_000_000, 1 << 26)], ids=str)
def test_direct_stage_steps(kind, distinct, n, hint):
    """Three recycled steps: the first finalize meets columns too short (replay -> the table path
    reports the count, the table intact), then every step runs the direct stage."""
    t, vals = _keys(kind, distinct, n, distinct)
    tab = _Table(t, hint)
    try:
        dev = DeviceColumn.from_host(Column.from_numbers(t, vals))
        exp_groups = len(np.unique(vals))
        check(lib().dbg_agg_reset(tab.ht.h))
        tab.add(dev)
        rc, g = tab.finalize(exp_groups // 2)
        assert rc == abi.DBG_ERR_INVALID and g == exp_groups
        rc, g = tab.finalize(exp_groups + 10)  # the table was kept: finalize again
        check(rc)
        _check(tab, g, vals)
        for step in range(2):
            check(lib().dbg_agg_reset(tab.ht.h))
            tab.add(dev)
            ffi.prof_reset()
            ffi.prof_enable(True)
            rc, g = tab.finalize(exp_groups + 10)
            ffi.prof_enable(False)
            assert "part_direct" in ffi.prof_read(), "the direct stage did not run"
            check(rc)
            _check(tab, g, vals)
            # recycled: the handle is empty again
            rc, g0 = tab.finalize(exp_groups + 10)
            check(rc)
            assert g0 == 0
    finally:
        tab.ht.close()


def test_direct_stage_full_slice_replays():
    """More distinct keys in one 4096-slot slice than it has slots: the direct stage gives up, the
    regular slices (overflow records + fixup) from the same sorted keys produce the result."""
    rng = np.random.default_rng(7)
    tab = _Table(col.Int64, 1 << 19)
    try:
        cap = C.c_uint64()
        check(lib().dbg_agg_capacity(tab.ht.h, C.byref(cap)))
        lg = cap.value.bit_length() - 1
        assert cap.value == 1 << lg and lg >= 20
        hi = rng.integers(1, 1 << (63 - lg), 5000, dtype=np.int64)
        # slot_mix(key) & (cap - 1) = i % 4096: every crowded key in slice 0
        crowd = np.array([slot_unmix((int(h) << lg) | int(i % 4096)) for i, h in enumerate(hi)], dtype=np.uint64).view(np.int64)
        other = rng.integers(-2**63, 2**63 - 1, 200_000, dtype=np.int64)
        pool = np.concatenate([crowd, other])
        vals = pool[rng.integers(0, len(pool), 1 << 21)]
        vals[: len(crowd)] = crowd  # every crowded key present
        dev = DeviceColumn.from_host(Column.from_numbers(col.Int64, vals))
        check(lib().dbg_agg_reset(tab.ht.h))
        tab.add(dev)
        cap2 = C.c_uint64()
        check(lib().dbg_agg_capacity(tab.ht.h, C.byref(cap2)))
        assert cap2.value == cap.value
        rc, g = tab.finalize(len(np.unique(vals)) + 10)
        check(rc)
        _check(tab, g, vals)
    finally:
        tab.ht.close()


def test_direct_stage_held_back_then_flushed():
    """A second batch before the finalize runs the first batch's held-back stage as the regular
    slices; a reset discards a held-back stage."""
    t, v1 = _keys("i64", 300_000, 1_500_000, 11)
    _, v2 = _keys("i64", 300_000, 1_200_000, 12)
    tab = _Table(t, 1 << 20)
    try:
        d1 = DeviceColumn.from_host(Column.from_numbers(t, v1))
        d2 = DeviceColumn.from_host(Column.from_numbers(t, v2))
        check(lib().dbg_agg_reset(tab.ht.h))
        tab.add(d1)
        tab.add(d2)
        allv = np.concatenate([v1, v2])
        rc, g = tab.finalize(len(np.unique(allv)) + 10)
        check(rc)
        _check(tab, g, allv)
        check(lib().dbg_agg_reset(tab.ht.h))
        tab.add(d1)  # abandoned
        check(lib().dbg_agg_reset(tab.ht.h))
        tab.add(d2)
        rc, g = tab.finalize(len(np.unique(allv)) + 10)
        check(rc)
        _check(tab, g, v2)
    finally:
        tab.ht.close()
