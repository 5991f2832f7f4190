"""The fused insert + finalize launch for COUNT(*) over a <= 16-bit key (ClickBench Q8 shape) and its
direct-mapped hand-off (agg.hip fused_dense): every workgroup adds its LDS counts into a dense
array indexed by the key, the last one finalizes from it.  Against the oracle: Int8 / UInt8 /
Int16 / UInt16 keys with negative values and full ranges, several predicates, consecutive steps
on one recycled table (the dense arrays must be clean again after every launch), a key count
larger than the table's view (overflow records, the host's grow-and-finalize-again protocol),
and the parked-row chain (DBG_X_DENSE=0 semantics: a table that is not empty at launch start)."""
import ctypes as C

import numpy as np
import pytest

from databend_amd import abi
from databend_amd import column as col
from databend_amd.aggregates import AggregateFunctionFactory
from databend_amd.aggregator import AggregateHashTable, AggregatorParams, HashTableConfig
from databend_amd.column import Column, abi_array
from databend_amd.device import DeviceColumn, empty
from databend_amd.ffi import check, lib
from databend_amd.filter import FilterProgram, cmp
from tests.parity import assert_results_equal
from tests.test_gpu_parity import oracle_aggregate

pytestmark = pytest.mark.gpu
F = AggregateFunctionFactory.instance()


class FusedRunner:
    """reset -> add_groups (device, deferred) -> finalize_into: the fused launch."""

    def __init__(self, ktype):
        self.ktype = ktype
        self.params = AggregatorParams([ktype], [F.get("count")])
        self.table = AggregateHashTable(self.params, HashTableConfig(True))
        check(lib().dbg_agg_set_recycle(self.table.h, 1))
        self.cap = 1024

    def step(self, key: Column, pred=None):
        import torch
        dk = DeviceColumn.from_host(key)
        n = len(key)
        keys = abi_array([dk.to_abi()])
        a = abi.dbg_column()
        a.dt = abi.dbg_datatype(-1, 0, 0, 0, 0)
        args = abi_array([a])
        fp = FilterProgram(cmp(0, pred[0], pred[1]), [dk]) if pred else None
        L = lib()
        check(L.dbg_agg_reset(self.table.h))
        check(L.dbg_agg_add_groups(self.table.h, keys, args, fp.ptr() if fp else None, n, 1))
        ng = C.c_uint64()
        sb = (C.c_uint64 * 1)()
        for _ in range(3):
            ka, ca = empty(self.ktype, self.cap), empty(col.UInt64, self.cap)
            ok = (abi.dbg_out_column * 1)()
            oa = (abi.dbg_out_column * 1)()
            ok[0].data = ka.data.data_ptr()
            oa[0].data = ca.data.data_ptr()
            scap = (C.c_uint64 * 1)(0)
            rc = L.dbg_agg_finalize_into(self.table.h, oa, ok, self.cap, scap, C.byref(ng), sb)
            if rc == abi.DBG_ERR_INVALID and ng.value > self.cap:
                self.cap = int(ng.value * 1.25) + 1
                continue
            check(rc)
            break
        torch.cuda.synchronize()
        m = ng.value
        kh = Column(self.ktype, ka.data[: m * self.ktype.width].cpu().numpy().view(self.ktype.np_dtype).copy())
        ch = Column(col.UInt64, ca.data[: m * 8].cpu().numpy().view(np.uint64).copy())
        return [kh], [ch]

    def close(self):
        self.table.close()


KEYS = [(col.Int8, -128, 128), (col.UInt8, 0, 256), (col.Int16, -32768, 32768), (col.UInt16, 0, 65536)]


@pytest.mark.parametrize("t,lo,hi", KEYS, ids=lambda x: repr(x))
def test_fused_dense_matches_oracle(t, lo, hi):
    rng = np.random.default_rng(abs(hash(repr(t))) % 2**32)
    r = FusedRunner(t)
    try:
        for step, (n, distinct, pred) in enumerate([(3_000_001, 33, ("<>", 0)), (2_000_000, 200, None),
                                                      (4_000_000, 17, (">", 5)), (1_000_000, 33, ("<>", 0))]):
            pool = rng.integers(lo, hi, distinct)
            pool[0] = 0
            pool[-1] = hi - 1  # the largest raw key (all-ones bits for the unsigned types)
            vals = np.where(rng.random(n) < 0.6, 0, pool[rng.integers(0, distinct, n)])
            key = Column.from_numbers(t, vals.astype(t.np_dtype))
            gk, ga = r.step(key, pred)
            filt = (cmp(0, pred[0], pred[1]), [key]) if pred else None
            ok, oa = oracle_aggregate([key], [("count", None)], filt)
            assert_results_equal(gk, ga, ok, oa)
    finally:
        r.close()


def test_fused_dense_many_keys_overflow_view():
    """30,000 distinct Int16 keys into a table sized for ~1,000: keys the LDS view cannot place
    become overflow records; the host grows the table and finalizes again — exact counts, and
    the next step on the same table is exact too (dense arrays cleaned)."""
    rng = np.random.default_rng(5)
    r = FusedRunner(col.Int16)
    try:
        for n, distinct in ((5_000_000, 30_000), (2_000_000, 40)):
            pool = rng.choice(np.arange(-32768, 32768), distinct, replace=False)
            key = Column.from_numbers(col.Int16, pool[rng.integers(0, distinct, n)].astype(np.int16))
            gk, ga = r.step(key)
            ok, oa = oracle_aggregate([key], [("count", None)])
            assert_results_equal(gk, ga, ok, oa)
    finally:
        r.close()
