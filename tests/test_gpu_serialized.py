"""AggregateMeta::Serialized: the partial states as the reference serializes them.

Expected bytes are restated from the reference's state structs (FUN/aggregate_sum.rs:64-170
NumberSumState / DecimalSumState, aggregate_avg.rs:38-201 Number/DecimalAvgState,
aggregate_count.rs:152-155, aggregate_min_max_any.rs:46-56 MinMaxAnyState {Option<T>}; borsh:
little-endian fixed-width integers and floats, Option = tag byte + value) and the adaptors' flag
bytes (aggregate_null_unary_adaptor.rs:200-207, aggregate_ornull_adaptor.rs:135-163, 175-179),
filled with the ORACLE's per-group values (sum, count, min/max, has-input).  No reference test
holds borsh bytes, so the byte layout is parity-unpinned beyond that restatement;
the values are pinned by the oracle.
"""
import struct

import numpy as np
import pytest

from databend_amd import column as col
from databend_amd.aggregates import AggregateFunctionFactory
from databend_amd.aggregator import AggregateHashTable, AggregatorParams, HashTableConfig
from databend_amd.column import Column
from databend_amd.ffi import Unsupported
from tests.test_gpu_parity import oracle_aggregate

pytestmark = pytest.mark.gpu
F = AggregateFunctionFactory.instance()


def _le(v, width, signed=True):
    return int(v).to_bytes(width, "little", signed=signed)


def _expected(fn, arg, vals):
    """vals: dict with the oracle's per-group sum / count / min / max / has (has-non-NULL)."""
    t = arg.dtype if arg is not None else None
    nullable = t is not None and t.nullable
    if fn == "count":
        return _le(vals["count"], 8, False)
    if fn == "sum":
        if t.type_id == col.abi.DECIMAL128:
            b = _le(vals["sum"], 16)
        elif t.type_id in (col.abi.FLOAT32, col.abi.FLOAT64):
            b = struct.pack("<d", vals["sum"])
        elif t.type_id in (col.abi.UINT8, col.abi.UINT16, col.abi.UINT32, col.abi.UINT64):
            b = _le(vals["sum"], 8, False)
        else:
            b = _le(vals["sum"], 8)
    elif fn == "avg":
        if t.type_id == col.abi.DECIMAL128:
            b = _le(vals["sum"], 16) + _le(vals["count"], 8, False)
        elif t.type_id in (col.abi.FLOAT32, col.abi.FLOAT64):
            b = struct.pack("<d", vals["sum"]) + _le(vals["count"], 8, False)
        else:
            b = _le(vals["sum"], 8) + _le(vals["count"], 8, False)
    else:  # min / max: Option<T> in the argument's own width
        v = vals[fn]
        if v is None:
            b = b"\x00"
        elif t.type_id == col.abi.DECIMAL128:
            b = b"\x01" + _le(v, 16)
        elif t.type_id == col.abi.FLOAT64:
            b = b"\x01" + struct.pack("<d", v)
        elif t.type_id == col.abi.FLOAT32:
            b = b"\x01" + struct.pack("<f", v)
        else:
            b = b"\x01" + _le(v, t.width, t.np_dtype(0).dtype.kind == "i" if t.np_dtype else True)
    if nullable:
        b += b"\x01" if vals["has"] else b"\x00"
    return b + b"\x01"  # OrNull flag: the group received rows


@pytest.mark.parametrize("on_device", [False, True])
def test_serialized_states_match_reference_encoding(on_device):
    rng = np.random.default_rng(31)
    n = 200_000
    k = Column.from_numbers(col.Int32, rng.integers(0, 3000, n))
    i16 = Column.from_numbers(col.Int16, rng.integers(-30000, 30000, n), validity=rng.random(n) > 0.3)
    u32 = Column.from_numbers(col.UInt32, rng.integers(0, 2**32 - 1, n))
    f = Column.from_numbers(col.Float64, rng.integers(-1000, 1000, n) / 4.0)
    d = Column.from_decimals(30, 2, [int(x) * (1 << 66) + 3 for x in rng.integers(-500, 500, n)])
    # a group whose nullable argument is all NULL: MIN/MAX serialize None
    i16.validity[k.data == 7] = False
    specs = [("count", None), ("sum", i16), ("min", i16), ("max", u32), ("avg", f), ("sum", d), ("min", d),
             ("avg", i16), ("count", i16)]
    fns = [F.get(fn, [], [c.dtype] if c is not None else []) for fn, c in specs]
    params = AggregatorParams([k.dtype], fns)
    ht = AggregateHashTable(params, HashTableConfig(True))
    try:
        if on_device:
            from databend_amd.device import DeviceColumn
            dk = DeviceColumn.from_host(k)
            dargs = {id(c): DeviceColumn.from_host(c) for _, c in specs if c is not None}
            ht.add_groups([dk], [None if c is None else dargs[id(c)] for _, c in specs], on_device=True)
        else:
            ht.add_groups([k], [c for _, c in specs])
        blk = ht.result_serialized()
    finally:
        ht.close()
    ns = len(specs)
    keys = blk.columns[ns].data
    # oracle per-group values: count(x), min, max (and sum) of each argument
    for j, (fn, c) in enumerate(specs):
        aggs = [("count", None)] if c is None else \
            [("count", c), ("min", c), ("max", c)] + ([("sum", c)] if fn in ("sum", "avg") else [])
        ok, oa = oracle_aggregate([k], aggs, threads=8)
        order = {int(x): i for i, x in enumerate(ok[0].data)}
        vals_cols = [a.values() for a in oa]
        got = blk.columns[j]
        for g, key in enumerate(keys):
            i = order[int(key)]
            raw = bytes(got.data[int(got.offsets[g]):int(got.offsets[g + 1])])
            if c is None:
                vals = {"count": vals_cols[0][i]}
            else:
                cnt, mn, mx = vals_cols[0][i], vals_cols[1][i], vals_cols[2][i]
                vals = {"count": cnt, "min": mn, "max": mx, "has": cnt > 0}
                if fn in ("sum", "avg"):
                    s = vals_cols[3][i]
                    vals["sum"] = 0 if s is None else s
            exp = _expected(fn, c, vals)
            assert raw == exp, f"agg {j} ({fn}) group {key}: {raw.hex()} != {exp.hex()}"


def test_serialized_rejects_sql_avg():
    k = Column.from_numbers(col.Int32, np.arange(10) % 3)
    v = Column.from_numbers(col.Int64, np.arange(10))
    params = AggregatorParams([k.dtype], [F.get("sql_avg", [], [v.dtype])])
    ht = AggregateHashTable(params, HashTableConfig(True))
    try:
        ht.add_groups([k], [v])
        with pytest.raises(Unsupported):
            ht.result_serialized()
    finally:
        ht.close()
