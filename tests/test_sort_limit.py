"""ORDER BY one column LIMIT k: the oracle pinned by the reference's own sort test, and the
device path (dbg_sort_limit_indices through databend_amd.sort) against the oracle.

Golden: src/query/expression/tests/it/sort.rs:32-104 (test_block_sort; Int64 column
[6, 4, 3, 2, 1, 1, 7], ASC, no limit and LIMIT 4 — the expected companion string column b1..b7
fixes the row indices).  Equal values: the reference leaves their order unspecified
(select_nth_unstable_by); this build and its oracle emit them in ascending row order, and the
parity bar below is exact index equality with that rule plus equality of the value sequence.
"""
import numpy as np
import pytest

from databend_amd import abi
from databend_amd import column as col
from databend_amd.column import Column
from oracle import oracle

GOLDEN = [6, 4, 3, 2, 1, 1, 7]


def test_oracle_reference_golden():
    c = Column.from_numbers(col.Int64, GOLDEN)
    # expected strings b5 b6 b4 b3 b2 b1 b7 -> rows 4 5 3 2 1 0 6 (sort.rs:49-54)
    assert oracle.sort_limit_indices(c, True, False, None).tolist() == [4, 5, 3, 2, 1, 0, 6]
    # LIMIT 4 -> b5 b6 b4 b3 (sort.rs:62-65)
    assert oracle.sort_limit_indices(c, True, False, 4).tolist() == [4, 5, 3, 2]


def _py_sort(values, valid, asc, nulls_first, limit):
    """Independent restatement with Python's sorted (common.rs:95-174; floats via totalOrder)."""
    import struct

    def tkey(x):
        if isinstance(x, float):
            b = struct.unpack("<q", struct.pack("<d", x))[0]
            return b ^ ((b >> 63) & 0x7FFFFFFFFFFFFFFF)  # array/ord.rs:48-56
        return int(x)

    n = len(values)
    nulls = [i for i in range(n) if not valid[i]]
    vals = [i for i in range(n) if valid[i]]
    vals.sort(key=lambda i: (tkey(values[i]) * (1 if asc else -1), i))
    order = nulls + vals if nulls_first else vals + nulls
    return order[: n if limit is None else min(limit, n)]


@pytest.mark.parametrize("asc", [True, False])
@pytest.mark.parametrize("nulls_first", [True, False])
@pytest.mark.parametrize("kind", ["i64", "u64", "f64", "i16"])
def test_oracle_matches_python_restatement(asc, nulls_first, kind):
    rng = np.random.default_rng(7)
    n = 300
    if kind == "f64":
        v = rng.normal(size=n)
        v[:6] = [np.nan, -np.nan, 0.0, -0.0, np.inf, -np.inf]
        dt = col.Float64
    elif kind == "u64":
        v = rng.integers(0, 2**64 - 1, n, dtype=np.uint64)
        v[:3] = [0, 2**64 - 1, 2**63]
        dt = col.UInt64
    elif kind == "i16":
        v = rng.integers(-5, 5, n).astype(np.int16)
        dt = col.Int16
    else:
        v = rng.integers(-2**63, 2**63 - 1, n, dtype=np.int64)
        v[:3] = [-2**63, 2**63 - 1, 0]
        dt = col.Int64
    valid = rng.random(n) < 0.8
    c = Column.from_numbers(dt, v, valid)
    pyv = [float(x) if kind == "f64" else int(x) for x in v]
    for limit in (None, 0, 1, 10, 299, 1000):
        got = oracle.sort_limit_indices(c, asc, nulls_first, limit).tolist()
        assert got == _py_sort(pyv, valid, asc, nulls_first, limit), (limit,)


# ---------------------------------------------------------------- device path
def _dev(c):
    from databend_amd.device import DeviceColumn
    return DeviceColumn.from_host(c)


@pytest.mark.gpu
def test_device_reference_golden():
    from databend_amd.sort import sort_limit_indices
    d = _dev(Column.from_numbers(col.Int64, GOLDEN))
    assert sort_limit_indices(d, True, False, None).cpu().tolist() == [4, 5, 3, 2, 1, 0, 6]
    assert sort_limit_indices(d, True, False, 4).cpu().tolist() == [4, 5, 3, 2]


CASES = [
    ("i64", 1000, 10), ("i64", 100000, 2048), ("u64", 50000, 100), ("i32", 70000, 1000),
    ("i16", 100000, 10), ("u8", 5000, 2048), ("f64", 100000, 37), ("f32", 30000, 500),
    ("date", 20000, 10), ("timestamp", 20000, 10), ("i64", 0, 10), ("i64", 5, 10), ("u64", 3000000, 10),
]


def _make(kind, n, seed):
    rng = np.random.default_rng(seed)
    if kind == "f64":
        v = rng.normal(size=n).round(2)  # many ties
        if n >= 6:
            v[:6] = [np.nan, -np.nan, 0.0, -0.0, np.inf, -np.inf]
        return Column.from_numbers(col.Float64, v)
    if kind == "f32":
        return Column.from_numbers(col.Float32, rng.normal(size=n).astype(np.float32).round(1))
    dts = {"i64": col.Int64, "u64": col.UInt64, "i32": col.Int32, "i16": col.Int16, "u8": col.UInt8,
           "date": col.Date, "timestamp": col.Timestamp}
    dt = dts[kind]
    info = np.iinfo(dt.np_dtype)
    hi = min(int(info.max), 1000) if kind in ("i16", "u8") else int(info.max)
    v = rng.integers(int(info.min), hi, n, dtype=dt.np_dtype, endpoint=True)
    if kind == "u64" and n > 10:  # COUNT-like: few distinct values, heavy ties
        v = rng.integers(1, 50, n).astype(np.uint64)
    return Column.from_numbers(dt, v)


@pytest.mark.gpu
@pytest.mark.parametrize("kind,n,limit", CASES)
@pytest.mark.parametrize("asc", [True, False])
def test_device_matches_oracle(kind, n, limit, asc):
    from databend_amd.sort import sort_limit_indices
    c = _make(kind, n, n + limit)
    d = _dev(c)
    for nullable in (False, True):
        cc = c
        dd = d
        if nullable:
            valid = np.random.default_rng(n).random(n) < 0.9
            cc = Column(c.dtype.wrap_nullable(), c.data, None, valid)
            dd = _dev(cc)
        for nf in (False, True):
            got = sort_limit_indices(dd, asc, nf, limit).cpu().numpy().astype(np.int64)
            exp = oracle.sort_limit_indices(cc, asc, nf, limit)
            assert got.tolist() == exp.tolist(), (kind, n, limit, asc, nullable, nf)


@pytest.mark.gpu
def test_device_sort_block_and_unsupported():
    from databend_amd.ffi import Unsupported
    from databend_amd.sort import SortColumnDescription, sort, sort_limit_indices
    cnt = Column.from_numbers(col.UInt64, [5, 9, 1, 9, 3])
    key = Column.from_numbers(col.Int16, [10, 20, 30, 40, 50])
    out = sort([_dev(cnt), _dev(key)], [SortColumnDescription(0, asc=False)], 3)
    assert out[0].to_host().data.tolist() == [9, 9, 5]
    assert out[1].to_host().data.tolist() == [20, 40, 10]
    big = _dev(Column.from_numbers(col.UInt64, np.arange(5000, dtype=np.uint64)))
    with pytest.raises(Unsupported):
        sort_limit_indices(big, True, False, 4096)
    with pytest.raises(Unsupported):
        sort_limit_indices(_dev(Column.from_strings(["a", "b"])), True, False, 1)
