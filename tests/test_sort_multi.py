"""ORDER BY several columns / String / Decimal128 LIMIT k: the oracle pinned by the reference's own
sort test, an independent Python restatement, and the device path (dbg_sort_limit_multi through
databend_amd.sort) against the oracle.

Golden: src/query/expression/tests/it/sort.rs:32-104 (test_block_sort): block
(Int64 [6, 4, 3, 2, 1, 1, 7], String b1..b7); `ORDER BY c1 DESC` over the strings gives
b7 b6 b5 b4 b3 b2 b1 (:67-80), `ORDER BY c0 ASC, c1 DESC` gives b6 b5 b4 b3 b2 b1 b7 (:81-101),
and the Decimal128 block with the same values (:106-140) sorts like the Int64 one.  Rows equal on
every sort column: the reference's unstable sort leaves their order open; this build and its
oracle emit them in ascending row order, and the parity bar is exact index equality.
"""
import numpy as np
import pytest

from databend_amd import column as col
from databend_amd.column import Column
from oracle import oracle

INTS = [6, 4, 3, 2, 1, 1, 7]
STRS = ["b1", "b2", "b3", "b4", "b5", "b6", "b7"]


def test_oracle_reference_golden():
    a = Column.from_numbers(col.Int64, INTS)
    s = Column.from_strings(STRS)
    d = Column.from_decimals(10, 0, INTS)
    assert oracle.sort_multi_limit_indices([s], [False], [False], None).tolist() == [6, 5, 4, 3, 2, 1, 0]
    assert oracle.sort_multi_limit_indices([a, s], [True, False], [False, False], None).tolist() == [5, 4, 3, 2, 1, 0, 6]
    assert oracle.sort_multi_limit_indices([d], [True], [False], None).tolist() == [4, 5, 3, 2, 1, 0, 6]
    assert oracle.sort_multi_limit_indices([d], [True], [False], 4).tolist() == [4, 5, 3, 2]


def _py_multi(rows, asc, nulls_first, limit):
    """Independent restatement: Python's sorted over per-row tuples (rows: list of per-column
    (valid, python value) pairs; values compare by Python order: ints, bytes, floats by total
    order key)."""
    def colkey(v, a, nf):
        valid, x = v
        if not valid:
            return (0 if nf else 2, 0)
        return (1, x if a else _Neg(x))

    order = sorted(range(len(rows)), key=lambda i: tuple(colkey(v, a, nf) for v, a, nf in zip(rows[i], asc, nulls_first)) + (i,))
    return order if limit is None else order[:limit]


class _Neg:
    __slots__ = ("x",)

    def __init__(self, x):
        self.x = x

    def __lt__(self, o):
        return o.x < self.x

    def __eq__(self, o):
        return self.x == o.x


def _total(f):
    b = int(np.float64(f).view(np.uint64))
    return (~b) & ((1 << 64) - 1) if b >> 63 else b | (1 << 63)


def _rand_block(rng, n):
    """(Int32 few values, nullable String with shared prefixes / embedded zeros / empty,
    nullable Decimal128 beyond 64 bits, Float64 with NaN / -0.0)."""
    i = rng.integers(0, 4, n).astype(np.int32)
    base = [b"", b"a", b"ab", b"ab\x00", b"abc", b"b", b"abcdefgh", b"abcdefghi", b"abcdefgh\x00", b"zz" * 20]
    sv = [base[j] if j < len(base) else (b"k%05d" % j) for j in rng.integers(0, 40, n)]
    svalid = rng.random(n) < 0.85
    dv = [int(x) * (10 ** 20) + int(y) for x, y in zip(rng.integers(-5, 5, n), rng.integers(0, 3, n))]
    dvalid = rng.random(n) < 0.9
    fv = rng.integers(-3, 3, n).astype(np.float64)
    if n >= 4:
        fv[:4] = [np.nan, -0.0, 0.0, -np.inf]
    cols = [Column.from_numbers(col.Int32, i), Column.from_strings(sv, validity=svalid),
            Column.from_decimals(38, 2, dv, validity=dvalid), Column.from_numbers(col.Float64, fv)]
    pyrows = [[(True, int(i[r])), (bool(svalid[r]), sv[r]), (bool(dvalid[r]), dv[r]), (True, _total(fv[r]))] for r in range(n)]
    return cols, pyrows


@pytest.mark.parametrize("seed", [1, 2])
def test_oracle_matches_python_restatement(seed):
    rng = np.random.default_rng(seed)
    n = 3000
    cols, pyrows = _rand_block(rng, n)
    for idx, asc, nf, limit in [((0, 1), (True, False), (False, True), None), ((1, 2, 3), (False, True, False), (True, False, True), 50),
                                ((3, 0), (False, False), (False, False), 7), ((2,), (True,), (True,), None)]:
        got = oracle.sort_multi_limit_indices([cols[j] for j in idx], asc, nf, limit).tolist()
        exp = _py_multi([[r[j] for j in idx] for r in pyrows], asc, nf, limit)
        assert got == exp, (idx, asc, nf, limit)


# ---------------------------------------------------------------- device path
def _dev(c):
    from databend_amd.device import DeviceColumn
    return DeviceColumn.from_host(c)


@pytest.mark.gpu
def test_device_reference_golden():
    from databend_amd.sort import SortColumnDescription, sort, sort_multi_limit_indices
    a, s = _dev(Column.from_numbers(col.Int64, INTS)), _dev(Column.from_strings(STRS))
    assert sort_multi_limit_indices([a, s], [SortColumnDescription(1, asc=False)], None).cpu().tolist() == [6, 5, 4, 3, 2, 1, 0]
    descs = [SortColumnDescription(0, asc=True), SortColumnDescription(1, asc=False)]
    assert sort_multi_limit_indices([a, s], descs, None).cpu().tolist() == [5, 4, 3, 2, 1, 0, 6]
    out = sort([a, s], descs, 3)
    assert out[0].to_host().data.tolist() == [1, 1, 2]
    d = _dev(Column.from_decimals(10, 0, INTS))
    assert sort_multi_limit_indices([d], [SortColumnDescription(0)], 4).cpu().tolist() == [4, 5, 3, 2]


MULTI = [  # (columns, asc, nulls_first, rows, limit)
    ((0, 1), (True, False), (False, True), 1500, None),      # every row a candidate
    ((0, 1), (True, False), (False, True), 200_000, 10),
    ((1,), (True,), (False,), 200_000, 2048),                # one String column
    ((1,), (False,), (True,), 50_000, 100),
    ((2,), (False,), (False,), 100_000, 37),                 # Decimal128 beyond 64 bits
    ((0, 2, 3), (False, True, False), (True, True, False), 300_000, 500),
    ((3, 1, 0), (True, True, True), (False, False, False), 100_000, 1),
    ((0,), (True,), (False,), 100_000, 2048),                # heavy ties -> row index levels
    ((0, 3), (True, True), (False, False), 0, 10),
]


@pytest.mark.gpu
@pytest.mark.parametrize("idx,asc,nf,n,limit", MULTI)
def test_device_matches_oracle(idx, asc, nf, n, limit):
    from databend_amd.sort import SortColumnDescription, sort_multi_limit_indices
    rng = np.random.default_rng(n + (limit or 0))
    cols, _ = _rand_block(rng, n)
    dev = [_dev(c) for c in cols]
    descs = [SortColumnDescription(j, asc=a, nulls_first=f) for j, a, f in zip(idx, asc, nf)]
    got = sort_multi_limit_indices(dev, descs, limit).cpu().numpy().astype(np.int64)
    exp = oracle.sort_multi_limit_indices([cols[j] for j in idx], asc, nf, limit)
    assert got.tolist() == exp.tolist()


@pytest.mark.gpu
def test_device_long_strings_and_unsupported():
    from databend_amd.ffi import Unsupported
    from databend_amd.sort import SortColumnDescription, sort_multi_limit_indices
    rng = np.random.default_rng(5)
    n = 20_000
    # URL-like strings sharing a 60-byte prefix: the select needs several key words
    sv = [b"https://example.com/some/long/common/prefix/for/every/row/" + b"%d" % x for x in rng.integers(0, 3000, n)]
    c = Column.from_strings(sv)
    k = Column.from_numbers(col.UInt64, rng.integers(0, 5, n).astype(np.uint64))
    dev = [_dev(k), _dev(c)]
    descs = [SortColumnDescription(0, asc=False), SortColumnDescription(1, asc=True)]
    got = sort_multi_limit_indices(dev, descs, 25).cpu().numpy().astype(np.int64)
    assert got.tolist() == oracle.sort_multi_limit_indices([k, c], [False, True], [False, False], 25).tolist()
    with pytest.raises(Unsupported):
        sort_multi_limit_indices(dev, descs, 4096)
