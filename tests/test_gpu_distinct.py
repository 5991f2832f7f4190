"""DISTINCT aggregates fused with the query's other aggregates (databend_amd/distinct.py) on the
GPU, against the oracle (plain aggregates) and the Python restatement of the DISTINCT
combinator (tests/distinct_ref.py, pinned by the reference's sum_distinct goldens).

ClickBench Q10 (benchmark/clickbench/hits/queries/09.sql):
  SELECT RegionID, SUM(AdvEngineID), COUNT(*) AS c, AVG(ResolutionWidth), COUNT(DISTINCT UserID)
  FROM hits GROUP BY RegionID ORDER BY c DESC LIMIT 10
"""
import json
import os

import numpy as np
import pytest

from databend_amd import abi
from databend_amd import column as col
from databend_amd.aggregates import AggregateFunctionFactory
from databend_amd.aggregator import AggregatorParams
from databend_amd.column import Column
from databend_amd.distinct import DistinctAggregator, count_distinct
from databend_amd.ffi import Unsupported
from databend_amd.filter import FilterProgram, cmp
from tests.distinct_ref import distinct_aggregate
from tests.parity import assert_results_equal
from tests.test_gpu_parity import oracle_aggregate

pytestmark = pytest.mark.gpu
F = AggregateFunctionFactory.instance()
HERE = os.path.dirname(os.path.abspath(__file__))
GOLD = json.load(open(os.path.join(HERE, "golden", "distinct_goldens.json")))


def _run(keys, aggs, filt=None, on_device=False):
    fns = [F.get(fn, [], [c.dtype] if c is not None else []) for fn, c in aggs]
    params = AggregatorParams([k.dtype for k in keys], fns)
    args = [c for _, c in aggs]
    fcols = filt[1] if filt is not None else None
    if on_device:
        from databend_amd.device import DeviceColumn
        keys = [DeviceColumn.from_host(k) for k in keys]
        args = [None if c is None else DeviceColumn.from_host(c) for c in args]
        if fcols is not None:
            fcols = [DeviceColumn.from_host(c) for c in fcols]
    prog = FilterProgram(filt[0], fcols) if filt is not None else None
    blk = DistinctAggregator(params).run(keys, args, filter_program=prog)
    na = len(aggs)
    return blk.columns[na:], blk.columns[:na]


@pytest.mark.parametrize("case", GOLD["cases"], ids=lambda c: f"{c['fn']}({c['arg']})-{'gb' if c['grouped'] else 'one'}")
def test_distinct_goldens_gpu(case):
    from tests.test_oracle_golden import example_column
    arg = example_column(case["arg"])
    key = Column.from_numbers(col.Int64, [0, 1, 0, 1] if case["grouped"] else [0, 0, 0, 0])
    gk, ga = _run([key], [(case["fn"], arg)])
    order = np.argsort(np.asarray(gk[0].values()))
    vals = ga[0].values()
    exp = [v if ok else None for v, ok in zip(case["values"], case["validity"])]
    assert [vals[i] for i in order] == exp, case["source"]
    assert ga[0].dtype.nullable == case["nullable"]


def test_slt_count_distinct_where():
    """03_0022_select_distinct.test:21-24: count(distinct number % 3) FROM numbers(1000) WHERE
    number > 3 = 3 (no GROUP BY in the SQL: one constant group here)."""
    num = np.arange(1000, dtype=np.uint64)
    arg = Column.from_numbers(col.UInt64, num % 3)
    const = Column.from_numbers(col.UInt8, np.zeros(1000, np.uint8))
    ncol = Column.from_numbers(col.UInt64, num)
    blk = count_distinct([const], arg, cmp(0, ">", 3), [ncol])
    assert blk.columns[0].values() == [3]


def _expected_distinct(keys_col, fn, x):
    kv = keys_col.values()
    xv = x.values()
    valid = [v is not None for v in xv]
    return distinct_aggregate(kv, fn, [0 if v is None else v for v in xv], valid)


@pytest.mark.parametrize("on_device", [False, True])
def test_clickbench_q10_shape(on_device):
    rng = np.random.default_rng(10)
    n = 200_000
    region = Column.from_numbers(col.Int32, rng.integers(0, 300, n))
    adv = Column.from_numbers(col.Int16, np.where(rng.random(n) < 0.9, 0, rng.integers(1, 33, n)))
    width = Column.from_numbers(col.Int16, rng.integers(0, 2560, n))
    user = Column.from_numbers(col.Int64, rng.integers(0, 40_000, n) * 7919)
    aggs = [("sum", adv), ("count", None), ("sql_avg", width), ("count_distinct", user)]
    gk, ga = _run([region], aggs, on_device=on_device)
    ok, oa = oracle_aggregate([region], aggs[:3])
    exp = _expected_distinct(region, "count", user)
    order = {k: i for i, k in enumerate(ok[0].values())}
    cd = [exp[k] for k in ok[0].values()]
    exp_cd = Column.from_numbers(col.UInt64, cd)
    assert_results_equal(gk, ga, ok, oa + [exp_cd])
    assert len(order) == len(gk[0])


@pytest.mark.parametrize("on_device", [False, True])
def test_several_distinct_with_nulls_filter_and_strings(on_device):
    rng = np.random.default_rng(12)
    n = 60_000
    k = Column.from_strings([b"g%d" % v for v in rng.integers(0, 200, n)])
    x = Column.from_numbers(col.Int64, rng.integers(0, 50, n), validity=rng.random(n) > 0.3)
    x.validity[np.asarray(k.values(), dtype=object) == b"g7"] = False  # a group whose x is all NULL
    s = Column.from_strings([b"s%d" % v for v in rng.integers(0, 30, n)], validity=rng.random(n) > 0.2)
    d = Column.from_decimals(15, 2, [int(v) for v in rng.integers(0, 40, n) * 25])
    y = Column.from_numbers(col.Int64, rng.integers(-100, 100, n))
    p = Column.from_numbers(col.Int32, rng.integers(0, 10, n))
    aggs = [("count_distinct", x), ("sum_distinct", x), ("count", None), ("count_distinct", s), ("max_distinct", d),
            ("sum", y), ("avg_distinct", x), ("min", y)]
    filt = (cmp(0, "<>", 3), [p])
    gk, ga = _run([k], aggs, filt=filt, on_device=on_device)
    sel = np.asarray(p.data) != 3
    from tests.test_gpu_parity import slice_col  # noqa: F401
    idx = np.nonzero(sel)[0]

    def take(c):
        vals = c.values()
        return [vals[i] for i in idx]

    kv = take(k)
    got = {kk: i for i, kk in enumerate(gk[0].values())}
    assert len(got) == len(set(kv))
    for j, (fn, c) in enumerate(aggs):
        if not fn.endswith("_distinct"):
            continue
        xs = take(c)
        exp = distinct_aggregate(kv, fn[: -len("_distinct")], [0 if v is None else v for v in xs],
                                 [v is not None for v in xs])
        vals = ga[j].values()
        for kk, i in got.items():
            e, g = exp[kk], vals[i]
            if isinstance(e, float):
                assert g is not None and abs(g - e) <= 1e-12 * abs(e), (fn, kk, g, e)
            else:
                assert g == e, (fn, kk, g, e)
    # the plain aggregates against the oracle on the filtered rows
    ok, oa = oracle_aggregate([k], [a for a in aggs if not a[0].endswith("_distinct")], filt=filt)
    plain = [ga[j] for j, a in enumerate(aggs) if not a[0].endswith("_distinct")]
    assert_results_equal(gk, plain, ok, oa)
    if b"g7" in got:  # all-NULL x: count 0, sum NULL
        assert ga[0].values()[got[b"g7"]] == 0 and ga[1].values()[got[b"g7"]] is None


def test_distinct_without_keys_is_unsupported():
    params = AggregatorParams([], [F.get("count_distinct", [], [col.Int64])])
    with pytest.raises(Unsupported):
        DistinctAggregator(params)


@pytest.mark.parametrize("mixed_bits", [False, True])
def test_distinct_through_partial_bucket_final(mixed_bits):
    """DISTINCT inside the processors (AGG/transform_aggregate_partial.rs:146-155 forces the max
    radix bits; the combinator's set travels with its group): two partials over host blocks, each
    with the main table and a pair table per distinct aggregate; TransformPartitionBucket aligns
    (mixed_bits: one partial written at fewer buckets, re-exported pairs bucketed by the group
    keys alone); TransformFinalAggregate merges T and dedupes the pairs across partials per bucket.
    Every bucket holds only its own groups; the union equals the single-node DistinctAggregator
    and the Python restatement of the combinator."""
    from databend_amd.aggregator import (DataBlock, HashTableConfig, TransformFinalAggregate, TransformPartialAggregate,
                                         TransformPartitionBucket)
    from oracle import oracle
    from tests.test_gpu_parity import slice_col
    rng = np.random.default_rng(77)
    n = 300_000
    region = Column.from_numbers(col.Int32, rng.integers(0, 500, n))
    user = Column.from_numbers(col.Int64, rng.integers(0, 30_000, n) * 7919, validity=rng.random(n) > 0.05)
    adv = Column.from_numbers(col.Int16, np.where(rng.random(n) < 0.9, 0, rng.integers(1, 33, n)))
    s = Column.from_strings([b"s%d" % v for v in rng.integers(0, 40, n)])
    aggs = [("sum", adv), ("count", None), ("count_distinct", user), ("count_distinct", s)]
    fns = [F.get(fn, [], [c.dtype] if c is not None else []) for fn, c in aggs]
    params = AggregatorParams([region.dtype], fns)
    cols = [region, adv, user, s]
    arg_idx = [1, None, 2, 3]
    cfg_a = HashTableConfig(max_radix_bits=5)
    cfg_b = HashTableConfig(max_radix_bits=3 if mixed_bits else 5)
    pa, pb = TransformPartialAggregate(params, cfg_a), TransformPartialAggregate(params, cfg_b)
    try:
        half = n // 2
        for p, lo, hi in ((pa, 0, half), (pb, half, n)):
            for b in range(lo, hi, 65536):
                e = min(hi, b + 65536)
                p.transform(DataBlock([slice_col(c, b, e) for c in cols]), [0], arg_idx)
        metas = pa.on_finish() + pb.on_finish()
        assert all(m.distinct is not None and len(m.distinct) == 2 for m in metas)
        bucket = TransformPartitionBucket(params)
        bucket.push(metas)
        parts = bucket.finish()
        maxp = 32
        final = TransformFinalAggregate(params)
        out = {}
        for part in parts:
            blk = final.transform(part)
            ks = blk.columns[4:]
            if not len(ks[0]):
                continue
            h = oracle.group_hash(ks)
            assert (((h & np.uint64((1 << 48) - 1)) >> np.uint64(48 - 5)) == part.bucket).all()
            for i, kk in enumerate(ks[0].values()):
                assert kk not in out
                out[kk] = tuple(c.values()[i] for c in blk.columns[:4])
    finally:
        pa.close()
        pb.close()
    ref = DistinctAggregator(params).run([region], [adv, None, user, s])
    exp = {kk: tuple(c.values()[i] for c in ref.columns[:4]) for i, kk in enumerate(ref.columns[4].values())}
    assert out == exp
    cd = _expected_distinct(region, "count", user)
    assert {k: v[2] for k, v in out.items()} == cd
    assert maxp == 32


def test_distinct_partial_compacts_its_tables():
    """A DISTINCT partial over many host blocks of String keys and String values keeps copies of
    the blocks its main table and pair tables reference; with a small compact_bytes it compacts
    them together, so the retained bytes follow the groups and value sets (bounded), and the
    result still equals the single-node DistinctAggregator."""
    from databend_amd.aggregator import DataBlock, TransformFinalAggregate, TransformPartialAggregate, TransformPartitionBucket
    from tests.test_gpu_parity import slice_col
    rng = np.random.default_rng(91)
    n = 400_000
    k = Column.from_strings([b"key-%05d" % v for v in rng.integers(0, 2000, n)])
    x = Column.from_strings([b"val-%03d" % v for v in rng.integers(0, 40, n)])
    i64 = Column.from_numbers(col.Int64, rng.integers(-1000, 1000, n))
    aggs = [("sum", i64), ("count_distinct", x)]
    fns = [F.get(fn, [], [c.dtype]) for fn, c in aggs]
    params = AggregatorParams([k.dtype], fns)
    limit = 4 << 20
    p = TransformPartialAggregate(params, compact_bytes=limit)
    peak = 0
    try:
        for b in range(0, n, 16384):
            e = min(n, b + 16384)
            p.transform(DataBlock([slice_col(c, b, e) for c in (k, i64, x)]), [0], [1, 2])
            peak = max(peak, p.distinct.retained_bytes())
        assert peak < 3 * limit, peak  # without compaction: every block's copy (> 20 MB)
        metas = p.on_finish()
    finally:
        p.close()
    bucket = TransformPartitionBucket(params)
    bucket.push(metas)
    final = TransformFinalAggregate(params)
    out = {}
    for part in bucket.finish():
        blk = final.transform(part)
        for i, kk in enumerate(blk.columns[2].values()):
            out[kk] = (blk.columns[0].values()[i], blk.columns[1].values()[i])
    ref = DistinctAggregator(params).run([k], [i64, x])
    exp = {kk: (ref.columns[0].values()[i], ref.columns[1].values()[i]) for i, kk in enumerate(ref.columns[2].values())}
    assert out == exp
