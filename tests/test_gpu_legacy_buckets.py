"""GPU parity of the legacy HashMethod path's buckets (enable_experimental_aggregate_hashtable = 0,
SURVEY.md §8f-3) through partial -> bucket -> final, against the oracle:

* a partial below group_by_two_level_threshold groups emits one single-level meta (bucket -1,
  AGG/transform_aggregate_partial.rs:422-428); above it, the non-empty of 256 buckets
  hash2bucket<8, true>(FastHash(key)) (:430-447, HT/partitioned_hashtable.rs:77-83);
* TransformPartitionBucket keeps all-single-level input as one bucket -1, and splits single-level
  inputs into the 256 buckets once any input is two-level (AGG/transform_partition_bucket.rs:
  205-300);
* every group of bucket b has the oracle's legacy FastHash bucket b, and the final results over
  all buckets equal the oracle's aggregate.
Keys cover FixedKeys (Int32 + nullable Int16 -> u64 packing), a single String (SingleBinary), and
HashMethodSerializer keys (two Strings, String + nullable Int32, Boolean + Int16)."""
import numpy as np
import pytest

from databend_amd import abi
from databend_amd import column as col
from databend_amd.aggregates import AggregateFunctionFactory
from databend_amd.aggregator import (LEGACY_BUCKETS, SINGLE_LEVEL_BUCKET, AggregatorParams, HashTableConfig,
                                     TransformFinalAggregate, TransformPartialAggregate, TransformPartitionBucket)
from databend_amd.column import Column, DataBlock
from databend_amd.ffi import Unsupported
from oracle import oracle
from tests.parity import assert_results_equal
from tests.test_gpu_parity import oracle_aggregate, slice_col
from tests.test_gpu_pipeline import concat

pytestmark = pytest.mark.gpu
F = AggregateFunctionFactory.instance()
BLOCK = 65536


def _data(case, n, groups, rng):
    if case == "fixed":
        g = rng.integers(0, groups, n)
        keys = [Column.from_numbers(col.Int32, g * 7 - 1000),
                Column.from_numbers(col.Int16, g % 5, validity=(g % 11) != 3)]
    else:
        words = ["w%06d" % i * (1 + i % 2) for i in range(groups)]
        keys = [Column.from_strings([words[i] for i in rng.integers(0, groups, n)])]
    v = Column.from_numbers(col.Int64, rng.integers(-1000, 1000, n))
    d = Column.from_decimals(15, 2, [int(x) for x in rng.integers(-10**9, 10**9, n)])
    return keys, [("count", None), ("sum", v), ("max", v), ("sql_avg", d)]


def _partial(params, keys, aggs, lo, hi, strategy=None):
    nk = len(keys)
    arg_idx, j = [], nk
    for _, c in aggs:
        arg_idx.append(None if c is None else j)
        j += c is not None
    p = TransformPartialAggregate(params, HashTableConfig(), staging_rows=1 << 20)
    if strategy is not None:
        p.hashtable.set_strategy(strategy)
    for s in range(lo, hi, BLOCK):
        e = min(hi, s + BLOCK)
        cols = [slice_col(k, s, e) for k in keys] + [slice_col(c, s, e) for _, c in aggs if c is not None]
        p.transform(DataBlock(cols), list(range(nk)), arg_idx)
    return p


def _final_all(params, parts, nk, na):
    final = TransformFinalAggregate.try_create(params)
    out_k, out_a = [[] for _ in range(nk)], [[] for _ in range(na)]
    for p in parts:
        blk = final.transform(p)
        ks = blk.columns[na:]
        if p.bucket != SINGLE_LEVEL_BUCKET:
            got = (oracle.legacy_group_hash(ks) >> np.uint64(24)) & np.uint64(255)
            assert (got == p.bucket).all(), f"bucket {p.bucket} holds groups of other buckets"
        for i in range(nk):
            out_k[i].append(ks[i])
        for i in range(na):
            out_a[i].append(blk.columns[i])
    return [concat(c) for c in out_k], [concat(c) for c in out_a]


@pytest.mark.parametrize("case,strategy", [("fixed", None), ("binary", None), ("fixed", abi.STRATEGY_PARTITIONED),
                                           ("binary", abi.STRATEGY_PARTITIONED)])
def test_legacy_two_level_and_split(case, strategy):
    """One partial above the threshold (two-level), one below (single-level, split by the bucket
    transform); the two-level partial on the HBM table or on the partitioned payload (its buckets
    come from the payload's group records)."""
    rng = np.random.default_rng(21 if case == "fixed" else 22)
    n_a, n_b = 400_000, 5_000
    keys_a, aggs = _data(case, n_a, 60_000, rng)
    keys_b, aggs_b = _data(case, n_b, 300, rng)
    keys = [concat([a, b]) for a, b in zip(keys_a, keys_b)]
    aggs = [(f, None if c is None else concat([c, cb])) for (f, c), (_, cb) in zip(aggs, aggs_b)]
    fns = [F.get(f, [], [c.dtype] if c is not None else []) for f, c in aggs]
    params = AggregatorParams([k.dtype for k in keys], fns, enable_experimental_aggregate_hashtable=False)
    pa = _partial(params, keys, aggs, 0, n_a, strategy)
    pb = _partial(params, keys, aggs, n_a, n_a + n_b)
    try:
        ma, mb = pa.on_finish(), pb.on_finish()
        assert len(mb) == 1 and mb[0].bucket == SINGLE_LEVEL_BUCKET and mb[0].legacy
        assert len(ma) > 200 and all(0 <= m.bucket < LEGACY_BUCKETS and m.max_partition_count == LEGACY_BUCKETS for m in ma)
        assert [m.bucket for m in ma] == sorted({m.bucket for m in ma})
        bt = TransformPartitionBucket(params)
        bt.push(mb + ma)
        parts = bt.finish()
        bs = [p.bucket for p in parts]
        assert bs == sorted(set(bs)) and bs[0] >= 0 and bs[-1] < LEGACY_BUCKETS
        gk, ga = _final_all(params, parts, len(keys), len(aggs))
        ok, oa = oracle_aggregate(keys, aggs, None, threads=8)
        assert_results_equal(gk, ga, ok, oa)
    finally:
        pa.close()
        pb.close()


def test_legacy_single_level_only():
    rng = np.random.default_rng(23)
    n = 120_000
    keys, aggs = _data("fixed", n, 2_000, rng)
    fns = [F.get(f, [], [c.dtype] if c is not None else []) for f, c in aggs]
    params = AggregatorParams([k.dtype for k in keys], fns, enable_experimental_aggregate_hashtable=False)
    pa = _partial(params, keys, aggs, 0, n // 2)
    pb = _partial(params, keys, aggs, n // 2, n)
    try:
        metas = pa.on_finish() + pb.on_finish()
        assert [m.bucket for m in metas] == [SINGLE_LEVEL_BUCKET] * 2
        bt = TransformPartitionBucket(params)
        bt.push(metas)
        parts = bt.finish()
        assert len(parts) == 1 and parts[0].bucket == SINGLE_LEVEL_BUCKET and len(parts[0].data) == 2
        gk, ga = _final_all(params, parts, len(keys), len(aggs))
        ok, oa = oracle_aggregate(keys, aggs, None, threads=8)
        assert_results_equal(gk, ga, ok, oa)
    finally:
        pa.close()
        pb.close()


def test_legacy_threshold_setting_and_serializer_keys():
    rng = np.random.default_rng(24)
    n = 50_000
    keys, aggs = _data("fixed", n, 1_000, rng)
    fns = [F.get(f, [], [c.dtype] if c is not None else []) for f, c in aggs]
    # a lower group_by_two_level_threshold turns the same partial two-level
    params = AggregatorParams([k.dtype for k in keys], fns, enable_experimental_aggregate_hashtable=False,
                              group_by_two_level_threshold=500)
    p = _partial(params, keys, aggs, 0, n)
    try:
        metas = p.on_finish()
        assert all(m.bucket >= 0 for m in metas) and sum(len(m.payload) for m in metas) == 1_000
    finally:
        p.close()



@pytest.mark.parametrize("case", ["two_strings", "string_nullable_int", "bool_int"])
def test_legacy_serializer_keys(case):
    """HashMethodSerializer keys (EXP/kernels/group_by.rs:48-95): two Strings (TPC-H Q1's
    l_returnflag, l_linestatus), a String with a nullable Int32, a Boolean with an Int16 — the
    buckets are hash2bucket<8> of the FastHash of the serialized key bytes (serialize_column_binary,
    group_by_hash/utils.rs:64-121), checked group by group against the oracle's restatement."""
    rng = np.random.default_rng(31)
    n = 300_000
    if case == "two_strings":
        g = rng.integers(0, 40_000, n)
        keys = [Column.from_strings(["a%d" % (x % 4000) for x in g]), Column.from_strings(["b" * (x % 13) for x in g])]
    elif case == "string_nullable_int":
        g = rng.integers(0, 30_000, n)
        keys = [Column.from_strings(["k%05d" % (x % 7000) for x in g]),
                Column.from_numbers(col.Int32, g % 11, validity=(g % 7) != 0)]
    else:
        g = rng.integers(0, 60_000, n)
        keys = [Column.from_bools(g % 2 == 0), Column.from_numbers(col.Int16, g % 30_000)]
    v = Column.from_numbers(col.Int64, rng.integers(-1000, 1000, n))
    aggs = [("count", None), ("sum", v)]
    fns = [F.get(f, [], [c.dtype] if c is not None else []) for f, c in aggs]
    params = AggregatorParams([k.dtype for k in keys], fns, enable_experimental_aggregate_hashtable=False)
    p = _partial(params, keys, aggs, 0, n)
    try:
        metas = p.on_finish()
        assert len(metas) > 100 and all(0 <= m.bucket < LEGACY_BUCKETS for m in metas)
        bt = TransformPartitionBucket(params)
        bt.push(metas)
        gk, ga = _final_all(params, bt.finish(), len(keys), len(aggs))
        ok, oa = oracle_aggregate(keys, aggs, None, threads=8)
        assert_results_equal(gk, ga, ok, oa)
    finally:
        p.close()


@pytest.mark.parametrize("ktype", [col.UInt16, col.Int8.wrap_nullable()])
def test_legacy_small_keys_stay_single_level(ktype):
    """HashMethodFixedKeys<u8> / <u16> (a UInt16 key, a nullable Int8 key = 2 key bytes) never go
    two-level (SUPPORT_PARTITIONED = false, aggregator_polymorphic_keys.rs:149,189), whatever the
    group count: one bucket -1 meta, as the reference emits."""
    rng = np.random.default_rng(25)
    n = 200_000
    if ktype == col.UInt16:
        k = Column.from_numbers(col.UInt16, rng.integers(0, 65536, n))
    else:
        k = Column.from_numbers(col.Int8, rng.integers(-128, 128, n), validity=rng.random(n) > 0.1)
    v = Column.from_numbers(col.Int64, rng.integers(-1000, 1000, n))
    aggs = [("count", None), ("sum", v)]
    fns = [F.get(f, [], [c.dtype] if c is not None else []) for f, c in aggs]
    params = AggregatorParams([k.dtype], fns, enable_experimental_aggregate_hashtable=False,
                              group_by_two_level_threshold=100)
    p = _partial(params, [k], aggs, 0, n)
    try:
        metas = p.on_finish()
        assert [m.bucket for m in metas] == [SINGLE_LEVEL_BUCKET]
        bt = TransformPartitionBucket(params)
        bt.push(metas)
        parts = bt.finish()
        gk, ga = _final_all(params, parts, 1, len(aggs))
        ok, oa = oracle_aggregate([k], aggs, None, threads=8)
        assert_results_equal(gk, ga, ok, oa)
    finally:
        p.close()
