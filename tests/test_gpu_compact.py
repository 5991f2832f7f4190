"""Key compaction (dbg_agg_compact): a referenced-key table (String / Decimal128 keys) rewritten
to one record batch of its groups, so the inputs it saw are released — the reference keeps only
new groups' keys in its payload arena (EAGG/payload_row.rs:111-130).  Checked against the oracle:

* host blocks: the library's copies of the blocks are freed (retained bytes fall to the groups'
  records) and later blocks still aggregate into the same groups;
* device inputs: after compaction the first batch's key bytes are overwritten on the device, and
  the results over both batches still equal the oracle's (no entry reads the old rows);
* TransformPartialAggregate compacts by itself past `compact_bytes`, through partial -> final;
* inline keys: nothing to compact."""
import numpy as np
import pytest

from databend_amd import column as col
from databend_amd.aggregates import AggregateFunctionFactory
from databend_amd.aggregator import (AggregateHashTable, AggregatorParams, HashTableConfig, TransformFinalAggregate,
                                     TransformPartialAggregate, TransformPartitionBucket)
from databend_amd.column import Column, DataBlock
from tests.parity import assert_results_equal
from tests.test_gpu_parity import oracle_aggregate, slice_col
from tests.test_gpu_pipeline import concat

pytestmark = pytest.mark.gpu
F = AggregateFunctionFactory.instance()


def _data(rng, n, groups):
    g = rng.integers(0, groups, n)
    words = ["phrase-%06d" % i + "x" * (i % 17) for i in range(groups)]
    s = Column.from_strings([words[i] for i in g])
    d = Column.from_decimals(20, 2, [int(x) * 10**15 + 7 for x in (g % 977)])
    v = Column.from_numbers(col.Int64, rng.integers(-1000, 1000, n))
    return [s, d], [("count", None), ("sum", v), ("min", v), ("avg", v)]


def _args(aggs, lo, hi):
    return [None if c is None else slice_col(c, lo, hi) for _, c in aggs]


def _result(ht, na):
    blk = ht.merge_result()
    return blk.columns[na:], blk.columns[:na]


def test_compact_host_blocks():
    rng = np.random.default_rng(41)
    n, blocks = 600_000, 6
    keys, aggs = _data(rng, n, 20_000)
    fns = [F.get(f, [], [c.dtype] if c is not None else []) for f, c in aggs]
    ht = AggregateHashTable(AggregatorParams([k.dtype for k in keys], fns), HashTableConfig(True))
    try:
        step = n // blocks
        for b in range(blocks):
            lo, hi = b * step, (b + 1) * step
            ht.add_groups([slice_col(k, lo, hi) for k in keys], _args(aggs, lo, hi), rows=hi - lo)
            if b == 3:
                before = ht.retained_bytes()
                assert ht.compact()
                after = ht.retained_bytes()
                assert after < before / 4, (before, after)
        gk, ga = _result(ht, len(aggs))
    finally:
        ht.close()
    ok, oa = oracle_aggregate(keys, aggs, threads=8)
    assert_results_equal(gk, ga, ok, oa)


def test_compact_releases_device_inputs():
    from databend_amd.device import DeviceColumn
    rng = np.random.default_rng(42)
    n = 400_000
    keys, aggs = _data(rng, n, 5_000)
    fns = [F.get(f, [], [c.dtype] if c is not None else []) for f, c in aggs]
    ht = AggregateHashTable(AggregatorParams([k.dtype for k in keys], fns), HashTableConfig(True))
    half = n // 2
    try:
        dk = [DeviceColumn.from_host(slice_col(k, 0, half)) for k in keys]
        da = [None if c is None else DeviceColumn.from_host(c) for c in _args(aggs, 0, half)]
        ht.add_groups(dk, da, rows=half, on_device=True)
        assert ht.compact()
        # the first batch's key bytes are gone: a stale reference would now compare garbage
        import torch
        torch.cuda.synchronize()
        dk[0].data.fill_(0xAB)
        dk[1].data.fill_(0x5C)
        dk2 = [DeviceColumn.from_host(slice_col(k, half, n)) for k in keys]
        da2 = [None if c is None else DeviceColumn.from_host(c) for c in _args(aggs, half, n)]
        ht.add_groups(dk2, da2, rows=n - half, on_device=True)
        gk, ga = _result(ht, len(aggs))
    finally:
        ht.close()
    ok, oa = oracle_aggregate(keys, aggs, threads=8)
    assert_results_equal(gk, ga, ok, oa)


def test_partial_auto_compact_pipeline():
    rng = np.random.default_rng(43)
    n = 300_000
    keys, aggs = _data(rng, n, 8_000)
    fns = [F.get(f, [], [c.dtype] if c is not None else []) for f, c in aggs]
    params = AggregatorParams([k.dtype for k in keys], fns)
    nk = len(keys)
    arg_idx, j = [], nk
    for _, c in aggs:
        arg_idx.append(None if c is None else j)
        j += c is not None
    p = TransformPartialAggregate(params, HashTableConfig(), staging_rows=1 << 16, compact_bytes=1 << 20)
    try:
        for s in range(0, n, 65536):
            e = min(n, s + 65536)
            cols = [slice_col(k, s, e) for k in keys] + [slice_col(c, s, e) for _, c in aggs if c is not None]
            p.transform(DataBlock(cols), list(range(nk)), arg_idx)
            assert p.hashtable.retained_bytes() < (4 << 20) + 8_000 * 256
        metas = p.on_finish()
        bt = TransformPartitionBucket(params)
        bt.push(metas)
        final = TransformFinalAggregate.try_create(params)
        out_k, out_a = [[] for _ in range(nk)], [[] for _ in range(len(aggs))]
        for part in bt.finish():
            blk = final.transform(part)
            for i in range(nk):
                out_k[i].append(blk.columns[len(aggs) + i])
            for i in range(len(aggs)):
                out_a[i].append(blk.columns[i])
    finally:
        p.close()
    ok, oa = oracle_aggregate(keys, aggs, threads=8)
    assert_results_equal([concat(c) for c in out_k], [concat(c) for c in out_a], ok, oa)


def test_compact_inline_keys_is_noop():
    k = Column.from_numbers(col.Int32, np.arange(1000) % 7)
    params = AggregatorParams([k.dtype], [F.get("count", [], [])])
    ht = AggregateHashTable(params, HashTableConfig(True))
    try:
        ht.add_groups([k], [None], rows=1000)
        assert not ht.compact()
        gk, ga = _result(ht, 1)
        assert sorted(gk[0].data.tolist()) == list(range(7))
    finally:
        ht.close()


def test_compact_keeps_strategy_many_groups():
    """the re-merged batch (one record per group) must not re-run the cardinality
    probe — with more than 2^20 groups it would see ratio ~1 and switch an AUTO handle to the
    partitioned payload, after which compact() does nothing."""
    rng = np.random.default_rng(44)
    n, groups = 4_400_000, 1_300_000
    g = rng.integers(0, groups, n)
    s = Column.from_strings(["k%07d" % i for i in g])
    keys, aggs = [s], [("count", None)]
    fns = [F.get("count", [], [])]
    ht = AggregateHashTable(AggregatorParams([s.dtype], fns), HashTableConfig(True))
    try:
        ht.add_groups(keys, [None], rows=n)
        assert ht.strategy()[0] == 0  # moderate cardinality (~0.3 groups per row): the HBM table
        assert ht.compact()
        assert ht.strategy()[0] == 0
        assert ht.compact()  # still a table that compaction rewrites
        gk, ga = _result(ht, 1)
    finally:
        ht.close()
    ok, oa = oracle_aggregate(keys, aggs, threads=8)
    assert_results_equal(gk, ga, ok, oa)
