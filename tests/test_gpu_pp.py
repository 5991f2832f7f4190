"""GPU parity of the radix-partitioned payload (pp.hip) against the oracle.

The partitioned strategy is the high-cardinality path: batches are scattered
into hash partitions (PartitionedPayload::append_rows, EAGG/partitioned_payload.rs:100-143) and
finalize aggregates every partition in one workgroup's LDS table.  Every key family, every
aggregate, filters, nullable keys/arguments, long string keys (> 39 bytes: referenced, not
inlined), several batches, multi-round partitions (more groups than one LDS table holds) and the
exchange export/merge are checked against the oracle on the same inputs.
"""
import numpy as np
import pytest

from databend_amd import abi
from databend_amd import column as col
from databend_amd.aggregator import AggregateHashTable, AggregatorParams, HashTableConfig
from databend_amd.column import Column
from databend_amd.filter import and_, cmp, is_null, not_, or_
from oracle import oracle
from tests.parity import assert_results_equal
from tests.test_gpu_parity import F, KEY_KINDS, _cat, _rand_inputs, gpu_aggregate, oracle_aggregate, slice_col

pytestmark = pytest.mark.gpu
PP = abi.STRATEGY_PARTITIONED


def check_pp(keys, aggs, filt=None, **kw):
    info = {}
    gk, ga = gpu_aggregate(keys, aggs, filt, strategy=PP, info=info, **kw)
    assert info["partitioned"]
    ok, oa = oracle_aggregate(keys, aggs, filt)
    assert_results_equal(gk, ga, ok, oa)
    return len(gk[0]) if gk else 0, info


def _long_strings(rng, n):
    words = [bytes(rng.integers(97, 123, rng.integers(30, 70))) for _ in range(3000)]
    return [Column.from_strings([words[i] for i in rng.integers(0, len(words), n)], validity=rng.random(n) > 0.05)]


@pytest.mark.parametrize("kind", KEY_KINDS + ["long_string"])
@pytest.mark.parametrize("on_device", [False, True])
def test_pp_random_keys_all_functions(kind, on_device):
    rng = np.random.default_rng(abs(hash(kind + "pp")) % 2**32)
    n = 200_000
    keys = _long_strings(rng, n) if kind == "long_string" else _rand_inputs(rng, n, kind)
    i64 = Column.from_numbers(col.Int64, rng.integers(-2**40, 2**40, n))
    i64n = Column.from_numbers(col.Int64, rng.integers(-1000, 1000, n), validity=rng.random(n) > 0.5)
    u32 = Column.from_numbers(col.UInt32, rng.integers(0, 2**32 - 1, n, dtype=np.uint64).astype(np.uint32))
    f64 = Column.from_numbers(col.Float64, rng.random(n) * 1000)
    f32 = Column.from_numbers(col.Float32, (rng.random(n) * 100).astype(np.float32))
    i8 = Column.from_numbers(col.Int8, rng.integers(-100, 100, n))
    dec = Column.from_decimals(15, 2, [int(v) for v in rng.integers(-10**12, 10**12, n)])
    dec38 = Column.from_decimals(38, 6, [int(v) * 10**20 for v in rng.integers(-10**9, 10**9, n)])
    aggs = [("count", None), ("count", i64n), ("sum", i64), ("sum", i64n), ("sum", u32), ("sum", f64), ("sum", dec),
            ("sum", dec38), ("avg", i64), ("avg", f64), ("avg", dec), ("avg", i64n), ("min", i64), ("max", i64n),
            ("min", f64), ("max", u32), ("max", dec), ("sum", i8), ("min", f32), ("avg", f32)]
    check_pp(keys, aggs, on_device=on_device, batches=3)


@pytest.mark.parametrize("kind", ["i64", "string"])
def test_pp_sql_avg(kind):
    """SQL avg (DBG_AGG_AVG_SQL: sum / if(count = 0, 1, count), decimal round-half-away divide)
    through the partitioned payload's fused finalize."""
    rng = np.random.default_rng(41)
    n = 300_000
    keys = _rand_inputs(rng, n, kind)
    dec = Column.from_decimals(15, 2, [int(v) for v in rng.integers(-10**12, 10**12, n)], validity=rng.random(n) > 0.1)
    dec38 = Column.from_decimals(38, 6, [int(v) * 10**20 for v in rng.integers(-10**9, 10**9, n)])
    i64n = Column.from_numbers(col.Int64, rng.integers(-1000, 1000, n), validity=rng.random(n) > 0.5)
    f64 = Column.from_numbers(col.Float64, rng.random(n) * 1000)
    check_pp(keys, [("count", None), ("sql_avg", dec), ("sql_avg", dec38), ("sql_avg", i64n), ("sql_avg", f64)],
             on_device=True, batches=2)


@pytest.mark.parametrize("kind", ["i64_hi", "string", "i64_i32"])
def test_pp_multi_round_partitions(kind):
    """capacity_hint = 1 sizes the final partitions for one group each: 512 partitions of
    thousands of groups, so most partitions take several LDS rounds (overflow records ping-pong
    between the level buffers)."""
    rng = np.random.default_rng(7)
    n = 3_000_000
    if kind == "i64_hi":
        keys = [Column.from_numbers(col.Int64, rng.integers(0, 2_500_000, n) * 7919 - 3)]
    elif kind == "string":
        keys = [Column.from_strings([b"k%07d" % v for v in rng.integers(0, 1_500_000, n)])]
    else:
        keys = [Column.from_numbers(col.Int64, rng.integers(0, 900_000, n)), Column.from_numbers(col.Int32, rng.integers(0, 3, n))]
    v = Column.from_numbers(col.Int64, rng.integers(0, 10, n))
    g, info = check_pp(keys, [("count", None), ("sum", v), ("max", v)], on_device=True, capacity_hint=1, batches=2)
    assert g > 1_000_000
    assert info["extra_rounds"] > 0


@pytest.mark.parametrize("on_device", [False, True])
def test_pp_filter_fused(on_device):
    rng = np.random.default_rng(15)
    n = 300_000
    adv = Column.from_numbers(col.Int32, np.where(rng.random(n) < 0.5, 0, rng.integers(1, 50_000, n)))
    s = Column.from_strings([b"" if r < 0.6 else b"p%d" % (r * 100000) for r in rng.random(n)])
    v = Column.from_numbers(col.Int64, rng.integers(0, 100, n), validity=rng.random(n) > 0.1)
    pred = or_(and_(cmp(0, "<>", 0), not_(cmp(1, "=", ""))), is_null(2))
    check_pp([adv], [("count", None), ("sum", v)], filt=(pred, [adv, s, v]), on_device=on_device)
    check_pp([s], [("count", None), ("max", v)], filt=(cmp(1, ">=", "p50"), [adv, s]), on_device=on_device)


def test_pp_empty_and_all_filtered():
    rng = np.random.default_rng(2)
    n = 10_000
    k = Column.from_numbers(col.Int64, rng.integers(0, 100, n))
    g, _ = check_pp([k], [("count", None)], filt=(cmp(0, "<", -5), [k]))
    assert g == 0


@pytest.mark.parametrize("kind", ["i64_i32", "string_nullable_date", "long_string"])
def test_pp_export_merge_matches_routing(kind):
    """Partitioned partials -> records by hash % 4 (Payload::scatter) -> merge_records into 4
    partitioned finals: each final holds exactly its routed groups; the union equals the oracle."""
    import torch
    rng = np.random.default_rng(31)
    n = 300_000
    keys = _long_strings(rng, n) if kind == "long_string" else _rand_inputs(rng, n, kind)
    v = Column.from_decimals(20, 3, [int(x) for x in rng.integers(-10**10, 10**10, n)])
    m = Column.from_numbers(col.Int32, rng.integers(-5, 5, n))
    fns = [F.get("count"), F.get("sum", [], [v.dtype]), F.get("min", [], [m.dtype]), F.get("avg", [], [m.dtype])]
    params = AggregatorParams([k.dtype for k in keys], fns)
    partials = []
    for lo, hi in ((0, n // 3), (n // 3, n)):
        ht = AggregateHashTable(params, HashTableConfig(True))
        ht.set_strategy(PP)
        ht.add_groups([slice_col(k, lo, hi) for k in keys], [None, slice_col(v, lo, hi), slice_col(m, lo, hi), slice_col(m, lo, hi)])
        partials.append(ht)
    W = 4
    finals = [AggregateHashTable(params, HashTableConfig(False)) for _ in range(W)]
    for f in finals:
        f.set_strategy(PP)
    w = partials[0].record_width()
    keep = []
    for ht in partials:
        counts, sbytes = ht.partition(W, 0)
        recs = torch.empty(max(1, sum(counts) * w), dtype=torch.uint8, device="cuda")
        strs = torch.empty(max(1, sum(sbytes)), dtype=torch.uint8, device="cuda")
        ht.export_records(recs, strs)
        torch.cuda.synchronize()
        ro, so = 0, 0
        for p in range(W):
            r = recs[ro * w:(ro + counts[p]) * w]
            s = strs[so:so + sbytes[p]] if sbytes[p] else strs[:1]
            finals[p].merge_records(r, s, [counts[p]], [sbytes[p]])
            keep.append((r, s))
            ro += counts[p]
            so += sbytes[p]
    nk, na = len(keys), 4
    all_k, all_a = [], []
    for p, f in enumerate(finals):
        blk = f.merge_result()
        ks, ags = blk.columns[na:], blk.columns[:na]
        if len(ks[0]):
            assert np.all(oracle.group_hash(ks) % W == p)
        all_k.append(ks)
        all_a.append(ags)
    ok, oa = oracle_aggregate(keys, [("count", None), ("sum", v), ("min", m), ("avg", m)])
    cat = lambda cols: Column(cols[0].dtype, *_cat(cols))
    gk = [cat([k[i] for k in all_k]) for i in range(nk)]
    ga = [cat([a[i] for a in all_a]) for i in range(na)]
    assert_results_equal(gk, ga, ok, oa)
    for t in partials + finals:
        t.close()


def test_pp_radix_buckets_scheme1():
    """dbg_agg_partition scheme 1 (radix buckets, bits [48 - r, 48) of the group hash,
    PartitionedPayload) from a partitioned table: each bucket holds exactly its groups."""
    import torch
    rng = np.random.default_rng(5)
    n = 200_000
    keys = _rand_inputs(rng, n, "i64_hi")
    params = AggregatorParams([keys[0].dtype], [F.get("count")])
    ht = AggregateHashTable(params, HashTableConfig(True))
    ht.set_strategy(PP)
    ht.add_groups(keys, [None])
    R = 16
    counts, _ = ht.partition(R, 1)
    w = ht.record_width()
    recs = torch.empty(max(1, sum(counts) * w), dtype=torch.uint8, device="cuda")
    ht.export_records(recs, torch.empty(1, dtype=torch.uint8, device="cuda"))
    torch.cuda.synchronize()
    raw = recs.cpu().numpy()[: sum(counts) * w].reshape(-1, w)
    h = raw[:, :8].copy().view(np.uint64).ravel()
    bucket = (h >> np.uint64(44)) & np.uint64(R - 1)
    starts = np.concatenate([[0], np.cumsum(counts)])
    for b in range(R):
        assert np.all(bucket[starts[b]:starts[b + 1]] == b)
    assert sum(counts) == len(np.unique(keys[0].data))
    ht.close()


@pytest.mark.parametrize("cfg,n", [(3, 6_000_000), (4, 5_000_000), (5, 8_000_000)])
def test_pp_benchmark_configs(cfg, n):
    """The bench runner (device datagen, fused finalize into device columns) on the partitioned
    strategy vs the oracle on the same rows."""
    from databend_amd import workloads
    res = workloads.run_config(cfg, n, steps=2, strategy=PP)
    assert res["partitioned"]
    cols = oracle.datagen(cfg, n)
    shape = workloads.SHAPES[cfg]
    keys = [cols[k] for k in shape.keys]
    aggs = [(f, cols[c] if c else None) for f, c in shape.aggs]
    filt = None
    if shape.predicate:
        name, op, const = shape.predicate
        filt = (cmp(0, op, const), [cols[name]])
    ok, oa = oracle_aggregate(keys, aggs, filt, threads=8)
    assert_results_equal(res["keys"], res["aggs"], ok, oa)


def test_pp_auto_probe_selects_partitioned_for_c4():
    """DBG_STRATEGY_AUTO: the cardinality probe of a 5M-row all-distinct batch (C4 shape) picks
    the partitioned payload; a 5M-row C2 batch (Int16 key) never probes and stays on the table."""
    from databend_amd import workloads
    r4 = workloads.run_config(4, 5_000_000, steps=1)
    assert r4["partitioned"] and r4["n_groups"] == 5_000_000
    r2 = workloads.run_config(2, 5_000_000, steps=1)
    assert not r2["partitioned"]


@pytest.mark.parametrize("kind", ["i64", "i64_i32", "dup_heavy", "skewed"])
def test_pp_record_centric(kind):
    """Record-centric aggregation of raw records (pp.hip pp_agg_rc_kernel): level-2 partitions of
    ~PP_RC_PART records aggregated in LDS rounds.  Mostly-unique keys (its target), keys with a few
    records each, and a skewed key holding a large share of the rows — whose partition exceeds one
    round's LDS and is spilled to the slot-table kernel — all against the oracle."""
    rng = np.random.default_rng(len(kind))
    n = 6_000_000
    if kind == "i64":
        keys = [Column.from_numbers(col.Int64, rng.permutation(n).astype(np.int64) * 7919 - 3)]
    elif kind == "i64_i32":
        keys = [Column.from_numbers(col.Int64, rng.integers(0, n, n)), Column.from_numbers(col.Int32, rng.integers(0, 2**31 - 1, n))]
    elif kind == "dup_heavy":
        keys = [Column.from_numbers(col.Int64, rng.integers(0, n // 3, n))]
    else:
        k = rng.integers(0, n, n)
        k[rng.random(n) < 0.3] = 42  # 30 % of the rows in one group
        keys = [Column.from_numbers(col.Int64, k)]
    i16 = Column.from_numbers(col.Int16, rng.integers(-3, 3, n))
    w = Column.from_numbers(col.Int16, rng.integers(0, 2560, n))
    g, info = check_pp(keys, [("count", None), ("sum", i16), ("sql_avg", w), ("min", w)], on_device=True)
    assert g > 1_000_000


@pytest.mark.parametrize("kind", ["c4_unique", "c4_dup", "c4_skewed", "i64_count", "i64_sum", "i64_i64", "small_table",
                                  "i32_minmax", "date_ts_4aggs", "u64_sum_avg", "u16_u8_count", "c4_unique_desc", "c4_skewed_desc"])
def test_pp_specialised_kernel(kind, monkeypatch):
    """The compile-time specialised aggregation (pp.hip pp_agg_spec_kernel) on every instantiated
    shape: C4 (Int64, Int32 keys; COUNT(*), SUM(Int16), AVG(Int16)) with mostly-unique keys, a few
    records per key, and a skewed key whose partition exceeds the kernel's register budget (spilled
    to the generic kernel); one-key COUNT / COUNT+SUM and two-Int64-key COUNT; and a forced small
    LDS table (probe-window misses re-inserted in pending rounds) — all against the oracle."""
    rng = np.random.default_rng(len(kind) * 7 + 1)
    n = 4_000_000
    i16 = Column.from_numbers(col.Int16, rng.integers(-3, 3, n))
    w = Column.from_numbers(col.Int16, rng.integers(-2560, 2560, n))
    aggs = [("count", None), ("sum", i16), ("sql_avg", w)]
    if kind.endswith("_desc"):  # the descriptor kernel on C4's shape (it also has a compile-time instance)
        monkeypatch.setenv("DBG_X_PPSPEC_DESC", "1")
        kind = kind[:-5]
    if kind in ("c4_unique", "small_table"):
        keys = [Column.from_numbers(col.Int64, rng.permutation(n).astype(np.int64) * 7919 - 3),
                Column.from_numbers(col.Int32, rng.integers(-2**31, 2**31 - 1, n))]
    elif kind == "c4_dup":
        keys = [Column.from_numbers(col.Int64, rng.integers(0, n // 3, n)), Column.from_numbers(col.Int32, rng.integers(0, 2, n))]
    elif kind == "c4_skewed":
        k = rng.integers(0, n, n)
        k[rng.random(n) < 0.2] = 42  # 20 % of the rows in one group: its partition is spilled
        keys = [Column.from_numbers(col.Int64, k), Column.from_numbers(col.Int32, np.zeros(n, dtype=np.int64))]
    elif kind == "i64_count":
        keys = [Column.from_numbers(col.Int64, rng.integers(-2**62, 2**62, n))]
        aggs = [("count", None)]
    elif kind == "i64_sum":
        keys = [Column.from_numbers(col.Int64, rng.integers(0, n // 2, n))]
        aggs = [("count", None), ("sum", Column.from_numbers(col.Int64, rng.integers(-2**50, 2**50, n)))]
    elif kind == "i32_minmax":  # shapes outside the benchmark: the kernel's class, not a list of queries
        keys = [Column.from_numbers(col.Int32, rng.integers(-2**31, 2**31 - 1, n))]
        aggs = [("count", None), ("min", Column.from_numbers(col.Int32, rng.integers(-2**31, 2**31 - 1, n))),
                ("max", Column.from_numbers(col.UInt16, rng.integers(0, 2**16, n))), ("sum", Column.from_numbers(col.Int8, rng.integers(-128, 128, n)))]
    elif kind == "date_ts_4aggs":
        keys = [Column.from_numbers(col.Date, rng.integers(0, 20000, n).astype(np.int32)),
                Column.from_numbers(col.Timestamp, rng.integers(0, n, n) * 1_000_000)]
        aggs = [("sum", Column.from_numbers(col.Int64, rng.integers(-2**40, 2**40, n))),
                ("avg", Column.from_numbers(col.UInt32, rng.integers(0, 2**32 - 1, n, dtype=np.uint64).astype(np.uint32))),
                ("max", Column.from_numbers(col.Int64, rng.integers(-2**62, 2**62, n))), ("count", None)]
    elif kind == "u64_sum_avg":
        keys = [Column.from_numbers(col.UInt64, rng.integers(0, 2**63, n, dtype=np.uint64))]
        aggs = [("sum", Column.from_numbers(col.UInt64, rng.integers(0, 2**40, n, dtype=np.uint64))),
                ("sql_avg", Column.from_numbers(col.Int32, rng.integers(-2**31, 2**31 - 1, n)))]
    elif kind == "u16_u8_count":
        keys = [Column.from_numbers(col.UInt16, rng.integers(0, 2**16, n)), Column.from_numbers(col.UInt8, rng.integers(0, 256, n))]
        aggs = [("count", None), ("min", Column.from_numbers(col.Int16, rng.integers(-2**15, 2**15, n)))]
    else:
        keys = [Column.from_numbers(col.Int64, rng.integers(0, n, n)), Column.from_numbers(col.Int64, rng.integers(0, 3, n))]
        aggs = [("count", None)]
    if kind == "small_table":
        monkeypatch.setenv("DBG_X_PPSPEC_CAP", "256")
    g, info = check_pp(keys, aggs, on_device=True, batches=2)
    assert info["specialised"]
    assert g > 1_000_000 or kind in ("c4_dup", "u16_u8_count")
    if kind == "small_table":
        assert info["extra_rounds"] > 0


def test_pp_specialised_many_spills():
    """Thousands of heavy keys (> 8192 records each, the specialised kernel's register budget)
    spread over most final partitions: more than 4096 partitions spill to the generic kernel.  The
    spill list holds one id per final partition, so none is dropped (a fixed 4096-entry list
    failed the whole aggregate with DBG_ERR_INTERNAL here).  Checked against numpy's unique counts."""
    rng = np.random.default_rng(2024)
    heavy, per, uniq = 6000, 8400, 8_000_000
    k = np.concatenate([np.repeat(rng.integers(2**40, 2**41, heavy), per), rng.integers(0, 2**39, uniq)])
    k = k[rng.permutation(len(k))].astype(np.int64)
    keys = [Column.from_numbers(col.Int64, k)]
    info = {}
    gk, ga = gpu_aggregate(keys, [("count", None)], strategy=PP, info=info, on_device=True)
    assert info["partitioned"] and info["specialised"]
    uk, uc = np.unique(k, return_counts=True)
    assert_results_equal(gk, ga, [Column.from_numbers(col.Int64, uk)], [Column.from_numbers(col.UInt64, uc.astype(np.uint64))])
