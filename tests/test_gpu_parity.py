"""GPU parity: libdbgpu_agg.so (through the C ABI) against the oracle on identical inputs.

Bar (BASELINE.json north_star): group sets, integer / Decimal128 / count results bit-exact;
float64 SUM/AVG within 1e-12 relative (tests/parity.py FLOAT_REL_TOL).
"""
import json
import os

import numpy as np
import pytest

from databend_amd import abi
from databend_amd import column as col
from databend_amd.aggregates import AggregateFunctionFactory
from databend_amd.aggregator import AggregateHashTable, AggregatorParams, HashTableConfig
from databend_amd.column import Column
from databend_amd.filter import FilterProgram, and_, cmp, is_null, not_, or_
from oracle import oracle
from tests.parity import assert_results_equal

pytestmark = pytest.mark.gpu

F = AggregateFunctionFactory.instance()
HERE = os.path.dirname(os.path.abspath(__file__))


def _torch():
    import torch
    return torch


def gpu_aggregate(keys, aggs, filt=None, on_device=False, capacity_hint=0, batches=1, strategy=abi.STRATEGY_AUTO, info=None):
    """aggs: list of (name, Column|None).  filt: (pred, [Columns]) or None.  info (dict, optional)
    receives the handle's strategy after the run."""
    fns = [F.get(n, [], [c.dtype] if c is not None else []) for n, c in aggs]
    params = AggregatorParams([k.dtype for k in keys], fns)
    ht = AggregateHashTable(params, HashTableConfig(True, capacity_hint))
    ht.set_strategy(strategy)
    try:
        n = len(keys[0])
        bounds = np.linspace(0, n, batches + 1).astype(int)
        for b in range(batches):
            lo, hi = int(bounds[b]), int(bounds[b + 1])
            ks = [slice_col(k, lo, hi) for k in keys]
            ars = [None if c is None else slice_col(c, lo, hi) for _, c in aggs]
            fp = None
            fcols = None
            if filt is not None:
                fcols = [slice_col(c, lo, hi) for c in filt[1]]
            if on_device:
                from databend_amd.device import DeviceColumn
                ks = [DeviceColumn.from_host(k) for k in ks]
                ars = [None if c is None else DeviceColumn.from_host(c) for c in ars]
                if fcols is not None:
                    fcols = [DeviceColumn.from_host(c) for c in fcols]
            if fcols is not None:
                fp = FilterProgram(filt[0], fcols)  # keeps the (device) columns alive
            ht.add_groups(ks, ars, rows=hi - lo, filter_program=fp, on_device=on_device)
        block = ht.merge_result()
        if info is not None:
            info["partitioned"], info["extra_rounds"] = ht.strategy()
            info["specialised"] = ht.pp_specialised()
    finally:
        ht.close()
    na = len(aggs)
    return block.columns[na:], block.columns[:na]


def oracle_aggregate(keys, aggs, filt=None, threads=4):
    specs = []
    for n, c in aggs:
        f = F.get(n, [], [c.dtype] if c is not None else [])
        specs.append((f.to_abi(), c))
    fp = FilterProgram(filt[0], [c.to_abi() for c in filt[1]]) if filt is not None else None
    return oracle.aggregate(keys, specs, filter_program=fp, threads=threads)


def slice_col(c: Column, lo, hi) -> Column:
    if c.dtype.type_id == abi.STRING:
        offs = c.offsets[lo:hi + 1]
        data = c.data[int(offs[0]):int(offs[-1])]
        return Column(c.dtype, data, (offs - offs[0]).astype(np.uint64), None if c.validity is None else c.validity[lo:hi])
    if c.dtype.type_id == abi.DECIMAL128:
        return Column(c.dtype, c.data[lo * 16:hi * 16], None, None if c.validity is None else c.validity[lo:hi])
    return Column(c.dtype, c.data[lo:hi], None, None if c.validity is None else c.validity[lo:hi])


def check_parity(keys, aggs, filt=None, **kw):
    gk, ga = gpu_aggregate(keys, aggs, filt, **kw)
    ok, oa = oracle_aggregate(keys, aggs, filt)
    assert_results_equal(gk, ga, ok, oa)
    return len(gk[0]) if gk else 0


# ------------------------------------------------------------------------------------------
GOLD = json.load(open(os.path.join(HERE, "golden", "agg_function_goldens.json")))


@pytest.mark.parametrize("case", GOLD["cases"], ids=lambda c: f"{c['fn']}({c['arg'] or ''})-{'gb' if c['grouped'] else 'one'}")
def test_function_goldens_gpu(case):
    from tests.test_oracle_golden import example_column
    from decimal import Decimal
    arg = example_column(case["arg"]) if case["arg"] else None
    key = Column.from_numbers(col.Int64, [0, 1, 0, 1] if case["grouped"] else [0, 0, 0, 0])
    keys, aggs = gpu_aggregate([key], [(case["fn"], arg)])
    order = np.argsort(np.asarray(keys[0].values()))
    vals = aggs[0].values()
    got = [vals[i] for i in order]
    exp = []
    for v, ok in zip(case["values"], case["validity"]):
        if not ok:
            exp.append(None)
        elif case["out_type"] == "Decimal128":
            exp.append(int(Decimal(v).scaleb(aggs[0].dtype.scale)))
        else:
            exp.append(v)
    assert got == exp, case["source"]
    assert aggs[0].dtype.nullable == case["nullable"]


@pytest.mark.parametrize("n", [100, 1000, 100_000])
@pytest.mark.parametrize("on_device", [False, True])
def test_agg_hashtable_closed_form_gpu(n, on_device):
    """agg_hashtable.rs:57-182 on the GPU: 8 key types (String..Boolean), ref-keyed table."""
    x = np.arange(n) % 4
    x2 = np.concatenate([x, x])
    keys = [Column.from_strings([str(v) for v in x2]), Column.from_numbers(col.Int64, x2),
            Column.from_numbers(col.Int32, x2), Column.from_numbers(col.Int16, x2), Column.from_numbers(col.Int8, x2),
            Column.from_numbers(col.Float32, x2.astype(np.float32)), Column.from_numbers(col.Float64, x2.astype(np.float64)),
            Column.from_bools(x2 != 0)]
    a = keys[1]
    gk, ga = gpu_aggregate(keys, [("min", a), ("max", a), ("sum", a), ("count", a)], on_device=on_device, batches=2)
    assert len(gk[0]) == 4
    rows = sorted(zip(*[c.values() for c in gk + ga]), key=lambda r: r[1])
    for g, r in enumerate(rows):
        assert r[0] == str(g).encode() and r[1] == g and r[7] == (g != 0)
        assert r[8:] == (g, g, g * n // 2, n // 2)


def _rand_inputs(rng, n, kind):
    if kind == "i16":
        return [Column.from_numbers(col.Int16, rng.integers(-50, 50, n))]
    if kind == "i64":  # includes -1 (the all-ones packed key -> sentinel slot)
        return [Column.from_numbers(col.Int64, rng.integers(-3, 3, n) * (1 << 40) - 1)]
    if kind == "i64_hi":
        u = rng.integers(0, n // 2, n).astype(np.uint64) * np.uint64(0x9E3779B97F4A7C15)
        return [Column.from_numbers(col.Int64, u.view(np.int64))]
    if kind == "i64_i32":
        return [Column.from_numbers(col.Int64, rng.integers(0, 300, n)), Column.from_numbers(col.Int32, rng.integers(0, 3, n))]
    if kind == "nullable_u8_i16":
        return [Column.from_numbers(col.UInt8, rng.integers(0, 5, n), validity=rng.random(n) > 0.2),
                Column.from_numbers(col.Int16, rng.integers(0, 7, n), validity=rng.random(n) > 0.3)]
    if kind == "string":
        words = [bytes(rng.integers(97, 100, rng.integers(0, 12))) for _ in range(500)]
        return [Column.from_strings([words[i] for i in rng.integers(0, 500, n)])]
    if kind == "string_nullable_date":
        words = [bytes(rng.integers(97, 123, rng.integers(1, 30))) for _ in range(50)]
        return [Column.from_strings([words[i] for i in rng.integers(0, 50, n)], validity=rng.random(n) > 0.1),
                Column.from_numbers(col.Date, rng.integers(19000, 19010, n).astype(np.int32))]
    if kind == "decimal":
        return [Column.from_decimals(20, 2, [int(v) for v in rng.integers(-5, 5, n) * 10**17])]
    if kind == "float":
        v = rng.integers(0, 20, n).astype(np.float64) / 4
        v[rng.random(n) < 0.05] = np.nan
        return [Column.from_numbers(col.Float64, v)]
    if kind == "bool_u64":
        return [Column.from_bools(rng.random(n) > 0.5), Column.from_numbers(col.UInt64, rng.integers(0, 2**64 - 1, n, dtype=np.uint64) % 9)]
    raise ValueError(kind)


KEY_KINDS = ["i16", "i64", "i64_hi", "i64_i32", "nullable_u8_i16", "string", "string_nullable_date", "decimal", "float", "bool_u64"]


@pytest.mark.parametrize("kind", KEY_KINDS)
@pytest.mark.parametrize("on_device", [False, True])
def test_random_keys_all_functions(kind, on_device):
    rng = np.random.default_rng(hash(kind) % 2**32)
    n = 200_000
    keys = _rand_inputs(rng, n, kind)
    i64 = Column.from_numbers(col.Int64, rng.integers(-2**40, 2**40, n))
    i64n = Column.from_numbers(col.Int64, rng.integers(-1000, 1000, n), validity=rng.random(n) > 0.5)
    u32 = Column.from_numbers(col.UInt32, rng.integers(0, 2**32 - 1, n, dtype=np.uint64).astype(np.uint32))
    # positive values: with cancellation no summation order (the reference's own threads
    # included) is within 1e-12 of another; the bar is stated for well-conditioned sums
    f64 = Column.from_numbers(col.Float64, rng.random(n) * 1000)
    dec = Column.from_decimals(15, 2, [int(v) for v in rng.integers(-10**12, 10**12, n)])
    dec38 = Column.from_decimals(38, 6, [int(v) * 10**20 for v in rng.integers(-10**9, 10**9, n)])
    aggs = [("count", None), ("count", i64n), ("sum", i64), ("sum", i64n), ("sum", u32), ("sum", f64), ("sum", dec),
            ("sum", dec38), ("avg", i64), ("avg", f64), ("avg", dec), ("avg", i64n), ("min", i64), ("max", i64n),
            ("min", f64), ("max", u32), ("max", dec), ("sql_avg", dec), ("sql_avg", dec38), ("sql_avg", i64n), ("sql_avg", f64)]
    check_parity(keys, aggs, on_device=on_device)


@pytest.mark.parametrize("on_device", [False, True])
def test_filter_fused(on_device):
    rng = np.random.default_rng(5)
    n = 300_000
    adv = Column.from_numbers(col.Int16, np.where(rng.random(n) < 0.9, 0, rng.integers(1, 33, n)))
    s = Column.from_strings([b"" if r < 0.8 else b"p%d" % (r * 100) for r in rng.random(n)])
    v = Column.from_numbers(col.Int64, rng.integers(0, 100, n), validity=rng.random(n) > 0.1)
    pred = or_(and_(cmp(0, "<>", 0), not_(cmp(1, "=", ""))), is_null(2))
    check_parity([adv], [("count", None), ("sum", v)], filt=(pred, [adv, s, v]), on_device=on_device)
    check_parity([s], [("count", None), ("max", v)], filt=(cmp(1, ">=", "p50"), [adv, s]), on_device=on_device)


@pytest.mark.parametrize("kind", ["i64_hi", "string", "i64_i32"])
def test_growth_and_overflow_retry(kind):
    """Tiny initial table, many groups: probe-limit overflow, deferred rows/records, rehash."""
    rng = np.random.default_rng(11)
    n = 400_000
    keys = _rand_inputs(rng, n, kind)
    if kind == "string":
        keys = [Column.from_strings([b"k%d" % v for v in rng.integers(0, 150_000, n)])]
    if kind == "i64_i32":
        keys = [Column.from_numbers(col.Int64, rng.integers(0, 90_000, n)), Column.from_numbers(col.Int32, rng.integers(0, 2, n))]
    v = Column.from_numbers(col.Int64, rng.integers(0, 10, n))
    for on_device in (False, True):
        g = check_parity(keys, [("count", None), ("sum", v)], on_device=on_device, capacity_hint=1, batches=3)
        assert g > 50_000


def test_decimal_sum_overflow_error():
    from databend_amd.ffi import DecimalOverflow
    big = 10**37 * 9
    keys = [Column.from_numbers(col.Int64, [1, 1])]
    d = Column.from_decimals(18, 0, [10**17, 10**17])  # p <= 18 => overflow-checked state
    gk, ga = gpu_aggregate(keys, [("sum", d)])
    assert ga[0].values() == [2 * 10**17]
    d2 = Column.from_decimals(38, 0, [big, big])  # p > 18: SUM does not check (wraps like the reference)
    gk, ga = gpu_aggregate(keys, [("sum", d2)])
    wrapped = (2 * big + 2**127) % 2**128 - 2**127
    assert ga[0].values() == [wrapped]
    d3 = Column.from_decimals(38, 0, [big, big])  # AVG with p > 18 checks; 2*big out of range
    with pytest.raises(DecimalOverflow):
        gpu_aggregate(keys, [("avg", d3)])


def test_slt_cases_gpu():
    from tests.test_oracle_golden import SLT, _row_order, _slt_expected, _slt_inputs
    from tests.parity import rows_of
    kind_name = {abi.AGG_COUNT: "count", abi.AGG_SUM: "sum", abi.AGG_AVG: "avg", abi.AGG_MIN: "min",
                 abi.AGG_MAX: "max", abi.AGG_AVG_SQL: "sql_avg"}
    for i, case in enumerate(SLT):
        keys, aggs, flt = _slt_inputs(i)
        names = [(kind_name[spec.kind], c) for spec, c in aggs]
        filt = (flt[0], flt[1]) if flt else None
        gk, ga = gpu_aggregate(keys, names, filt)
        got = sorted([list(r) for r in rows_of(gk, ga)], key=lambda r: _row_order(r, len(keys)))
        exp = _slt_expected(i, case)
        if "limit" in case["sql"]:
            got = got[:len(exp)]
        else:
            exp = sorted(exp, key=lambda r: _row_order(r, len(keys)))
        assert got == exp, case["source"]


def test_export_partition_merge_matches_routing():
    """Partial tables -> records partitioned by hash % 4 (Payload::scatter) -> 4 final tables.
    Each final holds exactly the groups with hash % 4 == its index; the union equals the oracle."""
    torch = _torch()
    rng = np.random.default_rng(3)
    n = 200_000
    key = Column.from_strings([b"s%d" % v for v in rng.integers(0, 20_000, n)])
    k2 = Column.from_numbers(col.Int32, rng.integers(0, 3, n))
    v = Column.from_decimals(20, 3, [int(x) for x in rng.integers(-10**10, 10**10, n)])
    fns = [F.get("count"), F.get("sum", [], [v.dtype]), F.get("min", [], [k2.dtype])]
    params = AggregatorParams([key.dtype, k2.dtype], fns)
    partials = []
    for lo, hi in ((0, n // 3), (n // 3, n)):
        ht = AggregateHashTable(params, HashTableConfig(True))
        ht.add_groups([slice_col(key, lo, hi), slice_col(k2, lo, hi)], [None, slice_col(v, lo, hi), slice_col(k2, lo, hi)])
        partials.append(ht)
    W = 4
    finals = [AggregateHashTable(params, HashTableConfig(False)) for _ in range(W)]
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
    all_k, all_a = [], []
    for p, f in enumerate(finals):
        blk = f.merge_result()
        ks, ags = blk.columns[3:], blk.columns[:3]
        if len(ks[0]):
            h = oracle.group_hash(ks)
            assert np.all(h % W == p)
        all_k.append(ks)
        all_a.append(ags)
    ok, oa = oracle_aggregate([key, k2], [("count", None), ("sum", v), ("min", k2)])
    cat = lambda cols: Column(cols[0].dtype, *_cat(cols))
    gk = [cat([k[i] for k in all_k]) for i in range(2)]
    ga = [cat([a[i] for a in all_a]) for i in range(3)]
    assert_results_equal(gk, ga, ok, oa)
    for t in partials + finals:
        t.close()


def _cat(cols):
    t = cols[0].dtype
    if t.type_id == abi.STRING:
        data = np.concatenate([c.data for c in cols])
        offs = [np.zeros(1, np.uint64)]
        base = 0
        for c in cols:
            offs.append(c.offsets[1:] + base)
            base += int(c.offsets[-1])
        o = np.concatenate(offs).astype(np.uint64)
    else:
        data = np.concatenate([c.data for c in cols])
        o = None
    v = None if cols[0].validity is None else np.concatenate([c.validity for c in cols])
    return data, o, v


@pytest.mark.parametrize("cfg", [1, 2, 3, 4, 5])
def test_device_datagen_matches_host(cfg):
    from databend_amd import workloads
    n = 100_003
    dev = workloads.generate_device(cfg, n)
    host = oracle.datagen(cfg, n)
    for name, hc in host.items():
        dc = dev[name].to_host()
        assert dc.values() == hc.values(), name


def test_c2_full_pipeline_parity():
    """C2 (AdvEngineID <> 0, COUNT(*)) at 20M rows, device-generated input vs the oracle."""
    from databend_amd import workloads
    n = 20_000_000
    res = workloads.run_config(2, n, steps=1)
    host = oracle.datagen(2, n)
    adv = host["AdvEngineID"]
    ok, oa = oracle_aggregate([adv], [("count", None)], filt=(cmp(0, "<>", 0), [adv]), threads=8)
    assert_results_equal(res["keys"], res["aggs"], ok, oa)
    assert sum(res["aggs"][0].values()) == int(np.count_nonzero(adv.data))


def test_filter_select_and_take():
    torch = _torch()
    from databend_amd.device import DeviceColumn
    from databend_amd.ffi import check, lib
    import ctypes as C
    rng = np.random.default_rng(9)
    n = 1_000_003
    a = Column.from_numbers(col.Int32, rng.integers(0, 100, n), validity=rng.random(n) > 0.05)
    s = Column.from_strings([b"x" * int(k) for k in rng.integers(0, 4, n)])
    pred = and_(cmp(0, ">=", 10), cmp(1, "<>", ""))
    da, ds = DeviceColumn.from_host(a), DeviceColumn.from_host(s)
    fp = FilterProgram(pred, [da.to_abi(), ds.to_abi()])
    sel = torch.empty(n, dtype=torch.int32, device="cuda")
    nsel = C.c_uint64()
    torch.cuda.synchronize()
    check(lib().dbg_filter_select(fp.ptr(), n, sel.data_ptr(), C.byref(nsel), None))
    exp = oracle.filter_select(FilterProgram(pred, [a.to_abi(), s.to_abi()]), n)
    got = sel[:nsel.value].cpu().numpy().astype(np.uint32)
    assert np.array_equal(got, exp)
    out = torch.empty(nsel.value * 4, dtype=torch.uint8, device="cuda")
    vbits = torch.empty((nsel.value + 7) // 8, dtype=torch.uint8, device="cuda")
    check(lib().dbg_take_fixed(C.byref(da.to_abi()), sel.data_ptr(), nsel.value, out.data_ptr(), vbits.data_ptr(), None))
    vals = out.cpu().numpy().view(np.int32)
    assert np.array_equal(vals, a.data[exp])


FAST_TYPES = [(col.Int8, -100, 100), (col.UInt8, 0, 250), (col.Int16, -3000, 3000), (col.UInt16, 0, 65000),
              (col.Int32, -10**6, 10**6), (col.UInt32, 0, 4 * 10**9), (col.Int64, -10**12, 10**12),
              (col.UInt64, 0, 2**63), (col.Date, 0, 20000)]


@pytest.mark.parametrize("t,lo,hi", FAST_TYPES, ids=lambda x: repr(x))
def test_fast_path_predicates(t, lo, hi):
    """agg_insert_fast: one integer key with `key <op> const` on itself — every op, constants
    inside and outside the type's range, a row count that leaves a ragged tail."""
    rng = np.random.default_rng(abs(hash(repr(t))) % 2**32)
    n = 1_000_003
    pool = rng.integers(lo, hi, 57, dtype=np.int64 if t.type_id != abi.UINT64 else np.uint64)
    vals = pool[rng.integers(0, 57, n)]
    key = Column.from_numbers(t, vals.astype(t.np_dtype))
    c = int(pool[3])
    cases = [("=", c), ("<>", c), ("<", c), ("<=", c), (">", c), (">=", c)]
    if t.type_id in (abi.INT8, abi.INT16):
        cases += [("<>", 10**6), ("<", -10**6), (">=", -10**6)]
    for op, const in cases:
        check_parity([key], [("count", None)], filt=(cmp(0, op, const), [key]), on_device=True)
    v = Column.from_numbers(col.Int64, rng.integers(0, 100, n))
    check_parity([key], [("count", None), ("sum", v), ("min", v)], filt=(cmp(0, "<>", c), [key]), on_device=True)


# (5, 20M): > 2048 x 4096 rows, so each workgroup of the queued filtered insert runs past the
# periodic LDS-flush checks (FLUSH_ROUND) with a full table of Zipf string keys.
@pytest.mark.parametrize("cfg,n", [(1, 6_001_215), (2, 10_000_000), (3, 3_000_000), (4, 2_000_000), (5, 3_000_000),
                                   (5, 20_000_000)])
def test_benchmark_configs_match_oracle(cfg, n):
    """Each BASELINE.json config through the bench's own runner (device datagen, fused
    finalize into device buffers, growth from the 1024-slot initial table) vs the oracle on the
    same rows generated on the host."""
    from databend_amd import workloads
    res = workloads.run_config(cfg, n, steps=2)
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


def test_recycling_finalize_two_batches_and_short_buffers():
    """dbg_agg_set_recycle: the fused small-table finalize re-initialises the table, so each
    reset -> add_groups -> finalize_into cycle sees only its own batch; a finalize into buffers
    that are too short must leave the table intact for the retry (no recycle)."""
    from databend_amd import workloads
    n = 2_000_000
    r = workloads.ConfigRunner(2, n, copies=2)
    try:
        r._alloc_out(4, [1])  # 32 groups do not fit: first finalize fails, runner retries larger
        for k in range(2):
            r.step(k)
            keys, aggs = r.results_host()
            cols = oracle.datagen(2, n, start=k * n)
            ok, oa = oracle_aggregate([cols["AdvEngineID"]], [("count", None)],
                                      (cmp(0, "<>", 0), [cols["AdvEngineID"]]), threads=8)
            assert_results_equal(keys, aggs, ok, oa)
            r._alloc_out(4, [1])
    finally:
        r.close()


@pytest.mark.parametrize("cfg_rows", [(2, 3_000_000)])
def test_fixed_exchange_two_partials_merge(cfg_rows):
    """dbg_agg_export_fixed -> concatenated buffers (what the RCCL all-gather produces) ->
    dbg_agg_merge_fixed -> finalize: equals one aggregation over both partials' rows.  Also an
    undersized buffer must make the merging finalize fail (never a silent partial result)."""
    import torch
    from databend_amd import workloads
    from databend_amd.exchange import fixed_capacity
    cfg, n = cfg_rows
    runners = [workloads.ConfigRunner(cfg, n, start=r * n) for r in range(2)]
    final = AggregateHashTable(runners[0].params, HashTableConfig(False))
    try:
        cap = fixed_capacity(runners[0].table)
        w = runners[0].table.record_width()
        out = torch.empty(2 * (cap + 1) * w, dtype=torch.uint8, device="cuda")
        for r, rn in enumerate(runners):
            rn.insert(0)
            rn.table.export_fixed(out[r * (cap + 1) * w:(r + 1) * (cap + 1) * w], cap)
        final.merge_fixed(out, 2, cap)
        blk = final.merge_result()
        cols = oracle.datagen(cfg, 2 * n)
        shape = workloads.SHAPES[cfg]
        name, op, const = shape.predicate
        ok, oa = oracle_aggregate([cols[k] for k in shape.keys], [(f, cols[c] if c else None) for f, c in shape.aggs],
                                  (cmp(0, op, const), [cols[name]]), threads=8)
        na = len(shape.aggs)
        assert_results_equal(blk.columns[na:], blk.columns[:na], ok, oa)
        # 32 groups into 8-record buffers: flagged incomplete
        final.reset()
        small = torch.empty(2 * 9 * w, dtype=torch.uint8, device="cuda")
        for r, rn in enumerate(runners):
            rn.insert(0)
            rn.table.export_fixed(small[r * 9 * w:(r + 1) * 9 * w], 8)
        final.merge_fixed(small, 2, 8)
        from databend_amd.ffi import DbgError
        with pytest.raises(DbgError):
            final.merge_result()
    finally:
        final.close()
        for rn in runners:
            rn.close()


@pytest.mark.parametrize("mode", ["single", "dual"])
@pytest.mark.parametrize("cfg,n", [(2, 2_000_000), (3, 500_000), (5, 500_000)])
def test_pipelined_batches_match_oracle(cfg, n, mode):
    """ConfigRunner.pipe_step: batch k's finalize (dbg_agg_finalize_into_async) is still in flight
    when batch k+1's insert is enqueued into the other table; each batch's published result,
    delivered by the next pipe_step (or pipe_drain for the last), equals the oracle over that
    batch's rows alone."""
    from databend_amd import workloads
    shape = workloads.SHAPES[cfg]
    r = workloads.ConfigRunner(cfg, n, copies=3)
    try:
        r.enable_pipeline(mode)
        got = []
        for k in range(4):
            r.pipe_step(k)
            if k:
                got.append(r.results_host())
        r.pipe_drain()
        got.append(r.results_host())
        for k, (keys, aggs) in enumerate(got):
            cols = oracle.datagen(cfg, n, start=(k % 3) * n)
            filt = None
            if shape.predicate:
                name, op, const = shape.predicate
                filt = (cmp(0, op, const), [cols[name]])
            ok, oa = oracle_aggregate([cols[c] for c in shape.keys],
                                      [(f, cols[c] if c else None) for f, c in shape.aggs], filt, threads=8)
            assert_results_equal(keys, aggs, ok, oa)
    finally:
        r.close()


PART_CASES = [
    # (key type, distinct keys, rows, capacity hint, batches)
    ("i64", 600_000, 3_000_000, 1 << 20, 2),      # slices hold every group (load ~0.3)
    ("i64", 1_500_000, 3_000_000, 1 << 19, 1),    # cap 2^20 too small: overflow records + growth
    ("i32", 400_000, 3_300_000, 1 << 19, 3),
    ("i16", 65_536, 2_000_000, 1 << 19, 1),       # every i16 value, including -1 (all-ones key)
    ("u8", 256, 1_200_000, 1 << 19, 1),
    ("i64", 600_000, 3_000_000, 1 << 26, 2),      # cap 2^27: two radix passes (8 + 7 bits); batch 2 into a used table
    ("i64", 700_000, 2_000_000, 1 << 28, 1),      # cap 2^29: three radix passes (6 + 6 + 5 bits)
]


@pytest.mark.parametrize("kind,distinct,n,hint,batches", PART_CASES, ids=lambda x: str(x))
def test_partitioned_insert(kind, distinct, n, hint, batches):
    """part.hip: radix-partitioned COUNT(*) insert (the LSD radix partition of mixed keys + one
    workgroup per 64 KB table slice in LDS).  Every batch holds >= 2^20 rows (the path's threshold); the
    sentinel key (all-ones), runs that leave a slice (overflow records -> agg_retry), growth,
    and several batches into one table are all covered."""
    rng = np.random.default_rng(distinct)
    t = {"i64": col.Int64, "i32": col.Int32, "i16": col.Int16, "u8": col.UInt8}[kind]
    if kind == "i64":
        pool = rng.integers(-2**63, 2**63 - 1, distinct, dtype=np.int64)
        pool[0] = -1  # packs to the EMPTY entry: sentinel slot
    elif kind == "i32":
        pool = rng.integers(-2**31, 2**31 - 1, distinct, dtype=np.int64)
        pool[0] = -1
    elif kind == "i16":
        pool = np.arange(-2**15, 2**15, dtype=np.int64)
    else:
        pool = np.arange(0, 256, dtype=np.int64)
    vals = pool[rng.integers(0, len(pool), n)]
    key = Column.from_numbers(t, vals.astype(t.np_dtype))
    g = check_parity([key], [("count", None)], on_device=True, capacity_hint=hint, batches=batches)
    assert g == len(np.unique(vals))


def _i128_column(rng, n, p, s, nullable):
    """Decimal128(p, s) values spanning the full 128-bit range of precision p (|v| < 10^p)."""
    lim = 10**p - 1
    small = rng.integers(-10**6, 10**6, n)
    vals = []
    for i in range(n):
        r = i % 7
        if r == 0:
            vals.append(lim - int(small[i] % 1000))
        elif r == 1:
            vals.append(-lim + int(small[i] % 1000))
        elif r == 2:
            vals.append(int(small[i]) * (1 << 64) + int(small[i] % 97))  # hi words differ, lo small
        else:
            vals.append(int(small[i]))
    valid = rng.random(n) > 0.2 if nullable else None
    if valid is not None:
        vals = [v if ok else None for v, ok in zip(vals, valid)]
    return Column.from_decimals(p, s, vals, validity=valid)


@pytest.mark.parametrize("groups,strategy", [(3, abi.STRATEGY_AUTO), (5000, abi.STRATEGY_AUTO),
                                             (200_000, abi.STRATEGY_PARTITIONED)],
                         ids=["hot-lds", "table", "partitioned"])
@pytest.mark.parametrize("nullable", [False, True])
def test_decimal128_wide_min_max(groups, strategy, nullable):
    """MIN/MAX of Decimal128 with precision > 18 (FUN/aggregate_min_max_any.rs:46-115): full
    128-bit order (hi signed, lo unsigned) through the seqlocked [seq, lo, hi] state — three
    groups put every row of a workgroup on the same LDS state (maximum contention), and the
    partitioned engine and the merge of exported records see the same states."""
    rng = np.random.default_rng(groups)
    n = 600_000 if groups < 100_000 else 2_400_000
    d = _i128_column(rng, n, 38, 4, nullable)
    k = Column.from_numbers(col.Int64, rng.integers(0, groups, n))
    aggs = [("min", d), ("max", d), ("count", d), ("sum", d)]
    check_parity([k], aggs, on_device=True, strategy=strategy)
    check_parity([k], [("max", d), ("min", d)], batches=3)


def test_decimal128_wide_min_max_exchange_merge():
    """The 3-word MIN/MAX state crosses dbg_agg_export_records -> dbg_agg_merge_records intact."""
    torch = _torch()
    rng = np.random.default_rng(3)
    n = 300_000
    d = _i128_column(rng, n, 30, 2, True)
    k = Column.from_numbers(col.Int32, rng.integers(0, 20_000, n))
    fns = [F.get("min", [], [d.dtype]), F.get("max", [], [d.dtype])]
    params = AggregatorParams([k.dtype], fns)
    final = AggregateHashTable(params, HashTableConfig(False))
    parts = []
    try:
        for lo, hi in ((0, n // 2), (n // 2, n)):
            p = AggregateHashTable(params, HashTableConfig(True))
            p.add_groups([slice_col(k, lo, hi)], [slice_col(d, lo, hi)] * 2)
            counts, sb = p.partition(4, 0)
            w = p.record_width()
            recs = torch.empty(max(1, sum(counts) * w), dtype=torch.uint8, device="cuda")
            strs = torch.empty(max(1, sum(sb)), dtype=torch.uint8, device="cuda")
            p.export_records(recs, strs)
            final.merge_records(recs, strs, counts, sb)
            parts.append(p)
        blk = final.merge_result()
    finally:
        final.close()
        for p in parts:
            p.close()
    ok, oa = oracle_aggregate([k], [("min", d), ("max", d)])
    assert_results_equal(blk.columns[2:], blk.columns[:2], ok, oa)


def test_filter_executor_take_strings_and_decimals():
    """FilterExecutor.filter on a device block with String (nullable), Decimal128 and Int16
    columns: dbg_filter_select + dbg_take_string / dbg_take_fixed equal numpy's take."""
    torch = _torch()
    from databend_amd.device import DeviceColumn
    from databend_amd.filter import FilterExecutor
    rng = np.random.default_rng(17)
    n = 500_001
    words = ["", "a", "bb", "search phrase %d" % 7, "x" * 40]
    sv = [words[i] for i in rng.integers(0, len(words), n)]
    svalid = rng.random(n) > 0.1
    s = Column.from_strings(sv, validity=svalid)
    d = Column.from_decimals(38, 3, [int(x) * (1 << 70) + 5 for x in rng.integers(-1000, 1000, n)])
    k = Column.from_numbers(col.Int16, rng.integers(-5, 5, n))
    dev = [DeviceColumn.from_host(c) for c in (s, d, k)]
    ex = FilterExecutor(and_(cmp(0, "<>", ""), cmp(1, ">", 0)), [0, 1])
    out = ex.filter(dev, n)
    torch.cuda.synchronize()
    dv = np.array(i128_vals := d.values(), dtype=object)
    keep = np.array([svalid[i] and sv[i] != "" and i128_vals[i] > 0 for i in range(n)])
    idx = np.nonzero(keep)[0]
    hs = out[0].to_host()
    got_s = [bytes(hs.data[int(hs.offsets[j]):int(hs.offsets[j + 1])]) for j in range(len(idx))]
    assert got_s == [sv[i].encode() for i in idx]
    assert np.array_equal(out[1].data.cpu().numpy(), d.data.reshape(-1, 16)[idx].reshape(-1))
    assert np.array_equal(out[2].data.cpu().numpy().view(np.int16), k.data[idx])
    vb = np.unpackbits(out[0].validity.cpu().numpy(), bitorder="little")[:len(idx)]
    assert vb.all()
    del dv
