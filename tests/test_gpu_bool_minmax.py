"""MIN / MAX of Boolean arguments on the GPU (MinMaxAnyState<BooleanType>,
FUN/aggregate_min_max_any.rs:116-150 — `with_simple_no_number_mapped_type` maps Boolean to its own
state; the result type is the argument's): false < true, NULL arguments skipped, an all-NULL group
NULL (OrNull).  Checked against the oracle on the HBM table and on the partitioned payload, and
through the borsh `Serialized` form (Option<bool> = tag byte + value byte) and its re-ingest.
No reference fixture holds a Boolean MIN/MAX, so the expected values are the oracle's restatement
of the state (parity against the restated semantics)."""
import numpy as np
import pytest

from databend_amd import abi
from databend_amd import column as col
from databend_amd.aggregates import AggregateFunctionFactory
from databend_amd.aggregator import AggregateHashTable, AggregatorParams, HashTableConfig
from databend_amd.column import Column
from tests.parity import assert_results_equal
from tests.test_gpu_parity import check_parity, oracle_aggregate

pytestmark = pytest.mark.gpu
F = AggregateFunctionFactory.instance()


def _inputs(rng, n, groups):
    g = rng.integers(0, groups, n)
    k = Column.from_numbers(col.Int32, g)
    b = Column.from_bools(rng.random(n) < 0.5)
    # mostly true, some groups never see false; nullable with one all-NULL group
    bn_vals = rng.random(n) < 0.97
    bn_valid = (rng.random(n) < 0.8) & (g != 5)
    bn = Column.from_bools(bn_vals, validity=bn_valid)
    return k, b, bn


@pytest.mark.parametrize("strategy", [abi.STRATEGY_AUTO, abi.STRATEGY_PARTITIONED])
@pytest.mark.parametrize("on_device", [False, True])
@pytest.mark.parametrize("groups", [6, 3000])
def test_bool_min_max_parity(strategy, on_device, groups):
    rng = np.random.default_rng(groups + 7)
    n = 300_000
    k, b, bn = _inputs(rng, n, groups)
    aggs = [("min", b), ("max", b), ("min", bn), ("max", bn), ("count", bn), ("count", None)]
    ng = check_parity([k], aggs, on_device=on_device, strategy=strategy)
    assert ng == groups


def test_bool_min_max_serialized_roundtrip():
    rng = np.random.default_rng(9)
    n = 100_000
    k, b, bn = _inputs(rng, n, 500)
    specs = [("min", b), ("max", bn), ("count", None)]
    fns = [F.get(fn, [], [c.dtype] if c is not None else []) for fn, c in specs]
    params = AggregatorParams([k.dtype], fns)
    ht = AggregateHashTable(params, HashTableConfig(True))
    try:
        ht.add_groups([k], [c for _, c in specs])
        blk = ht.result_serialized()
    finally:
        ht.close()
    ns = len(specs)
    keys = blk.columns[ns].data
    ok, oa = oracle_aggregate([k], [("min", b), ("max", bn)], threads=8)
    order = {int(x): i for i, x in enumerate(ok[0].data)}
    mins, maxs = oa[0].values(), oa[1].values()
    for g, key in enumerate(keys):
        i = order[int(key)]
        raw0 = bytes(blk.columns[0].data[int(blk.columns[0].offsets[g]):int(blk.columns[0].offsets[g + 1])])
        assert raw0 == b"\x01" + bytes([int(mins[i])]) + b"\x01", (key, raw0.hex())
        raw1 = bytes(blk.columns[1].data[int(blk.columns[1].offsets[g]):int(blk.columns[1].offsets[g + 1])])
        exp1 = (b"\x00" + b"\x00" if maxs[i] is None else b"\x01" + bytes([int(maxs[i])]) + b"\x01") + b"\x01"
        assert raw1 == exp1, (key, raw1.hex())
    # re-ingest (batch_merge) into a final table: the same results as aggregating the rows
    final = AggregateHashTable(params, HashTableConfig(False))
    try:
        final.merge_serialized(blk.columns[:ns], blk.columns[ns:])
        gk, ga = _result(final, ns)
    finally:
        final.close()
    ok, oa = oracle_aggregate([k], specs, threads=8)
    assert_results_equal(gk, ga, ok, oa)


def _result(table, n_aggs):
    blk = table.merge_result()
    return blk.columns[n_aggs:], blk.columns[:n_aggs]
