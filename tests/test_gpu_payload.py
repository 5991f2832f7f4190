"""GPU parity of the before-partial shuffle primitives (dbg_agg_payload_counts / export / import,
dbg_agg_exchange_payload) against the oracle.  Two ranks are simulated on one GPU by two
partitioned-mode handles: each exports its level-1 records for 2 ranks, the blocks are routed the
way exchange_payload's all-to-all routes them, each imports its share and finalizes — the union of
the two results equals one aggregation of all rows and the group sets are disjoint (one owner per
level-1 partition).  The RCCL collective itself runs at world size 1 (self send/recv)."""
import numpy as np
import pytest

from databend_amd import abi
from databend_amd import column as col
from databend_amd.aggregates import AggregateFunctionFactory
from databend_amd.aggregator import AggregateHashTable, AggregatorParams, HashTableConfig
from databend_amd.column import Column
from databend_amd.device import DeviceColumn
from databend_amd.exchange import payload_owned, payload_splits
from tests.parity import assert_results_equal
from tests.test_gpu_parity import oracle_aggregate

pytestmark = pytest.mark.gpu
F = AggregateFunctionFactory.instance()


def _data(seed, n):
    rng = np.random.default_rng(seed)
    watch = rng.integers(0, 3 * n, n)  # mostly unique, some repeats
    ip = rng.integers(0, 1000, n).astype(np.int32)
    refresh = (rng.random(n) < 0.1).astype(np.int16)
    width = rng.integers(0, 2561, n).astype(np.int16)
    return [Column.from_numbers(col.Int64, watch), Column.from_numbers(col.Int32, ip)], \
        [("count", None), ("sum", Column.from_numbers(col.Int16, refresh)), ("sum", Column.from_numbers(col.Int16, width)),
         ("avg", Column.from_numbers(col.Int16, width))]


def _table(keys, aggs, batches=1):
    fns = [F.get(n, [], [c.dtype] if c is not None else []) for n, c in aggs]
    t = AggregateHashTable(AggregatorParams([k.dtype for k in keys], fns), HashTableConfig(True))
    t.set_strategy(abi.STRATEGY_PARTITIONED)
    n = len(keys[0])
    bounds = np.linspace(0, n, batches + 1).astype(int)
    from tests.test_gpu_parity import slice_col
    for b in range(batches):
        lo, hi = int(bounds[b]), int(bounds[b + 1])
        ks = [DeviceColumn.from_host(slice_col(k, lo, hi)) for k in keys]
        ars = [None if c is None else DeviceColumn.from_host(slice_col(c, lo, hi)) for _, c in aggs]
        t.add_groups(ks, ars, rows=hi - lo, on_device=True)
    return t


def _result(t, na):
    block = t.merge_result()
    return block.columns[na:], block.columns[:na]


def _cat(a, b):
    """Row concatenation of two numeric Columns (either may carry validity)."""
    v = None
    if a.validity is not None or b.validity is not None:
        va = a.validity if a.validity is not None else np.ones(len(a), bool)
        vb = b.validity if b.validity is not None else np.ones(len(b), bool)
        v = np.concatenate([va, vb])
    dt = a.dtype if v is None else a.dtype.wrap_nullable()
    return Column(dt, np.concatenate([a.data, b.data]), None, v)


def test_payload_self_roundtrip():
    import torch
    keys, aggs = _data(1, 300_000)
    t = _table(keys, aggs, batches=3)
    counts, widths = t.payload_counts()
    assert int(counts[0].sum()) == 300_000 and int(counts[1].sum()) == 0
    send, recv = payload_splits(counts, counts[None], widths, 0, 1)
    buf = torch.empty(max(1, sum(send[0]) + sum(send[1])), dtype=torch.uint8, device="cuda")
    t.payload_export(1, buf)
    raw = buf[:sum(send[0])].clone()
    t.payload_import(1, 0, counts[None], raw, buf[:1])
    gk, ga = _result(t, len(aggs))
    t.close()
    ok, oa = oracle_aggregate(keys, aggs)
    assert_results_equal(gk, ga, ok, oa)


def test_payload_two_ranks_on_one_gpu():
    import torch
    (k0, a0), (k1, a1) = _data(2, 250_000), _data(3, 200_000)
    # the second rank shares half of its keys with the first
    k1[0].data[:100_000] = k0[0].data[:100_000]
    k1[1].data[:100_000] = k0[1].data[:100_000]
    tabs = [_table(k0, a0, 2), _table(k1, a1, 1)]
    cw = [t.payload_counts() for t in tabs]
    all_counts = np.stack([c for c, _ in cw])
    widths = cw[0][1]
    bufs, splits = [], []
    for r, t in enumerate(tabs):
        send, recv = payload_splits(cw[r][0], all_counts, widths, r, 2)
        b = torch.empty(max(1, sum(send[0]) + sum(send[1])), dtype=torch.uint8, device="cuda")
        t.payload_export(2, b)
        bufs.append(b)
        splits.append(send)
    torch.cuda.synchronize()
    for r, t in enumerate(tabs):  # what the all-to-all delivers: source-major blocks per kind
        got = []
        for k in range(2):
            parts = []
            for s in range(2):
                base = 0 if k == 0 else sum(splits[s][0])
                off = base + sum(splits[s][k][:r])
                parts.append(bufs[s][off:off + splits[s][k][r]])
            got.append(torch.cat(parts) if sum(x.numel() for x in parts) else torch.empty(1, dtype=torch.uint8, device="cuda"))
        t.payload_import(2, r, all_counts, got[0], got[1])
    res = [_result(t, len(a0)) for t in tabs]
    for t in tabs:
        t.close()
    keys = [_cat(k0[i], k1[i]) for i in range(2)]
    aggs = [(n, None if c is None else _cat(c, a1[j][1])) for j, (n, c) in enumerate(a0)]
    ok, oa = oracle_aggregate(keys, aggs)
    gk = [_cat(res[0][0][i], res[1][0][i]) for i in range(2)]
    ga = [_cat(res[0][1][j], res[1][1][j]) for j in range(len(aggs))]
    assert_results_equal(gk, ga, ok, oa)
    s0 = set(zip(res[0][0][0].values(), res[0][0][1].values()))
    s1 = set(zip(res[1][0][0].values(), res[1][0][1].values()))
    assert not (s0 & s1) and s0 and s1


def test_exchange_payload_rccl_world_1():
    from databend_amd.exchange import AbiComm
    keys, aggs = _data(4, 200_000)
    t = _table(keys, aggs)
    comm = AbiComm(AbiComm.unique_id(), 1, 0, 0)
    st = comm.exchange_payload(t)
    assert st["remote_bytes"] == 0 and st["received_records"] == 200_000
    gk, ga = _result(t, len(aggs))
    t.close()
    comm.close()
    ok, oa = oracle_aggregate(keys, aggs)
    assert_results_equal(gk, ga, ok, oa)


def test_payload_chunked_import_two_ranks_on_one_gpu():
    """the chunked primitives (counts / export from a segment, import of several chunks): each
    rank's batches shipped one at a time, routed like the all-to-all, imported as chunks."""
    import torch
    (k0, a0), (k1, a1) = _data(12, 240_000), _data(13, 180_000)
    k1[0].data[:90_000] = k0[0].data[:90_000]
    k1[1].data[:90_000] = k0[1].data[:90_000]
    from tests.test_gpu_parity import slice_col
    fns = [F.get(n, [], [c.dtype] if c is not None else []) for n, c in a0]
    tabs = []
    for keys in (k0, k1):
        t = AggregateHashTable(AggregatorParams([k.dtype for k in keys], fns), HashTableConfig(True))
        t.set_strategy(abi.STRATEGY_PARTITIONED)
        tabs.append(t)
    data = [(k0, a0), (k1, a1)]
    first = [(0, 0), (0, 0)]
    chunks = [[], []]  # per destination rank: (all_counts, raw, state) per chunk
    for c in range(3):  # three add_groups chunks per rank, each shipped before the next is added
        cws, bufs, splits = [], [], []
        for r, t in enumerate(tabs):
            keys, aggs = data[r]
            n = len(keys[0])
            lo, hi = n * c // 3, n * (c + 1) // 3
            t.add_groups([DeviceColumn.from_host(slice_col(k, lo, hi)) for k in keys],
                         [None if x is None else DeviceColumn.from_host(slice_col(x, lo, hi)) for _, x in aggs],
                         rows=hi - lo, on_device=True)
            cws.append(t.payload_counts_from(first[r]))
        all_counts = np.stack([cw[0] for cw in cws])
        widths = cws[0][1]
        for r, t in enumerate(tabs):
            send, recv = payload_splits(cws[r][0], all_counts, widths, r, 2)
            b = torch.empty(max(1, sum(send[0]) + sum(send[1])), dtype=torch.uint8, device="cuda")
            t.payload_export_from(2, first[r], b)
            bufs.append(b)
            splits.append(send)
            first[r] = cws[r][2]
        torch.cuda.synchronize()
        for r in range(2):
            got = []
            for k in range(2):
                parts = []
                for s in range(2):
                    base = 0 if k == 0 else sum(splits[s][0])
                    off = base + sum(splits[s][k][:r])
                    parts.append(bufs[s][off:off + splits[s][k][r]].clone())
                got.append(torch.cat(parts) if sum(x.numel() for x in parts) else None)
            chunks[r].append((all_counts, got[0], got[1]))
    for r, t in enumerate(tabs):
        cc = np.stack([x[0] for x in chunks[r]])
        t.payload_import_chunks(2, r, cc, [x[1] for x in chunks[r]], [x[2] for x in chunks[r]])
    res = [_result(t, len(a0)) for t in tabs]
    for t in tabs:
        t.close()
    keys = [_cat(k0[i], k1[i]) for i in range(2)]
    aggs = [(n, None if c is None else _cat(c, a1[j][1])) for j, (n, c) in enumerate(a0)]
    ok, oa = oracle_aggregate(keys, aggs)
    gk = [_cat(res[0][0][i], res[1][0][i]) for i in range(2)]
    ga = [_cat(res[0][1][j], res[1][1][j]) for j in range(len(aggs))]
    assert_results_equal(gk, ga, ok, oa)
    s0 = set(zip(res[0][0][0].values(), res[0][0][1].values()))
    s1 = set(zip(res[1][0][0].values(), res[1][0][1].values()))
    assert not (s0 & s1) and s0 and s1


def test_exchange_payload_chunk_rccl_world_1():
    """dbg_agg_exchange_payload_chunk at world size 1: three add_groups chunks, each shipped (self
    send / receive on the communicator's stream) before the next is added, the last call importing."""
    from databend_amd.exchange import AbiComm
    from tests.test_gpu_parity import slice_col
    keys, aggs = _data(14, 300_000)
    fns = [F.get(n, [], [c.dtype] if c is not None else []) for n, c in aggs]
    t = AggregateHashTable(AggregatorParams([k.dtype for k in keys], fns), HashTableConfig(True))
    t.set_strategy(abi.STRATEGY_PARTITIONED)
    comm = AbiComm(AbiComm.unique_id(), 1, 0, 0)
    received = 0
    for c in range(3):
        lo, hi = 100_000 * c, 100_000 * (c + 1)
        t.add_groups([DeviceColumn.from_host(slice_col(k, lo, hi)) for k in keys],
                     [None if x is None else DeviceColumn.from_host(slice_col(x, lo, hi)) for _, x in aggs],
                     rows=hi - lo, on_device=True)
        st = comm.exchange_payload_chunk(t, last=(c == 2))
        assert st["remote_bytes"] == 0
        received += st["received_records"]
    assert received == 300_000
    gk, ga = _result(t, len(aggs))
    t.close()
    comm.close()
    ok, oa = oracle_aggregate(keys, aggs)
    assert_results_equal(gk, ga, ok, oa)


def test_payload_shuffle_finish_ships_late_chunks_world_1():
    """exchange.PayloadShuffle over torch.distributed (RCCL, world 1) on a real partitioned table:
    chunk 0 shipped, chunks 1 and 2 added after the last ship() — finish() must ship them (the
    library's last=1 does the same), so the result is every row's aggregation."""
    import os
    import socket

    import torch
    import torch.distributed as dist
    from databend_amd.exchange import PayloadShuffle
    from tests.test_gpu_parity import slice_col
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    keys, aggs = _data(15, 300_000)
    fns = [F.get(n, [], [c.dtype] if c is not None else []) for n, c in aggs]
    t = AggregateHashTable(AggregatorParams([k.dtype for k in keys], fns), HashTableConfig(True))
    t.set_strategy(abi.STRATEGY_PARTITIONED)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    try:
        sh = PayloadShuffle(t, torch.device("cuda", torch.cuda.current_device()))
        for c in range(3):
            lo, hi = 100_000 * c, 100_000 * (c + 1)
            t.add_groups([DeviceColumn.from_host(slice_col(k, lo, hi)) for k in keys],
                         [None if x is None else DeviceColumn.from_host(slice_col(x, lo, hi)) for _, x in aggs],
                         rows=hi - lo, on_device=True)
            if c == 0:
                sh.ship()
        sh.finish()
        torch.cuda.synchronize()
        gk, ga = _result(t, len(aggs))
    finally:
        t.close()
        dist.destroy_process_group()
    ok, oa = oracle_aggregate(keys, aggs)
    assert_results_equal(gk, ga, ok, oa)
