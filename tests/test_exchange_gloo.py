"""World-size-2 (and 3) exchange on CPU with the gloo backend.

Exercises databend_amd.exchange.all_to_all_bytes — the same code path the GPU ranks run over
RCCL — with partial aggregates computed by the oracle on each rank's row slice, routed by the
reference's rule (destination = group hash % world, EAGG/payload.rs:356-391), merged on the
receiving rank.  The union of the ranks' final groups must equal a single global aggregation,
and every group must live on rank hash % world.
"""
import os
import socket
import struct

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _data(n=20_000):
    rng = np.random.default_rng(42)
    words = [b"w%d" % i for i in range(3000)]
    keys_s = [words[i] for i in rng.integers(0, 3000, n)]
    keys_i = rng.integers(0, 4, n).astype(np.int64)
    vals = rng.integers(-1000, 1000, n).astype(np.int64)
    return keys_s, keys_i, vals


def _params():
    from databend_amd import column as col
    from databend_amd.aggregates import AggregateFunctionFactory
    from databend_amd.aggregator import AggregatorParams
    F = AggregateFunctionFactory.instance()
    return AggregatorParams([col.String, col.Int64], [F.get("count"), F.get("sum", [], [col.Int64])])


def _worker(rank, world, port, q):
    """Each rank: oracle partial aggregate of its slice -> records in the library's exchange layout
    (dbg_agg_record_layout: what dbg_agg_export_records writes and dbg_agg_merge_records reads)
    partitioned by hash % world -> exchange_records (the RCCL path's code, here over gloo) ->
    merge of the received records, decoded with the same layout."""
    import sys
    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist
    from databend_amd import column as col
    from databend_amd.column import Column
    from databend_amd.exchange import exchange_records
    from oracle import oracle

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        params = _params()
        L = params.record_layout()
        W, so = L.width, L.state_off
        ks, ki, vals = _data()
        n = len(ki)
        lo, hi = n * rank // world, n * (rank + 1) // world
        keys = [Column.from_strings(ks[lo:hi]), Column.from_numbers(col.Int64, ki[lo:hi])]
        v = Column.from_numbers(col.Int64, vals[lo:hi])
        fns = params.aggregate_functions
        pk, pa = oracle.aggregate(keys, [(fns[0].to_abi(), None), (fns[1].to_abi(), v)])
        h = oracle.group_hash(pk)
        dest = (h % np.uint64(world)).astype(np.int64)
        s_vals, i_vals = pk[0].values(), pk[1].values()
        c_vals, sum_vals = pa[0].values(), pa[1].values()
        rec_parts, blob_parts = [[] for _ in range(world)], [[] for _ in range(world)]
        for g in range(len(i_vals)):
            d = int(dest[g])
            off = sum(len(b) for b in blob_parts[d])
            r = bytearray(W)
            struct.pack_into("<Q", r, 0, int(h[g]))
            struct.pack_into("<QQ", r, L.key_off[0], off, len(s_vals[g]))
            struct.pack_into("<q", r, L.key_off[1], i_vals[g])
            struct.pack_into("<Q", r, so + 8 * (L.agg_w0[0] - 1), c_vals[g])
            struct.pack_into("<q", r, so + 8 * (L.agg_w0[1] - 1), sum_vals[g])
            rec_parts[d].append(bytes(r))
            blob_parts[d].append(s_vals[g])
        recs = b"".join(b"".join(p) for p in rec_parts)
        blobs = b"".join(b"".join(p) for p in blob_parts)
        rsend = torch.frombuffer(bytearray(recs or b"\0"), dtype=torch.uint8)
        bsend = torch.frombuffer(bytearray(blobs or b"\0"), dtype=torch.uint8)
        counts = [len(p) for p in rec_parts]
        sbytes = [sum(len(b) for b in p) for p in blob_parts]
        rrecv, brecv, seg_records, seg_strings = exchange_records(rsend, bsend, counts, sbytes, W, "cpu")
        rb, bb = bytes(rrecv.numpy()), bytes(brecv.numpy())
        merged = {}
        ro = bo = 0
        for src in range(world):
            for k in range(seg_records[src]):
                base = ro + k * W
                hh, = struct.unpack_from("<Q", rb, base)
                off, ln = struct.unpack_from("<QQ", rb, base + L.key_off[0])
                ik, = struct.unpack_from("<q", rb, base + L.key_off[1])
                cnt, = struct.unpack_from("<Q", rb, base + so + 8 * (L.agg_w0[0] - 1))
                sm, = struct.unpack_from("<q", rb, base + so + 8 * (L.agg_w0[1] - 1))
                sk = bb[bo + off:bo + off + ln]
                assert hh % world == rank
                e = merged.setdefault((sk, ik), [0, 0])
                e[0] += cnt
                e[1] += sm
            ro += seg_records[src] * W
            bo += seg_strings[src]
        q.put((rank, merged))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_exchange_partials_gloo(world):
    import torch.multiprocessing as mp
    from databend_amd import column as col
    from databend_amd.aggregates import AggregateFunctionFactory
    from databend_amd.column import Column
    from oracle import oracle

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = {}
    for _ in range(world):
        r, m = q.get(timeout=240)
        results[r] = m
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # disjoint group sets, union == global aggregation
    all_keys = [k for m in results.values() for k in m]
    assert len(all_keys) == len(set(all_keys))
    ks, ki, vals = _data()
    F = AggregateFunctionFactory.instance()
    gk, ga = oracle.aggregate([Column.from_strings(ks), Column.from_numbers(col.Int64, ki)],
                              [(F.get("count").to_abi(), None),
                               (F.get("sum", [], [col.Int64]).to_abi(), Column.from_numbers(col.Int64, vals))])
    exp = {(s, i): [c, sm] for s, i, c, sm in zip(gk[0].values(), gk[1].values(), ga[0].values(), ga[1].values())}
    got = {k: v for m in results.values() for k, v in m.items()}
    assert got == exp


def _worker_fixed(rank, world, port, q):
    """Replicas + gather (the low-cardinality route of bench.py / exchange.gather_small): each
    rank packs its partial groups into an equal-size buffer with the group count in record 0,
    one all-gather moves them, the root merges."""
    import sys
    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist
    from databend_amd import column as col
    from databend_amd.aggregates import AggregateFunctionFactory
    from databend_amd.column import Column
    from databend_amd.exchange import all_gather_fixed
    from oracle import oracle

    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rng = np.random.default_rng(7)
        n = 50_000
        adv = np.where(rng.random(n) < 0.99, 0, rng.integers(1, 33, n)).astype(np.int16)
        lo, hi = n * rank // world, n * (rank + 1) // world
        F = AggregateFunctionFactory.instance()
        pk, pa = oracle.aggregate([Column.from_numbers(col.Int16, adv[lo:hi])], [(F.get("count").to_abi(), None)])
        h = oracle.group_hash(pk)
        cap, w = 64, 24
        buf = bytearray((cap + 1) * w)
        g = len(pk[0])
        struct.pack_into("<QQ", buf, 0, g, 0)
        for j, (k, c) in enumerate(zip(pk[0].values(), pa[0].values())):
            struct.pack_into("<QqQ", buf, (1 + j) * w, int(h[j]), int(k), int(c))
        send = torch.frombuffer(buf, dtype=torch.uint8)
        out = torch.empty(world * len(buf), dtype=torch.uint8)
        all_gather_fixed(send, out)
        merged = {}
        if rank == 0:
            ob = bytes(out.numpy())
            for r in range(world):
                base = r * len(buf)
                cnt, flags = struct.unpack_from("<QQ", ob, base)
                assert flags == 0 and cnt <= cap
                for j in range(cnt):
                    hh, k, c = struct.unpack_from("<QqQ", ob, base + (1 + j) * w)
                    merged[k] = merged.get(k, 0) + c
        q.put((rank, merged))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_fixed_gather_gloo(world):
    import torch.multiprocessing as mp
    from databend_amd import column as col
    from databend_amd.aggregates import AggregateFunctionFactory
    from databend_amd.column import Column
    from oracle import oracle

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker_fixed, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = {}
    for _ in range(world):
        r, m = q.get(timeout=240)
        results[r] = m
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    rng = np.random.default_rng(7)
    n = 50_000
    adv = np.where(rng.random(n) < 0.99, 0, rng.integers(1, 33, n)).astype(np.int16)
    F = AggregateFunctionFactory.instance()
    gk, ga = oracle.aggregate([Column.from_numbers(col.Int16, adv)], [(F.get("count").to_abi(), None)])
    exp = {int(k): int(c) for k, c in zip(gk[0].values(), ga[0].values())}
    assert results[0] == exp
    assert all(results[r] == {} for r in range(1, world))
