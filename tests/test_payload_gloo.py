"""The before-partial shuffle protocol (databend_amd.exchange.exchange_payload: the splits, the
count all-gather, one all_to_all_single per record kind, the import layout) at world sizes 2, 3
and 4 on CPU with gloo.  Each rank's table is a stand-in holding records tagged (source rank,
level-1 partition, serial) in the library's payload order (export: destination-major, partition-
major); after the exchange every rank must hold exactly the records of the partitions it owns
(p * world // 256 == rank), source-major and partition-major within a source — the layout
dbg_agg_payload_import turns into level-1 segments."""
import os
import socket

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class FakePayload:
    """payload_counts / export / import over CPU tensors; records are 8 bytes (raw) or 16 bytes
    (state): [src << 40 | part << 24 | serial] (+ a second word for state records)."""

    def __init__(self, rank, seed):
        rng = np.random.default_rng(seed)
        self.rank = rank
        self.counts = rng.integers(0, 40, (2, 256)).astype(np.uint64)
        self.counts[1, rng.random(256) < 0.7] = 0
        self.widths = (8, 16)
        self.imported = None

    def rec(self, k, p, i):
        v = (self.rank << 40) | (p << 24) | i
        return [v] if k == 0 else [v, ~v & ((1 << 63) - 1)]

    def payload_counts(self):
        return self.counts.copy(), self.widths

    def payload_export(self, n, buf):
        from databend_amd.exchange import payload_owned
        words = []
        for k in range(2):
            for d in range(n):
                lo, hi = payload_owned(d, n)
                for p in range(lo, hi):
                    for i in range(int(self.counts[k][p])):
                        words += self.rec(k, p, i)
        b = np.array(words, dtype=np.uint64).view(np.uint8)
        buf[:len(b)] = __import__("torch").from_numpy(b.copy())

    def payload_import(self, n, rank, all_counts, raw, state):
        self.imported = (all_counts.copy(), raw.numpy().copy(), state.numpy().copy())


def _worker(rank, world, port, q):
    import sys
    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist
    from databend_amd.exchange import exchange_payload, payload_owned
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        t = FakePayload(rank, 100 + rank)
        exchange_payload(t, "cpu")
        all_counts, raw, state = t.imported
        lo, hi = payload_owned(rank, world)
        # expected: source-major, partition-major within a source
        for k, buf in ((0, raw), (1, state)):
            words = buf.view(np.uint64) if buf.size % 8 == 0 else buf[:buf.size // 8 * 8].view(np.uint64)
            exp = []
            for s in range(world):
                src = FakePayload(s, 100 + s)
                assert (all_counts[s] == src.counts).all()
                for p in range(lo, hi):
                    for i in range(int(src.counts[k][p])):
                        exp += src.rec(k, p, i)
            got = list(words[:len(exp)])
            assert got == exp, (rank, k)
            assert int(all_counts[:, k, lo:hi].sum()) * t.widths[k] <= buf.size
        q.put((rank, "ok"))
    except Exception as e:  # pragma: no cover - reported to the parent
        import traceback
        q.put((rank, traceback.format_exc()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 4])
def test_payload_shuffle_protocol(world):
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=240) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    assert all(v == "ok" for v in res.values()), res


class FakeChunkedPayload:
    """A payload of several level-1 segments (one per add_groups chunk): counts / export from a
    segment on, and the chunked import.  Records: [src << 40 | seg << 32 | part << 16 | serial]."""

    def __init__(self, rank, seed, n_segs):
        rng = np.random.default_rng(seed)
        self.rank = rank
        self.segs = [rng.integers(0, 12, (2, 256)).astype(np.uint64) for _ in range(n_segs)]
        for c in self.segs:
            c[1, rng.random(256) < 0.7] = 0
        self.widths = (8, 16)
        self.n_visible = 0  # segments appended so far (the test appends them one ship at a time)
        self.imported = None

    def rec(self, k, g, p, i):
        v = (self.rank << 40) | (g << 32) | (p << 16) | i
        return [v] if k == 0 else [v, ~v & ((1 << 63) - 1)]

    def payload_counts_from(self, first):
        c = np.zeros((2, 256), np.uint64)
        for k in range(2):
            for g in range(first[k], self.n_visible):
                c[k] += self.segs[g][k]
        return c, self.widths, (self.n_visible, self.n_visible)

    def payload_export_from(self, n, first, buf):
        from databend_amd.exchange import payload_owned
        words = []
        for k in range(2):
            for d in range(n):
                lo, hi = payload_owned(d, n)
                for p in range(lo, hi):
                    for g in range(first[k], self.n_visible):
                        for i in range(int(self.segs[g][k][p])):
                            words += self.rec(k, g, p, i)
        if words:
            b = np.array(words, dtype=np.uint64).view(np.uint8)
            buf[:len(b)] = __import__("torch").from_numpy(b.copy())

    def payload_import_chunks(self, n, rank, cc, raws, states):
        self.imported = (cc.copy(), [r.numpy().copy() for r in raws], [s.numpy().copy() for s in states])


def _chunk_worker(rank, world, port, q, n_segs, shipped=None):
    """`shipped`: how many segments are shipped one by one before finish() (None = all of them);
    finish() must ship the rest as one last chunk."""
    import sys
    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist
    from databend_amd.exchange import PayloadShuffle, payload_owned
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        t = FakeChunkedPayload(rank, 200 + rank, n_segs)
        sh = PayloadShuffle(t, "cpu")
        k_ship = n_segs if shipped is None else shipped
        for g in range(n_segs):  # one add_groups chunk, then (for the first k_ship) its shipment
            t.n_visible = g + 1
            if g < k_ship:
                sh.ship()
        sh.finish()
        cc, raws, states = t.imported
        # chunk j holds segment j for j < k_ship; the last chunk holds every segment after that
        groups = [[g] for g in range(k_ship)] + ([list(range(k_ship, n_segs))] if k_ship < n_segs else [])
        assert cc.shape == (len(groups), world, 2, 256)
        lo, hi = payload_owned(rank, world)
        for j, segs in enumerate(groups):  # source-major, partition-major within a source, segments in order
            for k, buf in ((0, raws[j]), (1, states[j])):
                words = buf[:buf.size // 8 * 8].view(np.uint64)
                exp = []
                for s in range(world):
                    src = FakeChunkedPayload(s, 200 + s, n_segs)
                    assert (cc[j][s] == sum(src.segs[g] for g in segs)).all()
                    for p in range(lo, hi):
                        for g in segs:
                            for i in range(int(src.segs[g][k][p])):
                                exp += src.rec(k, g, p, i)
                assert list(words[:len(exp)]) == exp, (rank, j, k)
        q.put((rank, "ok"))
    except Exception:  # pragma: no cover - reported to the parent
        import traceback
        q.put((rank, traceback.format_exc()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,shipped", [(2, None), (3, None), (4, None), (2, 1), (3, 0)])
def test_chunked_payload_shuffle_protocol(world, shipped):
    """shipped = 1: records added after the last ship() reach their owners through finish();
    shipped = 0: finish() alone shuffles (no rank keeps an unshuffled payload)."""
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_chunk_worker, args=(r, world, port, q, 3, shipped)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=240) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    assert all(v == "ok" for v in res.values()), res


def test_payload_owned_covers_every_partition_once():
    from databend_amd.exchange import payload_owned
    for n in (1, 2, 3, 4, 5, 7, 8, 16, 256):
        owner = {}
        for d in range(n):
            lo, hi = payload_owned(d, n)
            for p in range(lo, hi):
                assert p not in owner
                owner[p] = d
                assert p * n // 256 == d
        assert sorted(owner) == list(range(256))


class KeyPayload:
    """ClickBench Q17's shape (one Int64 UserID key, COUNT(*)) as the level-1 payload a
    partitioned-mode table holds: one raw record per row — the key's 8 bytes (the library's raw
    width for this shape, exchange.payload_widths: (8, 16)) — in the level-1 partition given by the
    top 8 bits of the group hash (oracle.group_hash, the restated group_hash_columns), and no state
    records.  Export: destination-major, partition-major within a destination."""

    def __init__(self, rank, seed, pool, n):
        from oracle import oracle
        from databend_amd import column as col
        from databend_amd.column import Column
        rng = np.random.default_rng(seed)
        self.keys = pool[rng.zipf(1.3, n) % len(pool)]
        h = oracle.group_hash([Column.from_numbers(col.Int64, self.keys)])
        self.part = (h >> np.uint64(56)).astype(np.int64)
        self.counts = np.zeros((2, 256), np.uint64)
        np.add.at(self.counts[0], self.part, 1)
        self.widths = (8, 16)
        self.imported = None

    def payload_counts(self):
        return self.counts.copy(), self.widths

    def payload_export(self, n, buf):
        import torch
        order = np.argsort(self.part, kind="stable")  # partition-major = destination-major
        b = self.keys[order].astype(np.int64).view(np.uint8)
        buf[:len(b)] = torch.from_numpy(b.copy())

    def payload_import(self, n, rank, all_counts, raw, state):
        self.imported = (all_counts.copy(), raw.numpy().copy())


def _q17_worker(rank, world, port, q):
    import sys
    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist
    from databend_amd.exchange import exchange_payload, payload_owned
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        pool = np.random.default_rng(5).integers(-2**63, 2**63 - 1, 20_000, dtype=np.int64)
        t = KeyPayload(rank, 300 + rank, pool, 30_000)
        exchange_payload(t, "cpu")
        all_counts, raw = t.imported
        lo, hi = payload_owned(rank, world)
        n_in = int(all_counts[:, 0, lo:hi].sum())
        got = raw[:8 * n_in].view(np.int64)
        mine = {}
        for s in range(world):  # what every source holds of this rank's partitions
            src = KeyPayload(s, 300 + s, pool, 30_000)
            sel = (src.part >= lo) & (src.part < hi)
            for k in src.keys[sel]:
                mine[int(k)] = mine.get(int(k), 0) + 1
        u, c = np.unique(got, return_counts=True)
        assert dict(zip(u.tolist(), c.tolist())) == mine, rank  # the owner's GROUP BY key, COUNT(*)
        groups = [None] * world
        dist.all_gather_object(groups, sorted(mine))
        seen = set()
        for gset in groups:  # disjoint group sets, together every key of every rank
            assert not (seen & set(gset))
            seen |= set(gset)
        every = set()
        for s in range(world):
            every |= set(KeyPayload(s, 300 + s, pool, 30_000).keys.tolist())
        assert seen == every
        q.put((rank, "ok"))
    except Exception:  # pragma: no cover - reported to the parent
        import traceback
        q.put((rank, traceback.format_exc()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 4])
def test_q17_shape_before_partial_shuffle(world):
    """C3's shape through the before-partial shuffle: every key's rows meet on the rank that owns
    its level-1 partition, so one aggregation there gives its full COUNT(*), and the ranks' group
    sets are disjoint and cover every key."""
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_q17_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=240) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    assert all(v == "ok" for v in res.values()), res


def test_prefer_before_partial_rule():
    """group_by_shuffle_mode chosen by bytes: Q17 at 8 GPUs (1.25e8 rows, ~8e7 groups per GPU)
    ships rows; Q8-like low cardinality ships groups."""
    from databend_amd.exchange import prefer_before_partial
    assert prefer_before_partial(125_000_000, 80_000_000, (8, 16))
    assert not prefer_before_partial(125_000_000, 32, (8, 16))
    assert not prefer_before_partial(1_000, 499, (8, 16)) and prefer_before_partial(1_000, 500, (8, 16))
