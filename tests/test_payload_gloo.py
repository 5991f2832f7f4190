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
