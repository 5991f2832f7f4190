"""Multi-GPU exchange of partial aggregate states over torch.distributed (RCCL over xGMI).

Replaces Databend's cluster shuffle for the final-merge stage:
the reference routes every partial group to node `hash % n` (EAGG/payload.rs:356-391,
AGG/aggregate_exchange_injector.rs:154-235) and ships borsh-serialized states over Arrow Flight.
Here each rank exports its partial table as fixed-width records partitioned by the same
`hash % world` rule (dbg_agg_partition / dbg_agg_export_records), then

  1. all_to_all of the per-destination record/blob sizes (one small collective),
  2. all_to_all_single of the record bytes and of the string blobs (RCCL, uneven splits),
  3. merge of the received segments into this rank's final table (dbg_agg_merge_records).

Group sets of the ranks are disjoint afterwards (like the reference's per-node finals).  One
process per GPU; `backend="nccl"` is RCCL on ROCm.  `all_to_all_bytes` is backend-agnostic and
is exercised with gloo on CPU by the tests.

Low cardinality (a partial table of a few thousand slots at most, fixed-width keys) takes the
replicas + gather route of SURVEY.md §8e instead (`gather_small`): every rank writes its groups
into an equal-size buffer whose group count stays on the device (dbg_agg_export_fixed), one RCCL
all-gather moves the buffers, and the root merges them (dbg_agg_merge_fixed) — no host round
trip and no size exchange, which at these sizes would cost more than the data.
"""
from __future__ import annotations

from typing import List, Sequence, Tuple


def _dist():
    import torch.distributed as dist
    return dist


def all_to_all_counts(counts: Sequence[int], device) -> List[int]:
    """Every rank sends counts[d] to rank d; returns what each source sent to this rank."""
    import torch
    dist = _dist()
    send = torch.tensor(list(counts), dtype=torch.int64, device=device)
    recv = torch.empty_like(send)
    dist.all_to_all_single(recv, send)
    return [int(x) for x in recv.tolist()]


def all_to_all_bytes(send, send_splits: Sequence[int], device) -> Tuple["object", List[int]]:
    """Uneven all-to-all of a uint8 tensor: send[sum(send_splits[:d]) : ...] goes to rank d.
    Returns (received bytes ordered by source rank, per-source byte counts)."""
    import torch
    dist = _dist()
    recv_splits = all_to_all_counts(send_splits, device)
    recv = torch.empty(max(1, sum(recv_splits)), dtype=torch.uint8, device=device)
    out = recv[:sum(recv_splits)] if sum(recv_splits) else recv[:0]
    inp = send[:sum(send_splits)] if sum(send_splits) else send[:0]
    dist.all_to_all_single(out, inp, output_split_sizes=list(recv_splits), input_split_sizes=list(send_splits))
    return recv, recv_splits


def exchange_records(recs, strs, counts: Sequence[int], sbytes: Sequence[int], width: int, device):
    """All-to-all of partition-major exchange records (dbg_agg_export_records layout) and their
    string blobs: counts[d] records / sbytes[d] blob bytes go to rank d.  ONE collective carries
    both size vectors (the only host round trip), then the record and blob bytes move with one
    all_to_all_single each.  Returns (records, blobs, per-source record counts, per-source blob bytes)."""
    world = _dist().get_world_size()
    return _exchange_with_sizes(recs, strs, counts, sbytes, width, device, world)


def merge_splits(counts, sbytes, got_pairs, width: int):
    """Byte plan of the before_merge exchange on one rank (the plan dbg_agg_exchange follows,
    dbg_merge_exchange_plan): counts[d] / sbytes[d] are this rank's records / blob bytes for rank d,
    got_pairs[s] = (records, blob bytes) source s sends this rank.  Returns (record send splits,
    blob send splits, record receive splits, blob receive splits, per-source record counts), in
    bytes except the last; send order is export (partition-major) order, receive order is source
    order — the order dbg_agg_merge_records takes its segments in."""
    send_r = [int(c) * width for c in counts]
    send_s = [int(b) for b in sbytes]
    seg_records = [int(c) for c, _ in got_pairs]
    recv_r = [c * width for c in seg_records]
    recv_s = [int(b) for _, b in got_pairs]
    return send_r, send_s, recv_r, recv_s, seg_records


def _exchange_with_sizes(recs, strs, counts, sbytes, width, device, world):
    import torch
    dist = _dist()
    # [c_0, s_0, c_1, s_1, ...]: the pair for destination d is contiguous, so an even all-to-all
    # (2 int64 per peer) delivers each source's pair
    pairs = torch.tensor([x for d in range(world) for x in (counts[d], sbytes[d])], dtype=torch.int64, device=device)
    got = torch.empty_like(pairs)
    dist.all_to_all_single(got, pairs)
    got = got.view(world, 2).tolist()
    send_r, send_s, recv_r, seg_strings, seg_records = merge_splits(counts, sbytes, got, width)
    rrecv = torch.empty(max(1, sum(recv_r)), dtype=torch.uint8, device=device)
    srecv = torch.empty(max(1, sum(seg_strings)), dtype=torch.uint8, device=device)
    dist.all_to_all_single(rrecv[:sum(recv_r)], recs[:sum(send_r)],
                           output_split_sizes=recv_r, input_split_sizes=send_r)
    dist.all_to_all_single(srecv[:sum(seg_strings)], strs[:sum(send_s)],
                           output_split_sizes=seg_strings, input_split_sizes=send_s)
    return rrecv[:max(0, sum(seg_records) * width)], srecv[:sum(seg_strings)], seg_records, seg_strings


def exchange_partial(partial, final, device) -> dict:
    """Route `partial`'s groups to rank hash % world and merge what arrives into `final`
    (both AggregateHashTable).  The export and the collectives run in stream order on the current
    stream (no stream synchronisation); the host waits once, for the exchanged sizes.  Returns
    byte counts for reporting xGMI traffic."""
    import torch
    dist = _dist()
    world = dist.get_world_size()
    counts, sbytes = partial.partition(world, 0)
    w = partial.record_width()
    recs = torch.empty(max(1, sum(counts) * w), dtype=torch.uint8, device=device)
    strs = torch.empty(max(1, sum(sbytes)), dtype=torch.uint8, device=device)
    partial.export_records(recs, strs)
    rrecs, rstrs, seg_records, seg_strings = _exchange_with_sizes(recs, strs, counts, sbytes, w, device, world)
    final.merge_records(rrecs if rrecs.numel() else recs[:1], rstrs if rstrs.numel() else strs[:1], seg_records, seg_strings)
    me = dist.get_rank()
    sent = sum(c * w for c in counts) + sum(sbytes)
    return dict(sent_bytes=sent, remote_bytes=sent - counts[me] * w - sbytes[me], received_records=sum(seg_records))


def payload_owned(d: int, n: int, parts: int = 256):
    """Level-1 partitions of rank d: p with p * n // parts == d (dbg_agg_payload_*, abi.hip)."""
    return (d * parts + n - 1) // n, ((d + 1) * parts + n - 1) // n


def payload_splits(counts, all_counts, widths, rank: int, world: int):
    """Byte splits of the before-partial shuffle per record kind: send[k][d] (this rank's records of
    the partitions rank d owns) and recv[k][s] (source s's records of this rank's partitions)."""
    send = [[0] * world for _ in range(2)]
    recv = [[0] * world for _ in range(2)]
    lo_me, hi_me = payload_owned(rank, world)
    for k in range(2):
        for d in range(world):
            lo, hi = payload_owned(d, world)
            send[k][d] = int(counts[k][lo:hi].sum()) * widths[k]
            recv[k][d] = int(all_counts[d][k][lo_me:hi_me].sum()) * widths[k]
    return send, recv


def payload_widths(params) -> Tuple[int, int]:
    """(raw, state) payload record widths of a GROUP BY (dbg_payload_exchange_plan: the level-1
    record of one input row, and of one aggregated group) — host only."""
    import ctypes as C
    import numpy as np
    from .ffi import check, lib
    p, keep = params.to_abi(True, 0, -1)
    zeros = np.zeros(2 * 256, dtype=np.uint64)
    w = (C.c_uint32 * 2)()
    send = (C.c_uint64 * 2)()
    recv = (C.c_uint64 * 2)()
    check(lib().dbg_payload_exchange_plan(C.byref(p), 1, 0, zeros.ctypes.data_as(C.POINTER(C.c_uint64)), w, send, recv))
    del keep
    return int(w[0]), int(w[1])


def prefer_before_partial(rows: int, groups: int, widths: Tuple[int, int]) -> bool:
    """group_by_shuffle_mode for one rank's batch (settings_default.rs:469-474 offers both):
    before_partial ships every input row's raw record (rows x raw width) and aggregates once at the
    owner; before_merge aggregates here, ships the groups (groups x state width) and aggregates
    again.  The rows go first when they are the fewer bytes — mostly-unique keys, where the
    partial aggregation removes little (ClickBench Q17 at 8 GPUs: 1.25e8 rows per GPU and ~8e7
    groups: 1.0 GB of keys against 1.3 GB of group records)."""
    return rows * widths[0] <= groups * widths[1]


def exchange_payload(table, device) -> dict:
    """Before-partial shuffle (group_by_shuffle_mode = before_partial, settings_default.rs:469-473)
    of a partitioned-mode table over torch.distributed: every rank's level-1 records go to the rank
    owning their level-1 partition (dbg_agg_payload_export), with one all-gather of the per-partition
    counts and one all_to_all_single per record kind, and become that rank's payload
    (dbg_agg_payload_import) — aggregated once, by its finalize."""
    import numpy as np
    import torch
    dist = _dist()
    world, rank = dist.get_world_size(), dist.get_rank()
    counts, widths = table.payload_counts()
    mine = torch.from_numpy(counts.astype(np.int64).reshape(-1)).to(device)
    allc = torch.empty(world * mine.numel(), dtype=torch.int64, device=device)
    dist.all_gather_into_tensor(allc, mine)
    all_counts = allc.cpu().numpy().astype(np.uint64).reshape(world, 2, 256)
    send, recv = payload_splits(counts, all_counts, widths, rank, world)
    tot = [sum(send[0]), sum(send[1])]
    buf = torch.empty(max(1, tot[0] + tot[1]), dtype=torch.uint8, device=device)
    table.payload_export(world, buf)
    got = []
    for k in range(2):
        inp = buf[(tot[0] if k else 0):(tot[0] if k else 0) + tot[k]]
        out = torch.empty(max(1, sum(recv[k])), dtype=torch.uint8, device=device)
        dist.all_to_all_single(out[:sum(recv[k])], inp, output_split_sizes=recv[k], input_split_sizes=send[k])
        got.append(out)
    table.payload_import(world, rank, all_counts, got[0], got[1])
    sent = tot[0] + tot[1]
    return dict(sent_bytes=sent, remote_bytes=sent - send[0][rank] - send[1][rank],
                received_records=sum(recv[0]) // max(1, widths[0]) + sum(recv[1]) // max(1, widths[1]))


class PayloadShuffle:
    """The chunked before-partial shuffle over torch.distributed (the protocol
    dbg_agg_exchange_payload_chunk runs over RCCL): after each add_groups chunk, `ship()` sends the
    level-1 segments appended since the previous call — one all-gather of the chunk's counts, one
    asynchronous all_to_all_single per record kind — and returns without waiting, so the next
    chunk's level-1 work overlaps the transfer; `finish()` waits for every chunk and imports all of
    them (one level-1 segment per chunk and source).  Every rank calls ship() the same number of
    times."""

    def __init__(self, table, device):
        self.table, self.device = table, device
        self.first = (0, 0)
        self.chunks = []  # (all_counts [n][2][256], raw, state, works)

    def ship(self) -> dict:
        import numpy as np
        import torch
        dist = _dist()
        world, rank = dist.get_world_size(), dist.get_rank()
        counts, widths, nseg = self.table.payload_counts_from(self.first)
        mine = torch.from_numpy(counts.astype(np.int64).reshape(-1)).to(self.device)
        allc = torch.empty(world * mine.numel(), dtype=torch.int64, device=self.device)
        dist.all_gather_into_tensor(allc, mine)
        all_counts = allc.cpu().numpy().astype(np.uint64).reshape(world, 2, 256)
        send, recv = payload_splits(counts, all_counts, widths, rank, world)
        tot = [sum(send[0]), sum(send[1])]
        buf = torch.empty(max(1, tot[0] + tot[1]), dtype=torch.uint8, device=self.device)
        self.table.payload_export_from(world, self.first, buf)
        got, works = [], []
        for k in range(2):
            inp = buf[(tot[0] if k else 0):(tot[0] if k else 0) + tot[k]]
            out = torch.empty(max(1, sum(recv[k])), dtype=torch.uint8, device=self.device)
            works.append(dist.all_to_all_single(out[:sum(recv[k])], inp, output_split_sizes=recv[k],
                                                input_split_sizes=send[k], async_op=True))
            got.append(out)
        self.chunks.append((all_counts, got[0], got[1], works, buf))
        self.first = nseg
        sent = tot[0] + tot[1]
        return dict(sent_bytes=sent, remote_bytes=sent - send[0][rank] - send[1][rank],
                    received_records=sum(recv[0]) // max(1, widths[0]) + sum(recv[1]) // max(1, widths[1]))

    def finish(self):
        """Ship what add_groups appended after the last ship() (dbg_agg_exchange_payload_chunk with
        last = 1 does the same), wait for every chunk and import them all.  The decision to ship a
        last chunk is collective (one all-reduce of "segments pending"), so ranks that have nothing
        left still take part in the shipment of the ranks that have."""
        import numpy as np
        import torch
        dist = _dist()
        _, _, nseg = self.table.payload_counts_from(self.first)
        pending = torch.tensor([1 if tuple(nseg) != tuple(self.first) else 0], dtype=torch.int64, device=self.device)
        dist.all_reduce(pending, op=dist.ReduceOp.MAX)
        if int(pending.item()):
            self.ship()
        for _, _, _, works, _ in self.chunks:
            for w in works:
                w.wait()
        if not self.chunks:
            return
        cc = np.stack([c[0] for c in self.chunks])
        self.table.payload_import_chunks(dist.get_world_size(), dist.get_rank(), cc, [c[1] for c in self.chunks],
                                         [c[2] for c in self.chunks])
        self.chunks = []
        self.first = (0, 0)


class AbiComm:
    """A communicator of the C ABI (dbg_comm_*): the exchange a Rust host drives without torch.
    `unique_id` is created by one rank and handed to every rank by the host's own channel (here
    torch.distributed's object broadcast when a process group exists)."""

    def __init__(self, uid: bytes, n_ranks: int, rank: int, device: int = -1):
        import ctypes as C
        from .ffi import check, lib
        buf = (C.c_uint8 * 128).from_buffer_copy(uid)
        h = C.c_void_p()
        check(lib().dbg_comm_create(buf, n_ranks, rank, device, C.byref(h)))
        self.h = h
        self.n_ranks, self.rank = n_ranks, rank

    @staticmethod
    def unique_id() -> bytes:
        import ctypes as C
        from .ffi import check, lib
        buf = (C.c_uint8 * 128)()
        check(lib().dbg_comm_get_unique_id(buf))
        return bytes(buf)

    @classmethod
    def from_process_group(cls, device: int = -1) -> "AbiComm":
        dist = _dist()
        obj = [cls.unique_id() if dist.get_rank() == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        return cls(obj[0], dist.get_world_size(), dist.get_rank(), device)

    def exchange(self, partial, final) -> dict:
        """dbg_agg_exchange: route partial's groups to rank hash % n, merge arrivals into final."""
        import ctypes as C
        from . import abi
        from .ffi import check, lib
        st = abi.dbg_exchange_stats()
        check(lib().dbg_agg_exchange(self.h, partial.h, final.h, C.byref(st)))
        return dict(sent_bytes=st.sent_bytes, remote_bytes=st.remote_bytes, received_records=st.received_records,
                    received_string_bytes=st.received_string_bytes)

    def exchange_payload(self, table) -> dict:
        """dbg_agg_exchange_payload: the before-partial shuffle of a partitioned-mode table."""
        import ctypes as C
        from . import abi
        from .ffi import check, lib
        st = abi.dbg_exchange_stats()
        check(lib().dbg_agg_exchange_payload(self.h, table.h, C.byref(st)))
        return dict(sent_bytes=st.sent_bytes, remote_bytes=st.remote_bytes, received_records=st.received_records)

    def exchange_payload_chunk(self, table, last: bool) -> dict:
        """dbg_agg_exchange_payload_chunk: ship the segments since the previous call (asynchronous);
        last=True also waits for every chunk and imports them."""
        import ctypes as C
        from . import abi
        from .ffi import check, lib
        st = abi.dbg_exchange_stats()
        check(lib().dbg_agg_exchange_payload_chunk(self.h, table.h, 1 if last else 0, C.byref(st)))
        return dict(sent_bytes=st.sent_bytes, remote_bytes=st.remote_bytes, received_records=st.received_records)

    def close(self):
        if getattr(self, "h", None):
            from .ffi import lib
            lib().dbg_comm_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


_FIXED_BUFS = {}


def _fixed_buffer(key, nbytes, device):
    """Persistent exchange buffers: a stable address keeps the merge's batch descriptor cached
    on the device (no upload, so the next reset needs no stream synchronisation)."""
    import torch
    b = _FIXED_BUFS.get(key)
    if b is None or b.numel() != nbytes or b.device != torch.device(device):
        b = torch.empty(nbytes, dtype=torch.uint8, device=device)
        _FIXED_BUFS[key] = b
    return b


def all_gather_fixed(buf, out):
    """All-gather of equal-size uint8 buffers (out holds world * buf.numel() bytes, rank order)."""
    _dist().all_gather_into_tensor(out, buf)
    return out


def fixed_capacity(partial) -> int:
    """Records per fixed buffer: every group a table of this capacity can hold (cap + sentinel)."""
    return partial.capacity + 1


def gather_small(partial, final, device, root: int = 0, cap_records: int = 0):
    """Replicas + gather: merge every rank's `partial` groups into `final` on rank `root`.
    Returns the bytes each rank sent."""
    dist = _dist()
    world, rank = dist.get_world_size(), dist.get_rank()
    cap = cap_records or fixed_capacity(partial)
    w = partial.record_width()
    nbytes = (cap + 1) * w
    buf = _fixed_buffer(("send", str(device)), nbytes, device)
    out = _fixed_buffer(("recv", str(device)), world * nbytes, device)
    partial.export_fixed(buf, cap)
    all_gather_fixed(buf, out)
    if rank == root:
        final.merge_fixed(out, world, cap)
    return nbytes


class GatherPipeline:
    """Replicas + gather, pipelined over batches (bench.py, N > 1, low cardinality).

    stream s1: insert(k) -> export_fixed(k) into send[k % 2]
    stream s2: all-gather(k) -> (root) merge_fixed(k) -> fused finalize(k)
    The host enqueues batch k+1's insert and all-gather before it waits for finalize(k), so the
    exchange and final merge of one batch overlap the partial aggregation of the next.  Buffers
    and events are per parity; export(k+2) waits for all-gather(k) to have read send[k % 2]."""

    def __init__(self, runner, final, device, rank: int, world: int, root: int = 0):
        import torch
        self.runner, self.final, self.rank, self.world, self.root = runner, final, rank, world, root
        self.s1 = torch.cuda.current_stream()
        self.s2 = torch.cuda.Stream()
        runner.table.set_stream(self.s1)
        final.set_stream(self.s2)
        self.cap = fixed_capacity(runner.table)
        w = runner.table.record_width()
        n = (self.cap + 1) * w
        self.send = [torch.empty(n, dtype=torch.uint8, device=device) for _ in range(2)]
        self.recv = [torch.empty(world * n, dtype=torch.uint8, device=device) for _ in range(2)]
        self.ev_exp = [torch.cuda.Event() for _ in range(2)]
        self.ev_gath = [torch.cuda.Event() for _ in range(2)]
        self.used = [False, False]
        self.pending = None  # parity whose merge + finalize is still to be enqueued / waited
        self.bytes_per_rank = n

    def step(self, k: int) -> int:
        import torch
        p = k % 2
        r = self.runner
        r.insert(k)
        if self.used[p]:
            self.s1.wait_event(self.ev_gath[p])
        r.table.export_fixed(self.send[p], self.cap)
        self.ev_exp[p].record(self.s1)
        with torch.cuda.stream(self.s2):
            self.s2.wait_event(self.ev_exp[p])
            all_gather_fixed(self.send[p], self.recv[p])
            self.ev_gath[p].record(self.s2)
        self.used[p] = True
        n = self.drain()
        if self.rank == self.root:
            self.final.merge_fixed(self.recv[p], self.world, self.cap)
            r.finalize_async(self.final.h, p)
            self.pending = p
        return n

    def drain(self) -> int:
        """Wait for the finalize in flight (root only); returns its group count."""
        p, self.pending = self.pending, None
        return self.runner.finalize_wait(self.final.h, p) if p is not None else 0
