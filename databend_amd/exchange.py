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


def exchange_partial(partial, final, device) -> dict:
    """Route `partial`'s groups to rank hash % world and merge what arrives into `final`
    (both AggregateHashTable).  Returns byte counts for reporting xGMI traffic."""
    import torch
    dist = _dist()
    world = dist.get_world_size()
    counts, sbytes = partial.partition(world, 0)
    w = partial.record_width()
    recs = torch.empty(max(1, sum(counts) * w), dtype=torch.uint8, device=device)
    strs = torch.empty(max(1, sum(sbytes)), dtype=torch.uint8, device=device)
    partial.export_records(recs, strs)
    torch.cuda.current_stream().synchronize()
    rrecs, rsplits = all_to_all_bytes(recs, [c * w for c in counts], device)
    rstrs, rssplits = all_to_all_bytes(strs, list(sbytes), device)
    seg_records = [s // w for s in rsplits]
    final.merge_records(rrecs, rstrs, seg_records, rssplits)
    sent = sum(c * w for c in counts) + sum(sbytes)
    return dict(sent_bytes=sent, remote_bytes=sent - counts[dist.get_rank()] * w - sbytes[dist.get_rank()],
                received_records=sum(seg_records))
