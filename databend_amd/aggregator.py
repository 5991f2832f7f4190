"""Host mirror of Databend's aggregator processors over the C ABI.

Names, argument meaning and error behaviour follow the reference
(src/query/service/src/pipelines/processors/transforms/aggregator/ = AGG/):

* `AggregatorParams`            AGG/aggregator_params.rs:31-116
* `HashTableConfig`             EAGG/mod.rs:59-132 (knobs that matter on the GPU: capacity hint)
* `AggregateHashTable`          EAGG/aggregate_hashtable.rs:47-589, one table in HBM
* `TransformPartialAggregate`   AGG/transform_aggregate_partial.rs:107-468 (transform / on_finish)
* `TransformFinalAggregate`     AGG/transform_aggregate_final.rs:45-343 (transform -> DataBlock)
* `AggregateMeta`               AGG/aggregate_meta.rs:124-134 (partial payloads between stages)

Every call lands in libdbgpu_agg.so; the product path has no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field, replace
from typing import List, Optional, Sequence, Union

import numpy as np

from . import abi
from .aggregates import AggregateFunction
from .column import Column, DataBlock, DataType, abi_array, unpack_bits
from .ffi import check, lib

ColumnLike = Union[Column, "DeviceColumn"]  # noqa: F821


@dataclass
class AggregatorParams:
    """AggregatorParams::try_create (AGG/aggregator_params.rs:48-94)."""
    group_data_types: List[DataType]
    aggregate_functions: List[AggregateFunction]
    max_block_size: int = 65536
    # enable_experimental_aggregate_hashtable (settings_default.rs); False selects the legacy
    # HashMethod path's buckets: single-level (-1) below group_by_two_level_threshold groups, else
    # 256 buckets hash2bucket<8, true> of FastHash (AGG/transform_aggregate_partial.rs:330-350,
    # 415-447)
    enable_experimental_aggregate_hashtable: bool = True
    group_by_two_level_threshold: int = 20000

    def to_abi(self, partial: bool, capacity_hint: int, device: int):
        # a DISTINCT aggregate raises here (AggregateFunction.to_abi): DistinctAggregator runs it
        gt = (abi.dbg_datatype * max(1, len(self.group_data_types)))(*[t.to_abi() for t in self.group_data_types])
        ag = (abi.dbg_agg_spec * max(1, len(self.aggregate_functions)))(*[f.to_abi() for f in self.aggregate_functions])
        p = abi.dbg_agg_params(gt, len(self.group_data_types), ag, len(self.aggregate_functions), device,
                               1 if partial else 0, capacity_hint)
        return p, (gt, ag)

    def record_layout(self) -> "abi.dbg_record_layout":
        """The exchange-record layout of a table with these params (dbg_agg_record_layout), computed on
        the host: no device needed."""
        p, keep = self.to_abi(True, 0, -1)
        out = abi.dbg_record_layout()
        check(lib().dbg_agg_record_layout(C.byref(p), C.byref(out)))
        return out

    def empty_result_block(self) -> DataBlock:
        """AggregatorParams::empty_result_block (:103-115): [agg results..., group cols...]."""
        cols = []
        for f in self.aggregate_functions:
            rt = f.return_type()
            cols.append(_empty_column(rt))
        for t in self.group_data_types:
            cols.append(_empty_column(t))
        return DataBlock(cols)


def _empty_column(t: DataType) -> Column:
    if t.type_id == abi.STRING:
        return Column(t, np.zeros(0, np.uint8), np.zeros(1, np.uint64), np.zeros(0, bool) if t.nullable else None)
    if t.type_id == abi.DECIMAL128:
        return Column(t, np.zeros(0, np.uint8), None, np.zeros(0, bool) if t.nullable else None)
    if t.type_id == abi.BOOLEAN:
        return Column(t, np.zeros(0, bool), None, np.zeros(0, bool) if t.nullable else None)
    return Column(t, np.zeros(0, t.np_dtype), None, np.zeros(0, bool) if t.nullable else None)


MAX_PAGE_SIZE = 256 * 1024  # EAGG/mod.rs:50


class RadixBitsHint:
    """`current_max_radix_bits: Arc<AtomicU64>` (EAGG/mod.rs:62): the one piece of state shared
    by every partial table of a query, so their bucket counts converge (CAS loop of
    maybe_repartition, EAGG/aggregate_hashtable.rs:467-484)."""

    def __init__(self, bits: int):
        import threading
        self._v = bits
        self._lock = threading.Lock()

    def load(self) -> int:
        return self._v

    def fetch_max(self, bits: int) -> int:
        with self._lock:
            if bits > self._v:
                self._v = bits
            return self._v


@dataclass
class HashTableConfig:
    """HashTableConfig (EAGG/mod.rs:59-132).  The HBM table aggregates exactly, so
    max_partial_capacity has no GPU meaning; `capacity_hint` seeds the table size and the radix
    knobs decide how many buckets a partial emits (partial_bucket_bits)."""
    partial_agg: bool = False
    capacity_hint: int = 0
    current_max_radix_bits: RadixBitsHint = field(default_factory=lambda: RadixBitsHint(3))
    initial_radix_bits: int = 3
    max_radix_bits: int = 7
    repartition_radix_bits_incr: int = 2
    block_fill_factor: float = 1.8

    def with_partial(self, partial_agg: bool, active_threads: int = 1) -> "HashTableConfig":
        return replace(self, partial_agg=partial_agg)

    def cluster_with_partial(self, partial_agg: bool, node_nums: int) -> "HashTableConfig":
        return replace(self, partial_agg=partial_agg, repartition_radix_bits_incr=4)

    def with_initial_radix_bits(self, bits: int) -> "HashTableConfig":
        return replace(self, initial_radix_bits=bits, current_max_radix_bits=RadixBitsHint(bits))

    def update_current_max_radix_bits(self) -> None:
        self.current_max_radix_bits.fetch_max(self.max_radix_bits)


def payload_tuple_size(group_types: Sequence[DataType], n_aggs: int) -> int:
    """Payload::new (EAGG/payload.rs:88-130): validity byte per nullable key + rowformat_size of
    each key (EAGG/payload_row.rs:43-64; strings 4 + 8) + hash 8 + state address 8."""
    size = sum(1 for t in group_types if t.nullable)
    for t in group_types:
        size += 12 if t.type_id == abi.STRING else t.width
    return size + 8 + (8 if n_aggs else 0)


def partial_bucket_bits(config: HashTableConfig, n_groups: int, tuple_size: int) -> int:
    """The radix bits a partial table ends with: maybe_repartition (EAGG/aggregate_hashtable.rs:
    453-503) raises them by repartition_radix_bits_incr while the payload holds more than
    MAX_PAGE_SIZE * (block_fill_factor as usize) bytes per partition, up to max_radix_bits, and
    adopts the query-wide maximum.  The reference steps once per add_groups call; the GPU table
    knows its exact group count at on_finish and applies the rule to convergence."""
    bits = config.current_max_radix_bits.load()
    limit = MAX_PAGE_SIZE * int(config.block_fill_factor)
    mem = n_groups * tuple_size
    while config.partial_agg and bits < config.max_radix_bits and mem // (1 << bits) > limit:
        bits += config.repartition_radix_bits_incr
    return config.current_max_radix_bits.fetch_max(bits)


def _current_torch_stream():
    """Launch on torch's current stream so torch-produced device columns are stream-ordered."""
    try:
        import torch
        if torch.cuda.is_available():
            return torch.cuda.current_stream()
    except Exception:
        pass
    return None


def _arg_structs(aggs: Sequence[AggregateFunction], params: Sequence[Optional[ColumnLike]]):
    out = []
    for f, p in zip(aggs, params):
        if p is None:
            c = abi.dbg_column()
            c.dt = abi.dbg_datatype(-1, 0, 0, 0, 0)
            out.append(c)
        else:
            out.append(p.to_abi())
    return abi_array(out)


class AggregateHashTable:
    """One GPU aggregate table (a `dbg_agg_handle`)."""

    def __init__(self, params: AggregatorParams, config: HashTableConfig = None, device: int = -1, stream=None):
        config = config or HashTableConfig()
        self.params = params
        p, self._keep = params.to_abi(config.partial_agg, config.capacity_hint, device)
        h = C.c_void_p()
        check(lib().dbg_agg_create(C.byref(p), C.byref(h)))
        self.h = h
        self._retained = []  # device inputs must outlive the table (include/dbgpu_agg.h)
        if stream is None:
            stream = _current_torch_stream()
        if stream is not None:
            self.set_stream(stream)

    # ---- lifecycle
    def close(self):
        if self.h:
            lib().dbg_agg_destroy(self.h)
            self.h = None
            self._retained.clear()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_stream(self, stream):
        """stream: a torch.cuda.Stream (its hipStream_t) or None for the handle's own."""
        ptr = None if stream is None else stream.cuda_stream
        check(lib().dbg_agg_set_stream(self.h, ptr))

    def reset(self):
        check(lib().dbg_agg_reset(self.h))
        # retained device inputs may go: later reuse of their memory is stream-ordered after
        # every launch that reads them (the handle runs on torch's current stream)
        self._retained.clear()

    def compact(self) -> bool:
        """dbg_agg_compact: the table rewritten to reference one record batch of its groups, so the
        inputs of earlier add_groups calls are released (the reference's payload arena holds only
        new groups' keys, EAGG/payload_row.rs:111-130).  True when it rewrote the table."""
        done = C.c_int(0)
        check(lib().dbg_agg_compact(self.h, C.byref(done)))
        if done.value:
            self._retained.clear()  # no entry points at them any more (stream-ordered reuse)
        return bool(done.value)

    def retained_bytes(self) -> int:
        """Device bytes the handle keeps for referenced inputs (dbg_agg_retained_bytes)."""
        b = C.c_uint64()
        check(lib().dbg_agg_retained_bytes(self.h, C.byref(b)))
        return b.value

    def set_host_staging(self, rows: int):
        """Gather host blocks into launches of `rows` rows (dbg_agg_set_host_staging); 0 = off."""
        check(lib().dbg_agg_set_host_staging(self.h, rows))

    def set_strategy(self, strategy: int):
        """abi.STRATEGY_AUTO / STRATEGY_TABLE / STRATEGY_PARTITIONED (include/dbgpu_agg.h)."""
        check(lib().dbg_agg_set_strategy(self.h, strategy))

    def strategy(self):
        """(partitioned?, partitions of the last finalize that needed extra LDS rounds)."""
        p, r = C.c_int(), C.c_uint64()
        check(lib().dbg_agg_get_strategy(self.h, C.byref(p), C.byref(r)))
        return bool(p.value), r.value

    def set_partition_keys(self, n_keys: int):
        """Bucket groups (partition schemes 0 / 1) by the hash of their first n_keys key columns
        (0 = all): a DISTINCT pair table's buckets follow its group's keys."""
        check(lib().dbg_agg_set_partition_keys(self.h, n_keys))

    def pp_specialised(self) -> bool:
        """Whether the last partitioned finalize ran the compile-time specialised aggregation."""
        p, r = C.c_int(), C.c_uint64()
        check(lib().dbg_agg_get_strategy(self.h, C.byref(p), C.byref(r)))
        return p.value == 2

    # ---- AggregateHashTable::add_groups (+ fused filter)
    def add_groups(self, group_columns: Sequence[ColumnLike], params: Sequence[Optional[ColumnLike]],
                   rows: Optional[int] = None, filter_program=None, on_device: Optional[bool] = None) -> None:
        if rows is None:
            rows = len(group_columns[0])
        if on_device is None:
            on_device = not isinstance(group_columns[0], Column)
        keys = abi_array([c.to_abi() for c in group_columns])
        args = _arg_structs(self.params.aggregate_functions, params)
        fp = filter_program.ptr() if filter_program is not None else None
        check(lib().dbg_agg_add_groups(self.h, keys, args, fp, rows, 1 if on_device else 0))
        if on_device:
            self._retained.append((group_columns, params, filter_program))

    def add_groups_abi(self, keys: Sequence["abi.dbg_column"], args: Sequence["abi.dbg_column"], rows: int,
                       filter_program=None, on_device: bool = False) -> None:
        """add_groups over ready-made dbg_column structs (the caller keeps their memory alive, and
        device memory until reset/close)."""
        fp = filter_program.ptr() if filter_program is not None else None
        check(lib().dbg_agg_add_groups(self.h, abi_array(list(keys)), abi_array(list(args)), fp, rows,
                                       1 if on_device else 0))
        if on_device:
            self._retained.append(filter_program)

    # ---- merge_result
    def finalize(self):
        n = C.c_uint64()
        sb = (C.c_uint64 * max(1, len(self.params.group_data_types)))()
        check(lib().dbg_agg_finalize(self.h, C.byref(n), sb))
        return n.value, list(sb)

    def merge_result(self) -> DataBlock:
        """All groups as one host DataBlock [agg results..., group cols...]
        (TransformFinalAggregate output order, AGG/transform_aggregate_final.rs:128-133)."""
        n, sbytes = self.finalize()
        aggs, keys = self._out_buffers(n, sbytes)
        out_a = (abi.dbg_out_column * max(1, len(aggs)))()
        out_k = (abi.dbg_out_column * max(1, len(keys)))()
        for i, b in enumerate(aggs):
            out_a[i].data, out_a[i].offsets, out_a[i].validity = b["ptrs"]
        for i, b in enumerate(keys):
            out_k[i].data, out_k[i].offsets, out_k[i].validity = b["ptrs"]
        check(lib().dbg_agg_result(self.h, out_a, out_k, 0))
        cols = [self._to_column(b, n) for b in aggs] + [self._to_column(b, n) for b in keys]
        return DataBlock(cols)

    def merge_result_device(self) -> list:
        """All groups as device columns [agg results..., group cols...] (DeviceColumn, HBM): only the
        group count and string sizes reach the host."""
        from .device import DeviceColumn, empty
        n, sbytes = self.finalize()
        gt = self.params.group_data_types
        aggs = [empty(f.return_type(), n) for f in self.params.aggregate_functions]
        keys = [empty(t, n, string_bytes=sbytes[i]) for i, t in enumerate(gt)]
        out_a = (abi.dbg_out_column * max(1, len(aggs)))()
        out_k = (abi.dbg_out_column * max(1, len(keys)))()
        for arr, cols in ((out_a, aggs), (out_k, keys)):
            for i, c in enumerate(cols):
                arr[i].data = c.data.data_ptr()
                arr[i].offsets = c.offsets.data_ptr() if c.offsets is not None else None
                arr[i].validity = c.validity.data_ptr() if c.validity is not None else None
        check(lib().dbg_agg_result(self.h, out_a, out_k, 1))
        return aggs + keys

    def serialized_strides(self) -> List[int]:
        n = len(self.params.aggregate_functions)
        st = (C.c_uint32 * max(1, n))()
        check(lib().dbg_agg_serialized_stride(self.h, st))
        return list(st)[:n]

    def result_serialized(self) -> DataBlock:
        """AggregateMeta::Serialized's block (EAGG/payload_flush.rs:129-164): one Binary column of
        borsh states per aggregate (as byte strings), then the group columns."""
        n, sbytes = self.finalize()
        strides = self.serialized_strides()
        bin_t = DataType(abi.STRING)
        states = []
        for s in strides:
            data = np.zeros(max(1, n * s), np.uint8)
            offs = np.zeros(n + 1, np.uint64)
            states.append(dict(t=bin_t, data=data, offs=offs, val=None,
                               ptrs=(data.ctypes.data, offs.ctypes.data, None)))
        _, keys = self._out_buffers(n, sbytes)
        out_a = (abi.dbg_out_column * max(1, len(states)))()
        out_k = (abi.dbg_out_column * max(1, len(keys)))()
        for i, b in enumerate(states):
            out_a[i].data, out_a[i].offsets, out_a[i].validity = b["ptrs"]
        for i, b in enumerate(keys):
            out_k[i].data, out_k[i].offsets, out_k[i].validity = b["ptrs"]
        check(lib().dbg_agg_result_serialized(self.h, out_a, out_k, 0))
        cols = [self._to_column(b, n) for b in states] + [self._to_column(b, n) for b in keys]
        return DataBlock(cols)

    def _out_buffers(self, n, sbytes):
        def buf(t: DataType, strbytes=0):
            if t.type_id == abi.STRING:
                data = np.zeros(max(1, strbytes), np.uint8)
                offs = np.zeros(n + 1, np.uint64)
            else:
                data = np.zeros(max(1, n * t.width), np.uint8)
                offs = None
            val = np.zeros(max(1, (n + 7) // 8), np.uint8) if t.nullable else None
            return dict(t=t, data=data, offs=offs, val=val,
                        ptrs=(data.ctypes.data, offs.ctypes.data if offs is not None else None,
                              val.ctypes.data if val is not None else None))
        aggs = [buf(f.return_type()) for f in self.params.aggregate_functions]
        keys = [buf(t, sbytes[i]) for i, t in enumerate(self.params.group_data_types)]
        return aggs, keys

    @staticmethod
    def _to_column(b, n) -> Column:
        t: DataType = b["t"]
        if t.type_id == abi.STRING:
            offs = b["offs"]
            data = b["data"][:int(offs[-1])]
        elif t.type_id == abi.DECIMAL128:
            data, offs = b["data"][:16 * n], None
        elif t.type_id == abi.BOOLEAN:
            data, offs = b["data"][:n].astype(bool), None
        else:
            data, offs = b["data"][:n * t.width].view(t.np_dtype), None
        val = unpack_bits(b["val"], n) if b["val"] is not None else None
        return Column(t, data, offs, val)

    def merge_serialized(self, state_columns: Sequence[ColumnLike], group_columns: Sequence[ColumnLike],
                         rows: Optional[int] = None, on_device: Optional[bool] = None) -> None:
        """add_groups with agg_states: AggregateMeta::Serialized's block re-inserted with batch_merge
        (SerializedPayload::convert_to_aggregate_table, AGG/aggregate_meta.rs:57-101).
        state_columns: one Binary column of borsh states per aggregate."""
        if rows is None:
            rows = len(group_columns[0])
        if on_device is None:
            on_device = not isinstance(group_columns[0], Column)
        keys = abi_array([c.to_abi() for c in group_columns])
        states = abi_array([c.to_abi() for c in state_columns]) if state_columns else None
        check(lib().dbg_agg_merge_serialized(self.h, states, keys, rows, 1 if on_device else 0))
        if on_device:
            self._retained.append((state_columns, group_columns))

    # ---- partial-state records (exchange / partition bucket)
    def record_width(self) -> int:
        w = C.c_uint32()
        check(lib().dbg_agg_record_width(self.h, C.byref(w)))
        return w.value

    def partition(self, n_parts: int, scheme: int = 0):
        counts = (C.c_uint64 * n_parts)()
        sbytes = (C.c_uint64 * n_parts)()
        check(lib().dbg_agg_partition(self.h, n_parts, scheme, counts, sbytes))
        return list(counts), list(sbytes)

    def export_records(self, dev_records, dev_strings):
        """dev_records / dev_strings: torch uint8 cuda tensors sized from partition()."""
        check(lib().dbg_agg_export_records(self.h, dev_records.data_ptr(),
                                           dev_strings.data_ptr() if dev_strings is not None else None))

    def merge_records(self, dev_records, dev_strings, seg_records: Sequence[int], seg_strings: Sequence[int]):
        n = len(seg_records)
        sr = (C.c_uint64 * max(1, n))(*seg_records)
        ss = (C.c_uint64 * max(1, n))(*seg_strings)
        check(lib().dbg_agg_merge_records(self.h, dev_records.data_ptr(),
                                          dev_strings.data_ptr() if dev_strings is not None else None, n, sr, ss))
        self._retained.append((dev_records, dev_strings))

    # ---- before-partial shuffle of the partitioned payload (dbg_agg_payload_*)
    def payload_counts(self):
        """(counts [2][256] numpy u64: raw / state records per level-1 partition, record widths)."""
        import numpy as np
        c = (C.c_uint64 * 512)()
        w = (C.c_uint32 * 2)()
        check(lib().dbg_agg_payload_counts(self.h, c, w))
        return np.frombuffer(bytes(c), dtype=np.uint64).reshape(2, 256).copy(), (int(w[0]), int(w[1]))

    def payload_export(self, n_ranks: int, dev_buf):
        check(lib().dbg_agg_payload_export(self.h, n_ranks, dev_buf.data_ptr()))

    def payload_counts_from(self, first_seg):
        """Counts of the level-1 segments from first_seg[kind] on: (counts [2][256], widths,
        current segment counts) — one chunk of the chunked shuffle."""
        import numpy as np
        c = (C.c_uint64 * 512)()
        w = (C.c_uint32 * 2)()
        n = (C.c_uint32 * 2)()
        f = (C.c_uint32 * 2)(*first_seg)
        check(lib().dbg_agg_payload_counts_from(self.h, f, c, w, n))
        return np.frombuffer(bytes(c), dtype=np.uint64).reshape(2, 256).copy(), (int(w[0]), int(w[1])), (int(n[0]), int(n[1]))

    def payload_export_from(self, n_ranks: int, first_seg, dev_buf):
        f = (C.c_uint32 * 2)(*first_seg)
        check(lib().dbg_agg_payload_export_from(self.h, n_ranks, f, dev_buf.data_ptr()))

    def payload_import_chunks(self, n_ranks: int, rank: int, chunk_counts, raws, states):
        """chunk_counts: numpy u64 [n_chunks][n_ranks][2][256]; raws / states: per chunk the
        received records (source-major), or None."""
        import numpy as np
        import torch
        torch.cuda.current_stream().synchronize()
        arr = np.ascontiguousarray(chunk_counts, dtype=np.uint64)
        nc = arr.shape[0]
        ptr = arr.ctypes.data_as(C.POINTER(C.c_uint64))
        rp = (C.c_void_p * nc)(*[x.data_ptr() if x is not None else None for x in raws])
        sp = (C.c_void_p * nc)(*[x.data_ptr() if x is not None else None for x in states])
        check(lib().dbg_agg_payload_import_chunks(self.h, n_ranks, rank, nc, ptr, rp, sp))

    def payload_import(self, n_ranks: int, rank: int, all_counts, raw, state):
        """all_counts: numpy u64 [n_ranks][2][256]; raw / state: received records (source-major)."""
        import numpy as np
        import torch
        torch.cuda.current_stream().synchronize()  # the received buffers were written on torch's stream
        arr = np.ascontiguousarray(all_counts, dtype=np.uint64)
        ptr = arr.ctypes.data_as(C.POINTER(C.c_uint64))
        check(lib().dbg_agg_payload_import(self.h, n_ranks, rank, ptr, raw.data_ptr() if raw is not None else None,
                                           state.data_ptr() if state is not None else None))

    # ---- fixed-capacity exchange (low cardinality: replicas + gather)
    @property
    def capacity(self) -> int:
        cap = C.c_uint64()
        check(lib().dbg_agg_capacity(self.h, C.byref(cap)))
        return cap.value

    def export_fixed(self, dev_buf, cap_records: int):
        """Write this table's groups into dev_buf ((cap_records + 1) * record_width bytes), the
        group count staying on the device (include/dbgpu_agg.h, dbg_agg_export_fixed)."""
        check(lib().dbg_agg_export_fixed(self.h, dev_buf.data_ptr(), cap_records))

    def merge_fixed(self, dev_bufs, n_bufs: int, cap_records: int):
        check(lib().dbg_agg_merge_fixed(self.h, dev_bufs.data_ptr(), n_bufs, cap_records))
        self._retained.append(dev_bufs)


@dataclass
class Payload:
    """One bucket of a partial table's groups as partial-state records resident in HBM
    (the GPU form of `Payload`, EAGG/payload.rs:41-84): `n_records` records of
    dbg_agg_record_width bytes ([hash][keys][state words], include/dbgpu_agg.h) and the bucket's
    string blob.  `records` / `strings` are torch uint8 cuda tensors (views into one export)."""
    records: "object"
    strings: "object"
    n_records: int
    string_bytes: int

    def __len__(self):
        return self.n_records


@dataclass
class AggregateMeta:
    """AggregateMeta (AGG/aggregate_meta.rs:124-134).  AggregatePayload: one bucket of one
    partial (`bucket`, `payload`, `max_partition_count` = 2^radix bits of the partial that wrote
    it).  Serialized: the same bucket as a DataBlock [Binary state per aggregate..., group
    columns...] (SerializedPayload, :44-109) — what crosses the Flight exchange or comes back from
    spill, from a CPU node or a GPU one.  Partitioned: every payload of one bucket after alignment
    (`data`)."""
    bucket: int
    payload: Optional[Payload] = None
    max_partition_count: int = 1
    data: Optional[List["AggregateMeta"]] = None
    serialized: Optional[DataBlock] = None
    legacy: bool = False  # a legacy HashMethod partial's bucket (-1 = single-level, else 0..255)
    # DISTINCT aggregates: per distinct aggregate j, the bucket's distinct (keys..., x_j) pairs —
    # the AggregateDistinctCombinator sets that travel inside their groups' states in the reference
    # (FUN/aggregate_combinator_distinct.rs:94-105), bucketed by the group keys alone
    distinct: Optional[List[Payload]] = None

    @staticmethod
    def create_agg_payload(bucket: int, payload: Payload, max_partition_count: int) -> "AggregateMeta":
        return AggregateMeta(bucket, payload, max_partition_count)

    @staticmethod
    def create_serialized(bucket: int, block: DataBlock, max_partition_count: int) -> "AggregateMeta":
        return AggregateMeta(bucket, None, max_partition_count, serialized=block)

    @staticmethod
    def create_partitioned(bucket: int, data: List["AggregateMeta"]) -> "AggregateMeta":
        return AggregateMeta(bucket, None, 0, data)

    def is_partitioned(self) -> bool:
        return self.data is not None

    def is_serialized(self) -> bool:
        return self.serialized is not None


def _cuda_device():
    import torch
    return torch.device("cuda", torch.cuda.current_device())


SINGLE_LEVEL_BUCKET = -1  # SINGLE_LEVEL_BUCKET_NUM (AGG/transform_partition_bucket.rs)
LEGACY_BUCKETS = 256      # PartitionedHashtable<_, 8> (HT/partitioned_hashtable.rs)
LEGACY_SCHEME = 2


LEGACY_KEYS_U8, LEGACY_KEYS_U16 = 1, 2  # DBG_LEGACY_KEYS_U8 / _U16 (include/dbgpu_agg.h)


def legacy_hash_method(types: Sequence[DataType]):
    """dbg_legacy_hash_method: (kind, key bytes) of HashMethodKind::choose_hash_method_with_types
    (EXP/kernels/group_by.rs:48-95)."""
    arr = (abi.dbg_datatype * len(types))(*[t.to_abi() for t in types])
    k, kb = C.c_int(), C.c_uint32()
    check(lib().dbg_legacy_hash_method(arr, len(types), C.byref(k), C.byref(kb)))
    return k.value, kb.value


def export_buckets(table: AggregateHashTable, n_parts: int, scheme: int = 1) -> List[Payload]:
    """All groups of `table` as n_parts bucket payloads (dbg_agg_partition + export_records), in
    bucket order; scheme 1 = radix bits [48 - r, 48) (EAGG/partitioned_payload.rs:121, 267-275),
    scheme 0 = hash % n_parts (EAGG/payload.rs:377-383), scheme 2 = the legacy buckets
    hash2bucket<log2 n, true>(FastHash(key)) (HT/partitioned_hashtable.rs:77-83)."""
    import torch
    counts, sbytes = table.partition(n_parts, scheme)
    w = table.record_width()
    dev = _cuda_device()
    recs = torch.empty(max(1, sum(counts) * w), dtype=torch.uint8, device=dev)
    strs = torch.empty(max(1, sum(sbytes)), dtype=torch.uint8, device=dev)
    table.export_records(recs, strs)
    out, r0, s0 = [], 0, 0
    for c, b in zip(counts, sbytes):
        out.append(Payload(recs[r0 * w:(r0 + c) * w], strs[s0:s0 + b], c, b))
        r0, s0 = r0 + c, s0 + b
    return out


class TransformPartialAggregate:
    """AGG/transform_aggregate_partial.rs:107-468 — AccumulatingTransform over DataBlocks.
    Host blocks (<= max_block_size rows, settings_default.rs:131) are gathered by the library's
    host staging into launches of `staging_rows` rows (dbg_agg_set_host_staging)."""

    DEFAULT_STAGING_ROWS = 1 << 23
    DEFAULT_COMPACT_BYTES = 1 << 30

    def __init__(self, params: AggregatorParams, config: HashTableConfig = None, device: int = -1,
                 staging_rows: int = DEFAULT_STAGING_ROWS, compact_bytes: int = DEFAULT_COMPACT_BYTES):
        self.params = params
        self.config = (config or HashTableConfig()).with_partial(True)
        self.distinct = None
        if any(f.distinct for f in params.aggregate_functions):
            # a DISTINCT aggregate forces the table to its max radix bits (:146-155); its sets are
            # pair tables beside the main one (databend_amd/distinct.py)
            from .distinct import DistinctPartial
            self.config = self.config.with_initial_radix_bits(self.config.max_radix_bits)
            self.distinct = DistinctPartial(params, device)
            self.hashtable = self.distinct.table
        else:
            self.hashtable = AggregateHashTable(params, self.config, device)
        if staging_rows and self.distinct is None:
            self.hashtable.set_host_staging(staging_rows)
        # once the copies of host blocks a referenced-key table keeps exceed this, the table is
        # compacted to its groups (0 = never)
        self.compact_bytes = compact_bytes
        self._compacted_bytes = 0  # retained bytes right after the last compaction (its group records)

    @classmethod
    def try_create(cls, params: AggregatorParams, config: HashTableConfig = None, device: int = -1, **kw):
        return cls(params, config, device, **kw)

    def transform(self, block: DataBlock, group_indices: Sequence[int], arg_indices: Sequence[Optional[int]],
                  filter_program=None) -> List[DataBlock]:
        """execute_one_block (:235-327): group columns and per-aggregate argument columns picked
        from the block by index; the block's rows are added to the HBM table."""
        groups = [block.columns[i] for i in group_indices]
        args = [None if i is None else block.columns[i] for i in arg_indices]
        # the tables' inputs are compacted away on the bytes retained since the last compaction,
        # not on the total: the compacted group records themselves count towards the total, and
        # once they alone pass the limit a total-based trigger would compact again after every
        # block.  A DISTINCT partial compacts its main table and its pair tables together.
        owner = self.distinct if self.distinct is not None else self.hashtable
        if self.distinct is not None:
            self.distinct.add_groups(groups, args, block.num_rows(), filter_program)
        else:
            self.hashtable.add_groups(groups, args, rows=block.num_rows(), filter_program=filter_program)
        if self.compact_bytes and owner.retained_bytes() - self._compacted_bytes > self.compact_bytes:
            owner.compact()
            self._compacted_bytes = owner.retained_bytes()
        return []

    def on_finish(self) -> List[AggregateMeta]:
        """on_finish (:449-465): one AggregatePayload per non-empty radix bucket, bucket = hash bits
        [48 - r, 48), with r from the shared radix hint and this table's payload size.

        Legacy path (enable_experimental_aggregate_hashtable = 0, :415-447): the table stays
        single-level (bucket -1) until it holds group_by_two_level_threshold groups (the
        reference converts after the block that reaches it, :330-350; groups only grow, so the
        final count decides the same), then emits the non-empty of 256 buckets
        hash2bucket<8, true>(FastHash(key)) (HT/partitioned_hashtable.rs:77-83)."""
        if self.distinct is not None:
            return self.distinct.on_finish(1 << self.config.max_radix_bits)
        n_groups = sum(self.hashtable.partition(1, 1)[0])
        if not self.params.enable_experimental_aggregate_hashtable:
            if not n_groups:
                return []
            # HashMethodFixedKeys<u8> / <u16> never convert to two-level: SUPPORT_PARTITIONED is
            # false for them (aggregator_polymorphic_keys.rs:149,189; transform_aggregate_partial.rs:337)
            if n_groups < self.params.group_by_two_level_threshold or \
                    legacy_hash_method(self.params.group_data_types)[0] in (LEGACY_KEYS_U8, LEGACY_KEYS_U16):
                payloads = export_buckets(self.hashtable, 1, LEGACY_SCHEME)
                return [AggregateMeta(SINGLE_LEVEL_BUCKET, payloads[0], 1, legacy=True)]
            payloads = export_buckets(self.hashtable, LEGACY_BUCKETS, LEGACY_SCHEME)
            return [AggregateMeta(b, p, LEGACY_BUCKETS, legacy=True) for b, p in enumerate(payloads) if len(p)]
        tuple_size = payload_tuple_size(self.params.group_data_types, len(self.params.aggregate_functions))
        bits = partial_bucket_bits(self.config, n_groups, tuple_size)
        payloads = export_buckets(self.hashtable, 1 << bits)
        return [AggregateMeta.create_agg_payload(b, p, 1 << bits) for b, p in enumerate(payloads) if len(p)]

    def close(self):
        if self.distinct is not None:
            self.distinct.close()
        else:
            self.hashtable.close()


class TransformPartitionBucket:
    """NewTransformPartitionBucket (AGG/new_transform_partition_bucket.rs:25-576): collects every
    partial's AggregatePayloads, aligns those written with fewer buckets to the largest bucket
    count by repartitioning their rows (partition_payload, :389-429 — here a scratch table merges
    the payload and re-exports it at the larger radix), and emits one Partitioned meta per bucket
    in ascending bucket order."""

    def __init__(self, params: AggregatorParams, device: int = -1):
        self.params = params
        self.device = device
        self.inputs: List[AggregateMeta] = []

    def push(self, metas: Sequence[AggregateMeta]) -> None:
        self.inputs.extend(metas)

    def _partition_payload(self, meta: AggregateMeta, max_partition_count: int, scheme: int = 1) -> List[AggregateMeta]:
        """partition_payload (:389-429) for AggregatePayload, partition_block (:341-387) for
        Serialized: the rows re-inserted into a scratch table (merge_states / batch_merge), then
        exported as records at the larger radix."""
        if meta.distinct is not None:
            from .distinct import repartition_distinct
            return repartition_distinct(self.params, meta, max_partition_count, self.device)
        scratch = AggregateHashTable(self.params, HashTableConfig(True), self.device)
        try:
            if meta.is_serialized():
                _merge_serialized_block(scratch, self.params, meta.serialized)
            else:
                p = meta.payload
                scratch.merge_records(p.records, p.strings, [p.n_records], [p.string_bytes])
            out = export_buckets(scratch, max_partition_count, scheme)
            import torch
            torch.cuda.current_stream().synchronize()  # exports complete before the scratch goes
        finally:
            scratch.close()
        return [AggregateMeta(b, q, max_partition_count, legacy=meta.legacy) for b, q in enumerate(out) if len(q)]

    def _finish_legacy(self) -> List[AggregateMeta]:
        """TransformPartitionBucket (AGG/transform_partition_bucket.rs:140-300): with only
        single-level inputs, one Partitioned meta of bucket -1 (try_push_single_level); once any
        input is two-level, every single-level one is split into the 256 buckets
        (partition_hashtable / partition_block: hash2bucket<8, true> of the key's FastHash) and
        the buckets go out in ascending order (try_push_two_level)."""
        inputs, self.inputs = self.inputs, []
        if all(m.bucket == SINGLE_LEVEL_BUCKET for m in inputs):
            return [AggregateMeta(SINGLE_LEVEL_BUCKET, None, 0, inputs, legacy=True)]
        buckets = {}
        for m in inputs:
            split = [m] if m.bucket != SINGLE_LEVEL_BUCKET else self._partition_payload(m, LEGACY_BUCKETS, LEGACY_SCHEME)
            for a in split:
                buckets.setdefault(a.bucket, []).append(a)
        return [AggregateMeta(b, None, 0, buckets[b], legacy=True) for b in sorted(buckets)]

    def finish(self) -> List[AggregateMeta]:
        if not self.inputs:
            return []
        if any(m.legacy for m in self.inputs):
            return self._finish_legacy()
        maxp = max(m.max_partition_count for m in self.inputs)
        buckets = {}
        for m in self.inputs:
            aligned = [m] if m.max_partition_count == maxp else self._partition_payload(m, maxp)
            for a in aligned:
                buckets.setdefault(a.bucket, []).append(a)
        self.inputs = []
        return [AggregateMeta.create_partitioned(b, buckets[b]) for b in sorted(buckets)]


class TransformFinalAggregate:
    """AGG/transform_aggregate_final.rs:45-343 — per bucket, a fresh final table merges the states
    of every payload (transform_agg_hashtable, :71-156), then the output block
    [agg results..., group cols...]."""

    def __init__(self, params: AggregatorParams, device: int = -1):
        self.params = params
        self.device = device

    @classmethod
    def try_create(cls, params: AggregatorParams, device: int = -1):
        return cls(params, device)

    def transform(self, meta: AggregateMeta) -> DataBlock:
        """AggregatePayload -> combine_payload (merge_states); Serialized -> add_groups with the
        Binary states (batch_merge), as transform_agg_hashtable does for each variant."""
        items = list(meta.data) if meta.is_partitioned() else [meta]
        if any(f.distinct for f in self.params.aggregate_functions):
            from .distinct import final_distinct
            return final_distinct(self.params, items, self.device)
        items = [m for m in items if (m.is_serialized() and m.serialized.num_rows()) or
                 (m.payload is not None and len(m.payload))]
        if not items:
            return self.params.empty_result_block()
        final = AggregateHashTable(self.params, HashTableConfig(False), self.device)
        try:
            for m in items:
                if m.is_serialized():
                    _merge_serialized_block(final, self.params, m.serialized)
                else:
                    p = m.payload
                    final.merge_records(p.records, p.strings, [p.n_records], [p.string_bytes])
            return final.merge_result()
        finally:
            final.close()


def _merge_serialized_block(table: AggregateHashTable, params: AggregatorParams, block: DataBlock) -> None:
    """The Serialized DataBlock's column order is [states..., group columns...]
    (AGG/aggregate_meta.rs:80-84)."""
    na = len(params.aggregate_functions)
    cols = block.columns
    table.merge_serialized(cols[:na], cols[na:], rows=block.num_rows())


def serialize_payload(params: AggregatorParams, meta: AggregateMeta, device: int = -1) -> AggregateMeta:
    """TransformExchangeAggregateSerializer's AggregatePayload arm
    (AGG/serde/transform_exchange_aggregate_serializer.rs:121-240 -> Payload::aggregate_flush,
    EAGG/payload_flush.rs:129-164): one bucket's groups as AggregateMeta::Serialized, the block a
    remote (CPU or GPU) final stage merges."""
    scratch = AggregateHashTable(params, HashTableConfig(True), device)
    try:
        p = meta.payload
        scratch.merge_records(p.records, p.strings, [p.n_records], [p.string_bytes])
        block = scratch.result_serialized()
    finally:
        scratch.close()
    return AggregateMeta.create_serialized(meta.bucket, block, meta.max_partition_count)
