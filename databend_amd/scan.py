"""Scan side: Parquet column chunks and native pages decoded into HBM columns.

Host mirror of the Fuse read step this replaces —
`BlockReader::deserialize_parquet_chunks(num_rows, column_metas, column_chunks, compression, ..)`
(src/query/storages/fuse/src/io/read/block/parquet/mod.rs:45-60) and
`column_chunks_to_record_batch` (…/parquet/deserialize.rs:33-80): the chunks of the projected
leaf columns, raw bytes keyed by column id, become columns of one block.  Here each chunk goes
through `dbg_parquet_decode` (include/dbgpu_scan.h) and comes back as a `DeviceColumn` resident in
HBM, ready for `AggregateHashTable.add_groups(..., on_device=True)`.  There is no CPU fallback: a
chunk the GPU decoder declines raises `Unsupported` and the caller keeps the CPU reader, exactly
like the aggregation entry points.

The native (strawboat) format — `storage_format = 'native'` — goes through `dbg_native_decode`:
`deserialize_native_chunks` mirrors BlockReader::deserialize_native_chunks
(…/block/block_reader_native_deserialize.rs): per leaf column the raw page bytes plus the
ColumnMeta::Native page list (PageMeta { length, num_values }).
"""
from __future__ import annotations

import ctypes as C
from dataclasses import dataclass
from typing import Dict, Optional, Sequence

from . import abi
from .column import DataType
from .device import DeviceColumn, empty
from .ffi import check, lib

# TableCompression (storages/common/table_meta/src/table/table_compression.rs:25-31) -> codec
COMPRESSION_CODEC = {"none": abi.PQ_UNCOMPRESSED, "snappy": abi.PQ_SNAPPY, "lz4": abi.PQ_LZ4_RAW, "zstd": abi.PQ_ZSTD}


@dataclass
class ColumnChunk:
    """One leaf column chunk (DataItem::RawData) plus what its ColumnMeta / parquet schema say."""
    data: bytes
    physical_type: int
    max_def_level: int = 1
    type_length: int = 0
    codec: int = abi.PQ_UNCOMPRESSED

    def to_abi(self, keep: list) -> abi.dbg_parquet_chunk:
        buf = C.create_string_buffer(self.data, len(self.data))
        keep.append(buf)
        c = abi.dbg_parquet_chunk()
        c.host = C.cast(buf, C.c_void_p)
        c.device = None
        c.len = len(self.data)
        c.physical_type = self.physical_type
        c.type_length = self.type_length
        c.max_def_level = self.max_def_level
        c.codec = self.codec
        return c


@dataclass
class NativeColumnChunk:
    """One leaf column in the native format: its pages' bytes and ColumnMeta::Native's PageMetas."""
    data: bytes
    page_lengths: Sequence[int]
    page_rows: Sequence[int]
    nullable: bool = False

    def to_abi(self, keep: list) -> abi.dbg_native_column:
        buf = C.create_string_buffer(self.data, max(1, len(self.data)))
        lens = (C.c_uint64 * max(1, len(self.page_lengths)))(*self.page_lengths)
        rows = (C.c_uint64 * max(1, len(self.page_rows)))(*self.page_rows)
        keep += [buf, lens, rows]
        if len(self.page_lengths) != len(self.page_rows):
            raise ValueError("page_lengths and page_rows differ in length")
        c = abi.dbg_native_column()
        c.host = C.cast(buf, C.c_void_p)
        c.device = None
        c.len = len(self.data)
        c.page_lengths = lens
        c.page_rows = rows
        c.n_pages = len(self.page_lengths)
        c.nullable = 1 if self.nullable else 0
        return c

    @property
    def rows(self) -> int:
        return int(sum(self.page_rows))


class ParquetChunkDecoder:
    """A dbg_scan_ctx: device scratch reused across chunks, on one HIP stream."""

    def __init__(self, stream: Optional[int] = None):
        h = C.c_void_p()
        check(lib().dbg_scan_create(C.byref(h), C.c_void_p(stream) if stream else None))
        self.h = h

    def close(self):
        if self.h:
            lib().dbg_scan_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @staticmethod
    def chunk_rows(chunk: ColumnChunk) -> int:
        keep: list = []
        c = chunk.to_abi(keep)
        rows, pages = C.c_uint64(), C.c_uint32()
        check(lib().dbg_parquet_chunk_rows(C.byref(c), C.byref(rows), C.byref(pages)))
        return rows.value

    def decode(self, chunk: ColumnChunk, target: DataType, device="cuda") -> DeviceColumn:
        """The chunk as a device column of Databend type `target`."""
        keep: list = []
        c = chunk.to_abi(keep)
        n = self.chunk_rows(chunk)
        # String payload: the decompressed data pages bound PLAIN values; a dictionary-encoded
        # chunk may expand beyond that, so the call reports the size and is repeated once
        cap = max(64, 2 * len(chunk.data)) if target.type_id == abi.STRING else 0
        for _ in range(2):
            col = empty(target, n, device=device, string_bytes=cap)
            if target.type_id == abi.BOOLEAN:
                import torch
                col.data = torch.zeros(max(1, (n + 7) // 8), dtype=torch.uint8, device=device)
            out = abi.dbg_out_column()
            out.data = col.data.data_ptr()
            out.offsets = col.offsets.data_ptr() if col.offsets is not None else None
            out.validity = col.validity.data_ptr() if col.validity is not None else None
            rows, sbytes = C.c_uint64(), C.c_uint64()
            rc = lib().dbg_parquet_decode(self.h, C.byref(c), target.to_abi(), C.byref(out), n, cap, C.byref(rows),
                                          C.byref(sbytes))
            if rc == abi.DBG_ERR_INVALID and target.type_id == abi.STRING and sbytes.value > cap:
                cap = sbytes.value
                continue
            check(rc)
            return col
        raise RuntimeError("dbg_parquet_decode: string payload size did not converge")

    def decode_native(self, chunk: NativeColumnChunk, target: DataType, device="cuda") -> DeviceColumn:
        """Native pages as a device column of Databend type `target` (integer, Date, Timestamp,
        String); other types and the Freq / Patas codecs raise Unsupported."""
        keep: list = []
        c = chunk.to_abi(keep)
        n = chunk.rows
        # String payload: bounded by the page bytes except for dictionaries and one-value pages,
        # so the call reports the size and is repeated once
        cap = max(64, 2 * len(chunk.data)) if target.type_id == abi.STRING else 0
        for _ in range(2):
            col = empty(target, n, device=device, string_bytes=cap)
            out = abi.dbg_out_column()
            out.data = col.data.data_ptr() if col.data is not None else None
            out.offsets = col.offsets.data_ptr() if col.offsets is not None else None
            out.validity = col.validity.data_ptr() if col.validity is not None else None
            rows, sbytes = C.c_uint64(), C.c_uint64()
            rc = lib().dbg_native_decode(self.h, C.byref(c), target.to_abi(), C.byref(out), n, cap, C.byref(rows),
                                         C.byref(sbytes))
            if rc == abi.DBG_ERR_INVALID and target.type_id == abi.STRING and sbytes.value > cap:
                cap = sbytes.value
                continue
            check(rc)
            return col
        raise RuntimeError("dbg_native_decode: string payload size did not converge")


def deserialize_parquet_chunks(num_rows: int, fields: Dict[int, DataType], column_chunks: Dict[int, ColumnChunk],
                               decoder: Optional[ParquetChunkDecoder] = None) -> Dict[int, DeviceColumn]:
    """BlockReader::deserialize_parquet_chunks for the projected columns: column id -> device column."""
    dec = decoder or ParquetChunkDecoder()
    out = {}
    for cid, chunk in column_chunks.items():
        col = dec.decode(chunk, fields[cid])
        if col.length != num_rows:
            raise ValueError(f"column {cid}: {col.length} rows in the chunk, {num_rows} in the block")
        out[cid] = col
    return out


def deserialize_native_chunks(num_rows: int, fields: Dict[int, DataType], column_chunks: Dict[int, NativeColumnChunk],
                              decoder: Optional[ParquetChunkDecoder] = None) -> Dict[int, DeviceColumn]:
    """BlockReader::deserialize_native_chunks for the projected leaf columns: column id -> device column."""
    dec = decoder or ParquetChunkDecoder()
    out = {}
    for cid, chunk in column_chunks.items():
        col = dec.decode_native(chunk, fields[cid])
        if col.length != num_rows:
            raise ValueError(f"column {cid}: {col.length} rows in the pages, {num_rows} in the block")
        out[cid] = col
    return out
