"""Test helpers for the scan-side decode: column chunks located through pyarrow's footer reader
(test infrastructure — the Fuse host knows each chunk's offset from its ColumnMeta), pyarrow
types mapped to Databend targets, expected values per row."""
from __future__ import annotations

import datetime as dt
import decimal
import io
import os

import numpy as np
import pyarrow as pa
import pyarrow.parquet as pq

from databend_amd import abi
from databend_amd import column as col
from databend_amd.scan import ColumnChunk

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
CODEC = {"UNCOMPRESSED": abi.PQ_UNCOMPRESSED, "SNAPPY": abi.PQ_SNAPPY, "LZ4": abi.PQ_LZ4_RAW, "LZ4_RAW": abi.PQ_LZ4_RAW, "ZSTD": abi.PQ_ZSTD}
PTYPE = {"BOOLEAN": abi.PQ_BOOLEAN, "INT32": abi.PQ_INT32, "INT64": abi.PQ_INT64, "INT96": abi.PQ_INT96,
         "FLOAT": abi.PQ_FLOAT, "DOUBLE": abi.PQ_DOUBLE, "BYTE_ARRAY": abi.PQ_BYTE_ARRAY,
         "FIXED_LEN_BYTE_ARRAY": abi.PQ_FIXED_LEN_BYTE_ARRAY}


def file_chunks(buf: bytes):
    """[(name, ColumnChunk, arrow type)] of every leaf column of every row group."""
    f = pq.ParquetFile(io.BytesIO(buf))
    md = f.metadata
    out = []
    for g in range(md.num_row_groups):
        rg = md.row_group(g)
        for c in range(rg.num_columns):
            cc = rg.column(c)
            sc = md.schema.column(c)
            start = cc.dictionary_page_offset if cc.has_dictionary_page and cc.dictionary_page_offset else cc.data_page_offset
            ch = ColumnChunk(buf[start:start + cc.total_compressed_size], PTYPE[cc.physical_type], sc.max_definition_level,
                             sc.length or 0, CODEC[cc.compression])
            out.append((cc.path_in_schema, g, ch, f.schema_arrow.field(cc.path_in_schema).type))
    return out


def target_of(t: pa.DataType, nullable: bool = True) -> col.DataType:
    m = {pa.int8(): col.Int8, pa.int16(): col.Int16, pa.int32(): col.Int32, pa.int64(): col.Int64,
         pa.uint8(): col.UInt8, pa.uint16(): col.UInt16, pa.uint32(): col.UInt32, pa.uint64(): col.UInt64,
         pa.float32(): col.Float32, pa.float64(): col.Float64, pa.string(): col.String, pa.large_string(): col.String,
         pa.binary(): col.String, pa.bool_(): col.Boolean, pa.date32(): col.Date}
    if t in m:
        d = m[t]
    elif pa.types.is_timestamp(t):
        d = col.Timestamp
    elif pa.types.is_decimal(t):
        d = col.Decimal128(t.precision, t.scale)
    else:
        raise KeyError(t)
    return d.wrap_nullable() if nullable else d


def expected_values(arr: pa.ChunkedArray, t: pa.DataType) -> list:
    """Row values in the Column.values() form: ints, floats, bytes, bools, scaled decimals."""
    vals = arr.to_pylist()
    out = []
    for v in vals:
        if v is None:
            out.append(None)
        elif pa.types.is_decimal(t):
            out.append(int(v.scaleb(t.scale)))
        elif isinstance(v, str):
            out.append(v.encode())
        elif isinstance(v, dt.datetime):
            out.append(None)  # compared through the physical value instead
        elif isinstance(v, dt.date):
            out.append((v - dt.date(1970, 1, 1)).days)
        else:
            out.append(v)
    if pa.types.is_timestamp(t):
        phys = arr.cast(pa.int64()).to_pylist()
        out = phys
    return out


def sample_table(n: int, seed: int = 1) -> pa.Table:
    """Every physical type the decoder takes, nullable and not, with skewed and unique values."""
    rng = np.random.default_rng(seed)
    words = [("w%03d" % i) * int(1 + i % 5) for i in range(300)]
    return pa.table({
        "i16": pa.array(rng.integers(-300, 300, n).astype(np.int16), mask=rng.random(n) < 0.1),
        "u8": pa.array(rng.integers(0, 256, n).astype(np.uint8)),
        "i32": pa.array(rng.integers(-2**31, 2**31 - 1, n).astype(np.int32)),
        "i64": pa.array(rng.integers(-2**62, 2**62, n), mask=rng.random(n) < 0.02),
        "f32": pa.array(rng.random(n).astype(np.float32)),
        "f64": pa.array(rng.random(n) * 1e6, mask=rng.random(n) < 0.3),
        "s": pa.array([None if rng.random() < 0.05 else words[int(x)] for x in rng.integers(0, 300, n)]),
        "su": pa.array(["row-%d-%s" % (i, "x" * int(i % 23)) for i in range(n)]),
        "b": pa.array(rng.random(n) < 0.3, mask=rng.random(n) < 0.2),
        "d20": pa.array([decimal.Decimal(int(v)).scaleb(-2) for v in rng.integers(-10**15, 10**15, n)], type=pa.decimal128(20, 2)),
        "d38": pa.array([None if i % 7 == 0 else decimal.Decimal(int(v) * 10**20).scaleb(-6) for i, v in
                         enumerate(rng.integers(-10**9, 10**9, n))], type=pa.decimal128(38, 6)),
        "d9": pa.array([decimal.Decimal(int(v)).scaleb(-2) for v in rng.integers(-10**8, 10**8, n)], type=pa.decimal128(9, 2)),
        "date": pa.array(rng.integers(0, 20000, n).astype(np.int32), type=pa.date32()),
        "ts": pa.array(rng.integers(0, 2**50, n), type=pa.timestamp("us")),
    })


def write(t: pa.Table, **kw) -> bytes:
    bio = io.BytesIO()
    pq.write_table(t, bio, **kw)
    return bio.getvalue()
