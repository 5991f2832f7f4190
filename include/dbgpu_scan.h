/*
 * dbgpu_scan.h — scan side of the GROUP BY path: Parquet column chunks, as a
 * Fuse block stores them, decoded straight into HBM columns that dbg_agg_add_groups reads in
 * place (on_device = 1).  Part of libdbgpu_agg.so; errors through dbg_last_error().
 *
 * Replaces the decode step of the Fuse read path for one leaf column:
 *   BlockReader::deserialize_parquet_chunks        src/query/storages/fuse/src/io/read/block/parquet/mod.rs:45-60
 *     column_chunks_to_record_batch                …/io/read/block/parquet/deserialize.rs:33-80
 *       (arrow-rs `parquet` 52.2.0 ParquetRecordBatchReader over the chunk bytes, then
 *        Column::from_arrow, mod.rs:102-104)
 * for chunks written by blocks_to_parquet (src/query/storages/common/blocks/src/parquet_rs.rs:30-57:
 * one row group, PLAIN, dictionary disabled) with TableCompression None / Snappy / LZ4
 * (table_meta/src/table/table_compression.rs:25-31; Zstd stays on the CPU reader), and the
 * dictionary-encoded chunks of external / stage Parquet files (PLAIN_DICTIONARY, RLE_DICTIONARY).
 *
 * Supported: flat columns (max repetition level 0, max definition level 0 or 1), DATA_PAGE v1 and
 * v2, DICTIONARY_PAGE; encodings PLAIN, PLAIN_DICTIONARY, RLE_DICTIONARY, RLE (BOOLEAN values);
 * codecs UNCOMPRESSED, SNAPPY, LZ4_RAW.  Anything else: DBG_ERR_UNSUPPORTED (the caller keeps the
 * CPU reader).  Malformed pages: DBG_ERR_INVALID (every device read is bounds-checked).
 */
#ifndef DBGPU_SCAN_H
#define DBGPU_SCAN_H

#include "dbgpu_agg.h"

#ifdef __cplusplus
extern "C" {
#endif

/* parquet::format::Type / CompressionCodec values */
enum { DBG_PQ_BOOLEAN = 0, DBG_PQ_INT32 = 1, DBG_PQ_INT64 = 2, DBG_PQ_INT96 = 3, DBG_PQ_FLOAT = 4, DBG_PQ_DOUBLE = 5,
       DBG_PQ_BYTE_ARRAY = 6, DBG_PQ_FIXED_LEN_BYTE_ARRAY = 7 };
enum { DBG_PQ_UNCOMPRESSED = 0, DBG_PQ_SNAPPY = 1, DBG_PQ_ZSTD = 6, DBG_PQ_LZ4_RAW = 7 };

/* One column chunk: the bytes from its first page header (dictionary page if any) to the end of
 * its last page — ColumnMeta::offset_length of the Fuse block (DataItem::RawData, mod.rs:88-104). */
typedef struct dbg_parquet_chunk {
    const uint8_t* host;   /* the chunk bytes in host memory (page headers are parsed on the host) */
    const uint8_t* device; /* the same bytes resident in HBM, or NULL: the call uploads them */
    uint64_t len;
    int32_t physical_type; /* DBG_PQ_* type */
    int32_t type_length;   /* FIXED_LEN_BYTE_ARRAY width (Decimal128: 1..16 bytes, big-endian) */
    int32_t max_def_level; /* 0 required, 1 optional */
    int32_t codec;         /* DBG_PQ_* codec */
} dbg_parquet_chunk;

typedef struct dbg_scan_ctx dbg_scan_ctx;

/* A decode context: device scratch (decompressed pages, level / index / offset staging) reused
 * across chunks, and the HIP stream the kernels run on (NULL = the default stream). */
int dbg_scan_create(dbg_scan_ctx** out, void* hip_stream);
int dbg_scan_destroy(dbg_scan_ctx* ctx);

/* Host-only: the chunk's rows (sum of its data pages' num_values) and pages. */
int dbg_parquet_chunk_rows(const dbg_parquet_chunk* chunk, uint64_t* rows, uint32_t* n_pages);

/* Decode the chunk into caller-allocated device buffers for Databend type `target`:
 *   out->data     rows x width (BOOLEAN: ceil(rows / 8) bitmap bytes; STRING: max_string_bytes),
 *   out->offsets  rows + 1 u64 (STRING),
 *   out->validity ceil(rows / 8) bytes, LSB first (target.nullable; required when nulls occur).
 * Physical -> target as arrow-rs + Column::from_arrow convert them: INT32 -> Int8/16/32,
 * UInt8/16/32, Date, Decimal128 (p <= 9); INT64 -> Int64, UInt64, Timestamp, Decimal128 (p <= 18);
 * FLOAT -> Float32; DOUBLE -> Float64; FIXED_LEN_BYTE_ARRAY -> Decimal128 (big-endian two's
 * complement, sign-extended); BYTE_ARRAY -> String; BOOLEAN -> Boolean.
 * *rows and *string_bytes are always set; a String chunk whose payload exceeds max_string_bytes
 * returns DBG_ERR_INVALID with *string_bytes = the bytes needed (call again with a larger buffer).
 * Synchronises the stream once (device-side error flags and the string total are read back). */
int dbg_parquet_decode(dbg_scan_ctx* ctx, const dbg_parquet_chunk* chunk, dbg_datatype target, dbg_out_column* out,
                       uint64_t max_rows, uint64_t max_string_bytes, uint64_t* rows, uint64_t* string_bytes);

/* ---- Fuse native (strawboat) column pages -> HBM columns ----
 * Replaces, for one leaf column of a block of a `storage_format = 'native'` table,
 * BlockReader::deserialize_native_chunks -> NativeReader / column_iter_to_arrays
 * (FUSE/io/read/block/block_reader_native_deserialize.rs:23-26, 53-...; the pages' format:
 * src/common/arrow/src/native/{write,read,compression}).  The column's pages are the bytes
 * [ColumnMeta::offset, + total_len) with PageMeta {length, num_values} per page (mod.rs:27-72).
 * Page structure (validity, codec headers, Dict / Bitpacking tables) is parsed on the host from
 * `host`; values are decoded on the device.  Codecs: None / Lz4 / Zstd / Snappy, Rle, Dict,
 * OneValue, Bitpacking, DeltaBitpacking for integers (Int8..UInt64, Date, Timestamp); the same
 * minus the bit-packings for Decimal128 (i128 pages) and Float32 / Float64; None / Lz4 / Zstd / Snappy (the bitmap), Rle,
 * OneValue for Boolean; None / Lz4 / Zstd / Snappy, OneValue, Dict for String.  Freq (roaring
 * exceptions), Patas, Decimal256 and nested columns return DBG_ERR_UNSUPPORTED (the CPU reader).
 * Outputs as dbg_parquet_decode. */
typedef struct dbg_native_column {
    const uint8_t* host;          /* the column's pages in host memory */
    const uint8_t* device;        /* the same bytes resident in HBM, or NULL: the call uploads them */
    uint64_t len;
    const uint64_t* page_lengths; /* PageMeta.length, n_pages entries */
    const uint64_t* page_rows;    /* PageMeta.num_values */
    uint32_t n_pages;
    int32_t nullable;             /* the field is Optional: every page starts with its validity */
} dbg_native_column;
int dbg_native_decode(dbg_scan_ctx* ctx, const dbg_native_column* col, dbg_datatype target, dbg_out_column* out,
                      uint64_t max_rows, uint64_t max_string_bytes, uint64_t* rows, uint64_t* string_bytes);

#ifdef __cplusplus
}
#endif
#endif
