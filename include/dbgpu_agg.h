/*
 * dbgpu_agg.h — C ABI of the MI355X-native filter + hash GROUP BY path for Databend.
 *
 * This is the drop-in boundary.  Every entry point replaces one seam of the
 * reference's Rust pipeline; the seam is cited next to each declaration.  Paths are relative to
 * the Databend tree (sundy-li/databend @ 2024-10-24):
 *   EAGG/ = src/query/expression/src/aggregate/
 *   AGG/  = src/query/service/src/pipelines/processors/transforms/aggregator/
 *   FUN/  = src/query/functions/src/aggregates/
 *   EXP/  = src/query/expression/src/
 *
 * Conventions (mirroring the reference):
 *  - Every function returns a status code; DBG_OK == 0.  The message of the last failure on the
 *    calling thread is returned by dbg_last_error() (reference: Result<_, ErrorCode>).
 *  - Column buffers use Databend's in-memory layout (EXP/values.rs:157-176): fixed-width values are
 *    contiguous little-endian; Decimal128 is i128 LE; String is bytes + (len+1) u64 offsets
 *    (EXP/types/string.rs:220-223); validity and Boolean are arrow Bitmaps, LSB-first with a bit
 *    offset (EXP/types/nullable.rs:245-248).  No torch types appear in any signature.
 *  - A handle is used by one thread at a time (TransformPartialAggregate::transform takes &mut self);
 *    distinct handles may be used concurrently.  Each handle owns a HIP stream (or borrows the
 *    caller's, see dbg_agg_set_stream) and its device memory.
 *  - on_device == 0: column pointers are host memory, borrowed for the duration of the call only.
 *    on_device == 1: pointers are device memory on the handle's device; the table refers to key
 *    rows in place (the reference's Entry points into its payload, here into the input), so these
 *    buffers must stay valid and unmodified until dbg_agg_reset or dbg_agg_destroy returns.
 *    Host inputs are copied to device memory owned by the handle for the same lifetime.
 */
#ifndef DBGPU_AGG_H
#define DBGPU_AGG_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DBG_ABI_VERSION 1

/* ---- status codes (reference ErrorCode variants on this path) ---- */
enum {
    DBG_OK = 0,
    DBG_ERR_OVERFLOW = 1,    /* ErrorCode::Overflow — FUN/aggregate_sum.rs:147-153, aggregate_avg.rs:195-199 */
    DBG_ERR_OOM = 2,         /* device allocation failed */
    DBG_ERR_UNSUPPORTED = 3, /* type/function not on the GPU path: caller keeps the CPU path */
    DBG_ERR_INTERNAL = 4,    /* ErrorCode::Internal */
    DBG_ERR_INVALID = 5,     /* malformed argument */
    DBG_ERR_DEVICE = 6       /* HIP runtime failure */
};

/* ---- data types (EXP/types/: Number, Decimal128, Date, Timestamp, String, Boolean) ---- */
typedef enum {
    DBG_INT8 = 0,
    DBG_INT16 = 1,
    DBG_INT32 = 2,
    DBG_INT64 = 3,
    DBG_UINT8 = 4,
    DBG_UINT16 = 5,
    DBG_UINT32 = 6,
    DBG_UINT64 = 7,
    DBG_FLOAT32 = 8,
    DBG_FLOAT64 = 9,
    DBG_DECIMAL128 = 10, /* i128 LE, (precision, scale) — EXP/types/decimal.rs:653-655 */
    DBG_DATE = 11,       /* i32 days since epoch */
    DBG_TIMESTAMP = 12,  /* i64 microseconds since epoch */
    DBG_STRING = 13,     /* bytes + offsets */
    DBG_BOOLEAN = 14     /* bitmap */
} dbg_type;

typedef struct dbg_datatype {
    int32_t type;      /* dbg_type */
    uint8_t precision; /* Decimal128 only */
    uint8_t scale;     /* Decimal128 only */
    uint8_t nullable;  /* DataType::Nullable(..) wrapper */
    uint8_t reserved;
} dbg_datatype;

/* One Column (EXP/values.rs:157) — NullableColumn = inner column + validity Bitmap. */
typedef struct dbg_column {
    dbg_datatype dt;
    const void* data;         /* values; STRING: payload bytes; BOOLEAN: LSB-first bitmap */
    const uint64_t* offsets;  /* STRING: len+1 offsets into data; otherwise NULL */
    const uint8_t* validity;  /* read only when dt.nullable; NULL = all valid */
    uint64_t validity_offset; /* bit offset of row 0 in validity */
    uint64_t data_offset;     /* BOOLEAN: bit offset of row 0 in data; otherwise 0 */
    uint64_t len;             /* rows */
} dbg_column;

/* Writable output column: caller-allocated buffers sized from dbg_agg_finalize.
 * data: n_groups * width (STRING: string_bytes); offsets: n_groups+1 (STRING);
 * validity: ceil(n_groups/8) bytes, written LSB-first from bit 0 (only for nullable results). */
typedef struct dbg_out_column {
    dbg_datatype dt; /* filled by the library (result type) */
    void* data;
    uint64_t* offsets;
    uint8_t* validity;
} dbg_out_column;

/* ---- aggregate functions (FUN/aggregate_{count,sum,avg,min_max_any}.rs) ---- */
typedef enum {
    DBG_AGG_COUNT = 0, /* AggregateCountFunction: count(*) when arg_type < 0, count(x) otherwise */
    DBG_AGG_SUM = 1,   /* NumberSumState / DecimalSumState<OVERFLOW> */
    DBG_AGG_MIN = 2,   /* MinMaxAnyState<T, CmpMin> */
    DBG_AGG_MAX = 3,   /* MinMaxAnyState<T, CmpMax> */
    DBG_AGG_AVG = 4,   /* NumberAvgState / DecimalAvgState<OVERFLOW> */
    /* SQL avg(x): the planner rewrites it to sum(x) / if(count(x) = 0, 1, count(x))
     * (SQL/planner/semantic/aggregate_rewriter.rs:145-208); fused here into one aggregate with
     * AVG's state.  Numbers: f64 / f64 (the value NumberAvgState gives).  Decimal128(p, s): SUM's
     * state and range check, then the decimal divide by the count as Decimal(20, 0)
     * (FUNCS/scalars/decimal/arithmetic.rs:87-112): result Decimal(38, max(s, min(s + 6, 12)))
     * (EXP/types/decimal.rs:1015-1018), rounded half away from zero (do_round_div, :480-489). */
    DBG_AGG_AVG_SQL = 5
} dbg_agg_kind;

typedef struct dbg_agg_spec {
    int32_t kind;     /* dbg_agg_kind */
    dbg_datatype arg; /* arg.type < 0 => no argument (count(*)) */
    uint8_t or_null;  /* wrapped by AggregateFunctionOrNullAdaptor (factory.get(): 1) */
    uint8_t reserved[3];
} dbg_agg_spec;

/* ---- predicates (EXP/filter/select_expr.rs SelectExpr tree, flattened to postfix) ---- */
typedef enum { DBG_CMP_EQ = 0, DBG_CMP_NE, DBG_CMP_LT, DBG_CMP_LE, DBG_CMP_GT, DBG_CMP_GE } dbg_cmp;

typedef enum {
    DBG_PRED_CMP_CONST = 0, /* column <cmp> constant (constant in the column's own domain) */
    DBG_PRED_CMP_COLS = 1,  /* column <cmp> column2 (same type) */
    DBG_PRED_AND = 2,       /* pops 2, pushes 1 (SQL three-valued logic) */
    DBG_PRED_OR = 3,
    DBG_PRED_NOT = 4,       /* pops 1 */
    DBG_PRED_IS_NULL = 5,
    DBG_PRED_IS_NOT_NULL = 6,
    DBG_PRED_TRUE = 7
} dbg_pred_op;

typedef struct dbg_pred_node {
    int32_t op;   /* dbg_pred_op */
    int32_t cmp;  /* dbg_cmp */
    int32_t col;  /* index into dbg_filter.cols */
    int32_t col2; /* DBG_PRED_CMP_COLS */
    /* constant, interpreted by the column type: signed ints/date/timestamp/bool -> i64;
     * unsigned ints -> u64 bits in i64; floats -> f64; Decimal128 -> (i128_hi:i128_lo) at the
     * column's scale; String -> str/str_len bytes */
    int64_t i64;
    double f64;
    uint64_t i128_lo;
    int64_t i128_hi;
    const uint8_t* str;
    uint64_t str_len;
} dbg_pred_node;

/* A filter = predicate program over its own columns (TransformFilter over a DataBlock). */
typedef struct dbg_filter {
    const dbg_pred_node* nodes; /* postfix */
    int32_t n_nodes;
    int32_t n_cols;
    const dbg_column* cols;
} dbg_filter;

/* ---- aggregate hash table handle (EAGG/aggregate_hashtable.rs:47 AggregateHashTable) ---- */
typedef struct dbg_agg_handle dbg_agg_handle;

typedef struct dbg_agg_params {
    const dbg_datatype* group_types; /* AggregatorParams.group_data_types (AGG/aggregator_params.rs:31-94) */
    int32_t n_group_cols;
    const dbg_agg_spec* aggs; /* AggregatorParams.aggregate_functions */
    int32_t n_aggs;
    int32_t device;         /* HIP device ordinal; -1 = current device */
    int32_t partial;        /* 1 = TransformPartialAggregate, 0 = TransformFinalAggregate */
    uint64_t capacity_hint; /* expected groups; 0 = AggregateHashTable::initial_capacity() (32768) */
} dbg_agg_params;

const char* dbg_version(void);
/* Message of the last error on this thread (thread-local). */
const char* dbg_last_error(void);
int dbg_device_count(int* n);

/* Result type of an aggregate: AggregateFunction::return_type() after the factory's adaptors
 * (FUN/aggregate_function_factory.rs:157-220). */
int dbg_agg_result_type(const dbg_agg_spec* spec, dbg_datatype* out);

/* AggregateHashTable::new + HashTableConfig (builder_aggregate.rs:132-164). */
int dbg_agg_create(const dbg_agg_params* params, dbg_agg_handle** out);
void dbg_agg_destroy(dbg_agg_handle* h);
/* Launch on the caller's hipStream_t (NULL restores the handle's own stream).  The switch is
 * ordered on the device (work on the new stream waits for all work queued on the old one); the
 * host does not block, so a caller may alternate streams per call to overlap handles. */
int dbg_agg_set_stream(dbg_agg_handle* h, void* hip_stream);
/* Drop all groups and retained inputs, keep device memory (a fresh table for the next query). */
int dbg_agg_reset(dbg_agg_handle* h);

/* TransformPartialAggregate::transform -> AggregateHashTable::add_groups
 * (AGG/transform_aggregate_partial.rs:291-323, EAGG/aggregate_hashtable.rs:128-242), fused with the
 * TransformFilter that precedes it when filter != NULL (transform_filter.rs:73-92).
 * arg_cols holds n_aggs entries, one per aggregate (ignored for count(*)).  Asynchronous on the
 * handle's stream. */
int dbg_agg_add_groups(dbg_agg_handle* h, const dbg_column* group_cols, const dbg_column* arg_cols,
                       const dbg_filter* filter, uint64_t rows, int on_device);

/* Synchronise, resolve deferred work and report the result size (merge_result preparation,
 * EAGG/aggregate_hashtable.rs:427-451).  string_bytes[i] = payload bytes of group column i
 * (0 for non-string columns); may be NULL. */
int dbg_agg_finalize(dbg_agg_handle* h, uint64_t* n_groups, uint64_t* string_bytes);

/* TransformFinalAggregate output DataBlock [agg results..., group cols...]
 * (AGG/transform_aggregate_final.rs:128-133): fills caller buffers (host when on_device == 0). */
int dbg_agg_result(dbg_agg_handle* h, dbg_out_column* out_aggs, dbg_out_column* out_keys, int on_device);
/* AggregateMeta::Serialized (AGG/aggregate_meta.rs:44-109; EAGG/payload_flush.rs:129-164): the
 * partial states as Binary columns, one per aggregate, + the group columns — what the reference
 * ships over Flight or spills, so a CPU final stage (or a GPU one) merges them.  Each row is the
 * reference's own bytes: the borsh state (NumberSumState / DecimalSumState {value},
 * Number/DecimalAvgState {value, count: u64}, AggregateCountState u64, MinMaxAnyState
 * {value: Option<T>} in T's own width), then AggregateNullUnaryAdaptor's flag byte (nullable
 * argument), then AggregateFunctionOrNullAdaptor's flag byte (FUN/aggregator_common.rs:159-170,
 * adaptors/aggregate_null_unary_adaptor.rs:200-207, adaptors/aggregate_ornull_adaptor.rs:175-179).
 * After dbg_agg_finalize; out_states[a] is a Binary column: data sized n_groups * stride[a]
 * (dbg_agg_serialized_stride, an upper bound: MIN/MAX of a group without input is shorter),
 * offsets n_groups + 1.  Group order equals dbg_agg_result's.  SQL avg (DBG_AGG_AVG_SQL) has no
 * single reference state: DBG_ERR_UNSUPPORTED. */
int dbg_agg_serialized_stride(dbg_agg_handle* h, uint32_t* stride /* n_aggs */);
int dbg_agg_result_serialized(dbg_agg_handle* h, dbg_out_column* out_states, dbg_out_column* out_keys, int on_device);

/* AggregateMeta::Serialized -> this table: the final stage's ingest of a partial that crossed the
 * wire or went to spill as [Binary state per aggregate..., group columns...]
 * (SerializedPayload::convert_to_aggregate_table, AGG/aggregate_meta.rs:57-101, reached from
 * TransformFinalAggregate::transform_agg_hashtable, AGG/transform_aggregate_final.rs:71-156, and
 * NewTransformPartitionBucket::partition_block, AGG/new_transform_partition_bucket.rs:341-387).
 * Each row's group is probed and every state is merged with AggregateFunction::merge's meaning
 * (batch_merge, EAGG/aggregate_function.rs:96-103): the bytes are the layout
 * dbg_agg_result_serialized writes (borsh state, NullUnary flag, OrNull flag).  state_cols[a] is a
 * non-null Binary column (dt.type = DBG_STRING, offsets rows + 1) for aggregate a; group_cols as
 * in dbg_agg_add_groups.  Errors: DBG_ERR_INVALID when a state's length does not match its
 * aggregate; DBG_ERR_UNSUPPORTED for SQL avg, or for a state whose NULL result the GPU state
 * cannot carry (OrNull flag 0 / None on a non-nullable argument: states the reference's partial
 * never writes).  Device inputs are retained like dbg_agg_add_groups'; parse errors are reported
 * by this call (it synchronises the stream once). */
int dbg_agg_merge_serialized(dbg_agg_handle* h, const dbg_column* state_cols, const dbg_column* group_cols, uint64_t rows,
                             int on_device);

/* Fused finalize + result into device buffers (on_device outputs) in one host round trip:
 * count, scan and write are enqueued together and the group count is read back once.  Buffers
 * hold max_groups rows (and max_string_bytes[c] payload bytes per string key column, may be NULL
 * without string keys).  *n_groups / string_bytes are always set; if the buffers were too small
 * the call returns DBG_ERR_INVALID and can be repeated with larger ones (the table is intact). */
int dbg_agg_finalize_into(dbg_agg_handle* h, dbg_out_column* out_aggs, dbg_out_column* out_keys,
                          uint64_t max_groups, const uint64_t* max_string_bytes, uint64_t* n_groups,
                          uint64_t* string_bytes);

/* The same in two halves: _async enqueues the finalize (the output columns fill in stream order)
 * and returns; _wait delivers *n_groups / string_bytes (and any error) — other launches can be
 * enqueued in between, e.g. the next batch's insert into another handle.  At most one finalize
 * per handle is in flight; the out column structs are copied by _async. */
int dbg_agg_finalize_into_async(dbg_agg_handle* h, dbg_out_column* out_aggs, dbg_out_column* out_keys,
                                uint64_t max_groups, const uint64_t* max_string_bytes);
int dbg_agg_finalize_wait(dbg_agg_handle* h, uint64_t* n_groups, uint64_t* string_bytes);

/* Recycle mode (default off): a dbg_agg_finalize_into that delivers every group of a small table
 * (low cardinality, finalized in one workgroup) also re-initialises the table in that same
 * launch, leaving the handle as dbg_agg_reset would — the result columns are then the only copy
 * of the groups, and the next dbg_agg_reset costs no launch.  The partial table of
 * TransformPartialAggregate is dropped after on_finish (transform_aggregate_partial.rs:449-465),
 * so a processor that reuses one handle per batch stream loses nothing.
 * Also in recycle mode: the insert of an on-device dbg_agg_add_groups that takes the fast path
 * (one non-null integer key, optional `key <op> constant` filter, small table) is enqueued by the
 * NEXT call on the handle, and a dbg_agg_finalize_into(_async) then runs insert and finalize in
 * one launch (the last workgroup of the insert finalizes).  The device columns of such a batch
 * must therefore stay unchanged until that next call returns — true of DataBlocks, which are
 * immutable once produced (EXP/block.rs).  Launch errors of the insert surface from that call. */
int dbg_agg_set_recycle(dbg_agg_handle* h, int on);
/* Bucket groups in dbg_agg_partition schemes 0 / 1 by the group hash of their first `n_keys` key
 * columns (0 = all, the default).  A DISTINCT aggregate's pair table (keys..., x) set to the
 * query's key count lands every pair in the bucket of its group (AggregateDistinctCombinator's set
 * travels inside the group's state, src/query/functions/src/aggregates/
 * aggregate_combinator_distinct.rs:94-105).  Table strategy only (DBG_ERR_UNSUPPORTED once the
 * handle is partitioned). */
int dbg_agg_set_partition_keys(dbg_agg_handle* h, int n_keys);

/* Host-block staging (default off).  The reference hands TransformPartialAggregate blocks of at
 * most max_block_size = 65,536 rows (src/query/settings/src/settings_default.rs:131), one
 * AggregateHashTable::add_groups per block (AGG/transform_aggregate_partial.rs:291-323).  With
 * staging on, a host-resident (on_device = 0) dbg_agg_add_groups appends the block's rows to a
 * host staging area of `rows` rows and returns; the staged rows go to the device as one batch
 * when the area is full, when a block arrives with a different filter program, and before any
 * call that reads the table (finalize, result, partition, export, merge) — so results are those
 * of one add_groups per block.  Type and length errors are still reported by the appending call;
 * device errors of a staged batch surface from the call that flushes it.  A block of >= `rows`
 * rows, and every on_device call, is added directly (after a flush).  dbg_agg_reset discards
 * staged rows.  rows = 0 turns staging off (after a flush). */
int dbg_agg_set_host_staging(dbg_agg_handle* h, uint64_t rows);

/* Aggregation strategy of a handle (set after create or reset, before any batch):
 *   DBG_STRATEGY_AUTO        — the first large batch (>= 4M rows) into an empty handle is probed
 *                              (distinct group hashes of 2^20 sampled rows); an estimated > 1M groups
 *                              selects the partitioned payload, otherwise the HBM table.  The
 *                              reference adapts the same way at run time (clear_ht / radix
 *                              repartition of a partial table, EAGG/aggregate_hashtable.rs:225-239,
 *                              453-503).
 *   DBG_STRATEGY_TABLE       — always the HBM hash table with LDS staging (low / mid cardinality).
 *   DBG_STRATEGY_PARTITIONED — always the radix-partitioned payload (PartitionedPayload,
 *                              EAGG/partitioned_payload.rs:100-143): batches are scattered into
 *                              hash partitions, finalize aggregates each partition in LDS.
 * In partitioned mode a capacity_hint (dbg_agg_params) is the expected group count that sizes the
 * final partitions; dbg_agg_export_fixed / dbg_agg_merge_fixed return DBG_ERR_UNSUPPORTED. */
enum { DBG_STRATEGY_AUTO = 0, DBG_STRATEGY_TABLE = 1, DBG_STRATEGY_PARTITIONED = 2 };
/* Setting a strategy also forgets the cardinality the handle's last finalize observed (which
 * otherwise decides the next first batch's strategy and table size without a probe). */
int dbg_agg_set_strategy(dbg_agg_handle* h, int strategy);
/* *partitioned = the handle's current mode (0 table, 1 partitioned payload, 2 partitioned payload
 * whose last finalize ran the compile-time specialised aggregation); *extra_rounds (may be NULL) =
 * partitions of the last partitioned finalize whose groups needed more than one LDS round. */
int dbg_agg_get_strategy(dbg_agg_handle* h, int* partitioned, uint64_t* extra_rounds);

/* ---- partial-state records: exchange / partition bucket (EAGG/payload.rs:356-391,
 *      EAGG/partitioned_payload.rs:100-143, AGG/aggregate_exchange_injector.rs:154-235) ----
 * A record = [hash u64][group keys, fixed part][state words]; string keys are (u64 offset, u64 len)
 * into a per-partition string blob.  scheme 0: partition = hash % n_parts (cluster routing,
 * StrengthReducedU64); scheme 1: partition = (hash & mask) >> (48 - r) with n_parts = 2^r
 * (radix buckets); scheme 2: the legacy HashMethod path's buckets (enable_experimental_aggregate_
 * hashtable = 0), partition = hash2bucket<r, true>(FastHash(key)) = bits [32 - r, 32) of the
 * CRC32C FastHash of the group's FixedKeys / SingleBinary key (HT/partitioned_hashtable.rs:77-83,
 * HT/traits.rs:172-330; the key packing as dbg_legacy_group_hash), n_parts = 2^r — 256 for the
 * reference's PartitionedHashtable<_, 8>.  Scheme 2 with HashMethodSerializer keys (String +
 * anything, Boolean, > 32 packed bytes) returns DBG_ERR_UNSUPPORTED.  Records still carry the new
 * group hash at offset 0 whatever the scheme. */
int dbg_agg_record_width(dbg_agg_handle* h, uint32_t* width);
/* The record layout of a handle built from `params`, computed on the host (no device needed): a
 * mixed CPU/GPU exchange or a test packs and unpacks records with it.  Offsets are in bytes from
 * the record start; the group hash (u64) is at 0; a string key's (offset u64, len u64) pair is at
 * key_off; state word j (1-based, as agg_w0 / flags_word count them) is the u64 at
 * state_off + 8 * (j - 1).  SUM/AVG of Decimal128 hold (lo, hi) words, AVG appends its count;
 * MIN/MAX of Decimal128 with precision > 18 hold (sequence, lo, hi): the sequence word is even in
 * every exported record and is ignored by a merge. */
typedef struct dbg_record_layout {
    uint32_t width;
    uint32_t state_off;
    uint32_t key_off[8];
    uint32_t validity_off[8]; /* nullable key columns only */
    int32_t agg_w0[32];       /* first state word of each aggregate */
    int32_t agg_words[32];
    int32_t flags_word;       /* -1: no "has input" flags word (OrNull of nullable arguments) */
    int32_t n_words;
} dbg_record_layout;
int dbg_agg_record_layout(const dbg_agg_params* params, dbg_record_layout* out);
int dbg_agg_partition(dbg_agg_handle* h, uint32_t n_parts, int scheme, uint64_t* rec_counts,
                      uint64_t* string_bytes);
/* Write every partition's records, partition-major and contiguous, into dev_records
 * (rec_counts[p] records of `width` bytes for p = 0..n_parts-1) and every partition's string blob
 * into dev_strings (string_bytes[p] bytes each, same order; record string offsets are relative to
 * the partition's blob).  Device buffers; asynchronous.  Call after dbg_agg_partition. */
int dbg_agg_export_records(dbg_agg_handle* h, void* dev_records, void* dev_strings);
/* Key compaction: a table with referenced keys (String, Decimal128, wide tuples) points at the
 * input rows that created its groups, so by default the inputs stay resident until
 * dbg_agg_reset.  dbg_agg_compact rewrites the table so that it references one record batch of
 * exactly its groups (keys, string bytes, states) — the reference's payload arena holds only new
 * groups' keys too (EAGG/payload_row.rs:111-130) — after which the caller's device input columns
 * of earlier dbg_agg_add_groups calls may be freed and the library's copies of host blocks are
 * released.  O(groups) device work, synchronous.  A no-op for inline keys and in partitioned mode
 * (*compacted, may be NULL: 1 when the table was rewritten).
 * dbg_agg_retained_bytes reports the device bytes the handle keeps for its inputs (copies of host
 * blocks, received and compacted records; not the caller's own device columns). */
int dbg_agg_compact(dbg_agg_handle* h, int* compacted);
int dbg_agg_retained_bytes(dbg_agg_handle* h, uint64_t* bytes);
/* merge_states of received records into this table (combine_payload,
 * EAGG/aggregate_hashtable.rs:383-425).  The buffers hold n_segments concatenated segments
 * (one per source, each as written by dbg_agg_export_records for one partition);
 * seg_records[i] / seg_string_bytes[i] give each segment's size.  Device buffers, retained like
 * on_device inputs (until dbg_agg_reset / dbg_agg_destroy). */
int dbg_agg_merge_records(dbg_agg_handle* h, const void* dev_records, const void* dev_strings,
                          int32_t n_segments, const uint64_t* seg_records,
                          const uint64_t* seg_string_bytes);

/* ---- multi-GPU exchange over RCCL ----
 * Replaces, for the final-merge stage, the cluster shuffle of AggregateMeta between nodes
 * (AGG/aggregate_exchange_injector.rs:154-354: Payload::scatter by hash % n, EAGG/payload.rs:
 * 356-391, then Flight).  One process (or thread) per GPU; the host distributes a unique id the
 * way the reference's cluster layer distributes its endpoints, every rank creates its
 * communicator with it, then calls dbg_agg_exchange collectively: the partial table's groups are
 * routed to rank hash % n_ranks, sizes move with one RCCL all-gather (the only host round trip),
 * records and string blobs with grouped send/recv over xGMI, and what arrives is merged into the
 * rank's final table (merge_states).  Group sets of the ranks' finals are disjoint afterwards.
 * RCCL is loaded on first use (DBG_ERR_UNSUPPORTED without it; DBG_RCCL_LIB overrides its path). */
#define DBG_COMM_ID_BYTES 128
typedef struct dbg_comm dbg_comm;
typedef struct dbg_exchange_stats {
    uint64_t sent_bytes;             /* records + blobs this rank exported */
    uint64_t remote_bytes;           /* of which left the GPU (xGMI) */
    uint64_t received_records;
    uint64_t received_string_bytes;
} dbg_exchange_stats;
int dbg_comm_get_unique_id(uint8_t* id /* DBG_COMM_ID_BYTES */);
int dbg_comm_create(const uint8_t* id, int n_ranks, int rank, int device /* -1 = current */, dbg_comm** out);
void dbg_comm_destroy(dbg_comm* c);
/* Collective over the communicator's ranks.  partial and final live on the communicator's device
 * and have the same dbg_agg_params (partial = 1 / 0).  Asynchronous except for the size
 * all-gather; stats may be NULL.  A rank whose partition or export fails still takes part in the
 * size all-gather and in one ok-flag all-gather before any send or receive, so every rank returns
 * an error together and none is left blocked.  Send buffers live in the communicator and receive
 * buffers in the final table (grown only, reused once the table has been reset), so a repeated
 * step allocates no device memory. */
int dbg_agg_exchange(dbg_comm* c, dbg_agg_handle* partial, dbg_agg_handle* final_table, dbg_exchange_stats* stats);
/* The byte plan dbg_agg_exchange follows on rank `rank` (host only, no device work):
 * all_sizes[s * 2n + 2d + {0, 1}] = the records / string bytes source s sends rank d (as
 * gathered); record_width receives the params' exchange record bytes (may be NULL);
 * send_bytes[d] / send_bytes[n + d] = this rank's record / blob bytes for rank d (export order);
 * recv_bytes[s] / recv_bytes[n + s] and recv_records[s] = what source s sends this rank (merge
 * order).  Offsets are the prefix sums. */
int dbg_merge_exchange_plan(const dbg_agg_params* params, uint32_t n_ranks, uint32_t rank, const uint64_t* all_sizes,
                            uint32_t* record_width, uint64_t* send_bytes, uint64_t* recv_bytes, uint64_t* recv_records);

/* ---- before-partial shuffle of the partitioned payload (mostly-unique keys) ----
 * group_by_shuffle_mode = before_partial (src/query/settings/src/settings_default.rs:469-473;
 * the rows are scattered before any aggregation, HashFlightScatter, servers/flight/v1/scatter/
 * flight_scatter_hash.rs:133-200).  When every rank's handle is in partitioned mode
 * (dbg_agg_set_strategy(PARTITIONED), fixed-width keys) its level-1 records — written by
 * add_groups, not yet aggregated — are routed by level-1 partition: partition p of 256 (top 8 bits
 * of the group hash) goes to rank p * n / 256, so every group's records meet on one rank and are
 * aggregated once, by that rank's finalize.  Routing differs from HashFlightScatter's SipHash: the
 * exchange is GPU-to-GPU only (a mixed CPU/GPU cluster uses dbg_agg_exchange, before_merge).
 *   counts: part_counts[kind][p] (2 x 256: raw / state records per level-1 partition), widths[kind]
 *           record bytes (host only);
 *   export: the records packed destination-major (kind 0 for ranks 0..n-1, then kind 1), each
 *           destination's records partition-major, into dev_buf (sum of counts x widths bytes);
 *   import: replace the payload with records received from n_ranks sources: raw_records /
 *           state_records source-major, each source's block holding the records of this rank's
 *           partitions; part_counts[source][kind][p] are the sources' counts;
 *   exchange_payload: the whole collective over RCCL (one all-gather of the counts, grouped
 *           send/recv), then import.  DBG_ERR_UNSUPPORTED on every rank if any rank cannot take part.
 * export and import are synchronous (they return with dev_buf written / the records copied):
 * buffers produced or released on another stream need no further ordering. */
int dbg_agg_payload_counts(dbg_agg_handle* h, uint64_t* part_counts /* 2 x 256 */, uint32_t* widths /* 2, may be NULL */);
int dbg_agg_payload_export(dbg_agg_handle* h, uint32_t n_ranks, void* dev_buf);
int dbg_agg_payload_import(dbg_agg_handle* h, uint32_t n_ranks, uint32_t rank, const uint64_t* part_counts /* n x 2 x 256 */,
                           const void* raw_records, const void* state_records);
int dbg_agg_exchange_payload(dbg_comm* c, dbg_agg_handle* h, dbg_exchange_stats* stats);
/* Chunked form, overlapping the transfer with the next chunk's level-1 work.  The payload is a
 * list of level-1 segments (one per add_groups batch); the _from variants count / export the
 * segments from first_seg[kind] on (n_segs receives the current segment counts, may be NULL);
 * import_chunks takes n_chunks shipments: raw_records[c] / state_records[c] laid out as for
 * dbg_agg_payload_import, part_counts[c][source][kind][p].
 * dbg_agg_exchange_payload_chunk ships the segments appended since its previous call on this
 * handle: the chunk's counts all-gathered on the communicator's own stream (no wait for the
 * chunk's scatter), receive buffers per chunk, a collective ok, the export on the table's stream
 * into one of two send buffers, and the grouped send/recv on the communicator's stream behind
 * it — it returns without waiting, so the caller's next add_groups overlaps the transfer.  With
 * last = 1 it also waits for every transfer and imports all chunks (one level-1 segment per chunk
 * and source); until then the handle's finalize must not run.  Every rank makes the same number
 * of calls.  dbg_agg_reset drops an unfinished shuffle's arrivals. */
int dbg_agg_payload_counts_from(dbg_agg_handle* h, const uint32_t first_seg[2], uint64_t* part_counts /* 2 x 256 */,
                                uint32_t* widths, uint32_t* n_segs /* 2 */);
int dbg_agg_payload_export_from(dbg_agg_handle* h, uint32_t n_ranks, const uint32_t first_seg[2], void* dev_buf);
int dbg_agg_payload_import_chunks(dbg_agg_handle* h, uint32_t n_ranks, uint32_t rank, uint32_t n_chunks,
                                  const uint64_t* part_counts /* n_chunks x n x 2 x 256 */, const void* const* raw_records,
                                  const void* const* state_records);
int dbg_agg_exchange_payload_chunk(dbg_comm* c, dbg_agg_handle* h, int last, dbg_exchange_stats* stats);
/* The byte plan dbg_agg_exchange_payload follows on rank `rank` (host only, no device work):
 * all_counts[source][kind][p] (n x 2 x 256) as gathered; widths[kind] receives the params' payload
 * record bytes (may be NULL); send_bytes[kind * n + d] = this rank's kind records of the partitions
 * rank d owns (export order), recv_bytes[kind * n + s] = source s's kind records of this rank's
 * partitions (import order). */
int dbg_payload_exchange_plan(const dbg_agg_params* params, uint32_t n_ranks, uint32_t rank, const uint64_t* all_counts,
                              uint32_t* widths, uint64_t* send_bytes, uint64_t* recv_bytes);

/* ---- fixed-capacity exchange: replicas + gather for low-cardinality tables ----
 * Replaces, for small inline-key partial tables, the Serialized/Flight hand-off of
 * TransformPartialAggregate::on_finish (AGG/transform_aggregate_partial.rs:449-465) to the final
 * node's TransformFinalAggregate (AGG/transform_aggregate_final.rs:71-156).  A buffer holds
 * (cap_records + 1) records of dbg_agg_record_width bytes: record 0 = [u64 group count][u64 flags],
 * records 1..count = the groups ([hash][keys][state words]).  The count stays on the device, so
 * an all-gather of equal-size buffers (RCCL) and the merge run without a host round trip.
 * Inline (fixed-width, <= 8 byte) keys and tables of at most 8192 slots only
 * (DBG_ERR_UNSUPPORTED otherwise: use dbg_agg_partition + dbg_agg_export_records).  A partial
 * with more groups than cap_records, or with unresolved overflow, marks its buffer incomplete;
 * the merging handle's finalize then fails with DBG_ERR_INVALID. */
/* Current slot capacity of the table (a table holds at most capacity + 1 groups). */
int dbg_agg_capacity(dbg_agg_handle* h, uint64_t* slots);
/* In recycle mode (dbg_agg_set_recycle) the export also leaves the table empty, as
 * dbg_agg_reset would. */
int dbg_agg_export_fixed(dbg_agg_handle* h, void* dev_buf, uint64_t cap_records);
/* Merge n_bufs fixed buffers laid end to end (an all-gather output) into h; the buffers are
 * retained until dbg_agg_reset like on_device inputs. */
int dbg_agg_merge_fixed(dbg_agg_handle* h, const void* dev_bufs, int32_t n_bufs, uint64_t cap_records);

/* ---- standalone filter (FilterExecutor::select + take, EXP/filter/filter_executor.rs:73-128) ----
 * sel_out (device) receives the ascending u32 row indices where the predicate is TRUE;
 * *n_sel its count (synchronous). */
int dbg_filter_select(const dbg_filter* filter, uint64_t rows, uint32_t* sel_out, uint64_t* n_sel,
                      void* hip_stream);
/* DataBlock::take (EXP/kernels/take.rs:56-91) of one fixed-width column on device:
 * out[i] = in[sel[i]] (value bytes; validity gathered into out_validity bit-packed when non-NULL). */
int dbg_take_fixed(const dbg_column* col, const uint32_t* sel, uint64_t n_sel, void* out_data,
                   uint8_t* out_validity, void* hip_stream);
/* DataBlock::take of one String column on device (StringColumn, EXP/kernels/take.rs:56-91):
 * out_offsets (n_sel + 1 u64, device) receives the offsets from 0, *total_bytes the payload size;
 * if it exceeds data_cap the call returns DBG_ERR_INVALID with *total_bytes set and no bytes
 * copied (size the buffer and call again), otherwise out_data receives the selected rows' bytes.
 * Validity as dbg_take_fixed.  Synchronous. */
int dbg_take_string(const dbg_column* col, const uint32_t* sel, uint64_t n_sel, uint64_t* out_offsets, void* out_data,
                    uint64_t data_cap, uint8_t* out_validity, uint64_t* total_bytes, void* hip_stream);

/* ---- legacy HashMethod path (enable_experimental_aggregate_hashtable = 0) ----
 * dbg_legacy_hash_method mirrors HashMethodKind::choose_hash_method_with_types
 * (EXP/kernels/group_by.rs:48-97); dbg_legacy_group_hash computes, on device columns, the FastHash
 * of each row's legacy group key (HT/traits.rs:172-330, the x86_64 sse4.2 build: CRC32C of the
 * key's little-endian u64 words from u64::MAX, no final inversion): FixedKeys<T> packs the keys as
 * build_keys_vec does (EXP/kernels/group_by_hash/method_fixed_keys.rs:74-100, 366-470: columns
 * widest first, null bytes after the values), SingleBinary hashes the string bytes (an empty
 * string: u64::MAX).  out_bucket (optional) receives hash2bucket<bucket_bits, true>
 * (HT/partitioned_hashtable.rs:77-83).  Serializer keys (Boolean, mixed strings) return
 * DBG_ERR_UNSUPPORTED.  Synchronous. */
enum {
    DBG_LEGACY_KEYS_U8 = 1, DBG_LEGACY_KEYS_U16, DBG_LEGACY_KEYS_U32, DBG_LEGACY_KEYS_U64, DBG_LEGACY_KEYS_U128,
    DBG_LEGACY_KEYS_U256, DBG_LEGACY_SINGLE_BINARY, DBG_LEGACY_SERIALIZER
};
int dbg_legacy_hash_method(const dbg_datatype* types, int n, int* kind, uint32_t* key_bytes);
int dbg_legacy_group_hash(const dbg_column* cols, int n, uint64_t rows, uint64_t* out_hash, uint32_t* out_bucket,
                          int bucket_bits, void* hip_stream);

/* ---- ORDER BY one column LIMIT k (DataBlock::sort, EXP/kernels/sort.rs:79-107 -> arrow
 * sort_to_indices / indices_sorted_unstable_by, src/common/arrow/src/arrow/compute/sort/common.rs:95-174)
 * over a device-resident fixed-width number column (ints, date, timestamp, float32/64, boolean) —
 * the sort that ends every ClickBench GROUP BY, run on the aggregate result while it is in HBM.
 * idx_out (device, >= min(limit, rows) u32) receives the row indices of the first
 * min(limit, rows) rows in sort order: NULLs first or last (nulls_first) in ascending row order;
 * values by ord::total_cmp (integers) / total_cmp_f32|f64 (floats, IEEE totalOrder), reversed when
 * asc == 0; equal values in ascending row order (the reference leaves their order unspecified:
 * select_nth_unstable_by).  *n_out = min(limit, rows).  limit > 2048, Decimal128 and STRING
 * columns return DBG_ERR_UNSUPPORTED.  Synchronous on hip_stream. */
int dbg_sort_limit_indices(const dbg_column* col, uint64_t rows, int asc, int nulls_first, uint64_t limit,
                           uint32_t* idx_out, uint64_t* n_out, void* hip_stream);
/* ORDER BY several columns LIMIT k: DataBlock::sort with n_cols descriptions (EXP/kernels/sort.rs:
 * 79-107 -> arrow lexsort_to_indices with a limit) over device-resident number, Decimal128 and
 * String columns (1..8, each its own asc / nulls_first).  Rows compare column by column: NULLs
 * first or last per the column's nulls_first; values by ord::total_cmp (integers, i128 decimals),
 * IEEE totalOrder (floats), byte-wise then by length (strings), reversed when asc[c] == 0.  Rows
 * equal on every column come out in ascending row order (the reference leaves them unspecified).
 * idx_out (device, >= min(limit, rows) u32) receives the row indices in order; *n_out =
 * min(limit, rows).  limit > 2048 returns DBG_ERR_UNSUPPORTED.  Synchronous on hip_stream. */
int dbg_sort_limit_multi(const dbg_column* cols, int n_cols, const int* asc, const int* nulls_first, uint64_t rows,
                         uint64_t limit, uint32_t* idx_out, uint64_t* n_out, void* hip_stream);

/* ---- in-library kernel timing (HIP events around each launch; off by default) ---- */
int dbg_prof_enable(int on);
int dbg_prof_reset(void);
/* i-th kernel seen so far: name, summed milliseconds, launches.  Returns DBG_ERR_INVALID past end. */
int dbg_prof_get(int i, const char** name, double* total_ms, uint64_t* launches);
/* An empty kernel (dbg_marker_kernel) on hip_stream: delimits a region in a rocprofv3 trace or
 * counter collection (scripts/pmc_step_traffic.py attributes the dispatches between two markers). */
int dbg_prof_marker(void* hip_stream);

/* ---- synthetic workload generator (the numbers_mt analog) ----
 * Fills caller-allocated device buffers for rows [row_start, row_start+rows) of config cfg,
 * deterministically from seed (counter-based splitmix64, include/dbgpu_datagen.h).  outs[] per cfg:
 *   1: shipdate i32, returnflag bytes, linestatus bytes, returnflag offsets u64 (rows+1),
 *      linestatus offsets, quantity, extprice, discount, tax, disc_price, charge (Decimal128 each)
 *   2: AdvEngineID i16            3: UserID i64
 *   4: WatchID i64, ClientIP i32, IsRefresh i16, ResolutionWidth i16
 *   5: SearchPhrase lengths u64 (pass 1; aux = phrase CDF, 2^23 u64)
 *   6: SearchPhrase bytes (pass 2; outs = {offsets (rows+1), bytes}; aux = phrase CDF) */
int dbg_datagen(int cfg, uint64_t seed, uint64_t row_start, uint64_t rows, void** outs, int n_outs,
                const uint64_t* aux, void* hip_stream);

#ifdef __cplusplus
}
#endif
#endif /* DBGPU_AGG_H */
