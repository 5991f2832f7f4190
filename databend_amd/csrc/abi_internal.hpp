// abi_internal.hpp — what the C-ABI translation units share: the handle (one AggregateHashTable in
// HBM), its finalize state, and the error / HIP-check helpers.  abi.hip implements the handle's
// entry points, exchange.hip the multi-GPU exchange over RCCL.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <vector>
#include <chrono>

#include "agg.hpp"
#include "host_stage.hpp"
#include "legacy.hpp"
#include "serde.hpp"

#include "filter.hpp"
#include "sort.hpp"

// ------------------------------------------------------------------------------------------
// errors
// ------------------------------------------------------------------------------------------
int fail(int code, const std::string& msg);

#define HIPCHECK(expr)                                                                         \
    do {                                                                                       \
        hipError_t _e = (expr);                                                                \
        if (_e != hipSuccess)                                                                  \
            return fail(DBG_ERR_DEVICE, std::string(#expr) + ": " + hipGetErrorString(_e));    \
    } while (0)

#define RETURN_IF(rc) \
    do {              \
        int _r = (rc); \
        if (_r != DBG_OK) return _r; \
    } while (0)

// ------------------------------------------------------------------------------------------
// handle
// ------------------------------------------------------------------------------------------
struct DevBuf {
    void* p = nullptr;
    size_t bytes = 0;
};

struct FinState {
    bool active = false;
    std::vector<dbg_out_column> aggs, keys;
    u64 max_groups = 0;
    bool has_max_str = false;
    std::vector<u64> max_str;
    u64 cap_str[DBG_MAX_KEYS] = {};
    bool zero_copy = false;
    u64 seq = 0;
    bool direct = false;  // the held-back partitioned insert's direct stage wrote the results (part_slice_direct)
};

struct dbg_agg_handle {
    int device = 0;
    hipStream_t own_stream = nullptr, stream = nullptr;
    Spec spec{};
    Spec* dspec = nullptr;
    std::vector<dbg_datatype> result_types;
    std::vector<int> src_kinds;  // dbg_agg_kind as created (AVG_SQL is stored as AVG)
    bool partial = true;

    // table
    u64* slots = nullptr;
    u64 cap = 0;
    u64 init_cap = 0;  // from the capacity hint: the table never shrinks below it
    // An on-device fast-path insert whose launch is held back until the next call: a
    // finalize_into_async of a small table then runs in the same launch (FusedFin); any other
    // call launches it first (flush_deferred).
    bool def_on = false;
    bool def_clean = false;  // the table was empty (recycled / reset) when the insert was held back
    u32 def_bid = 0;
    u64 def_rows = 0;
    BatchDesc def_hb;
    u64* counters = nullptr;   // device, CNT_WORDS
    u64* hcounters = nullptr;  // pinned
    u64* hcounters_dev = nullptr;  // its device mapping (finalize_small writes it directly)
    u64* dense = nullptr;          // fused_dense's direct-mapped counts + presence bitmap (zero between launches)
    // overflow lists (deferred)
    u64* ovf_rows = nullptr;
    u64 ovf_rows_cap = 0;
    u64* ovf_recs = nullptr;
    u64 ovf_recs_cap = 0;
    u64 pending_rows = 0, pending_recs = 0;
    // parking rows of per-workgroup partial tables (TableDesc::scratch)
    u64* scratch = nullptr;
    u32 scr_blocks = 0;

    // batches (ids 1..n_batches); descs in device memory, staged through pinned memory
    BatchDesc* dbatches = nullptr;
    u64 batch_cap = 0;
    u32 n_batches = 0;
    // descriptor cache: ids 1..n_cached hold immutable descriptors of device-resident inputs
    // (pointers only), kept across dbg_agg_reset so a re-submitted batch needs no upload
    u32 n_cached = 0;
    std::vector<std::pair<u64, BatchDesc>> desc_cache;  // (content hash, host copy); index = id - 1
    std::vector<BatchDesc*> pinned_descs;   // pinned staging desc per batch id (pooled)
    std::vector<BatchDesc*> pinned_chunks;  // their allocations
    std::vector<DevBuf> owned;             // device copies of host inputs / filter constants
    // before_merge exchange receive buffers (records, string blobs) when this is the final table:
    // kept across resets and grown only, so a step allocates nothing; `xrecv_busy` while the table
    // may reference them (merged since the last reset) — an exchange then allocates fresh ones
    DevBuf xrecv[2];
    bool xrecv_busy = false;
    // chunked before-partial shuffle (dbg_agg_exchange_payload_chunk): level-1 segments from
    // xfirst[k] on are not shipped yet; what arrived per call waits in xchunks until the last call.
    // The receive buffers belong to the communicator (one grow-only pair per chunk slot, received
    // into on its stream), so no step allocates or frees them and the handle never frees memory a
    // transfer may still be writing.
    struct XChunk {
        std::vector<u64> pc;  // [n][2][P] counts of the chunk, every source
        const void* recv[2] = {nullptr, nullptr};
    };
    std::vector<XChunk> xchunks;
    u32 xfirst[2] = {0, 0};

    // finalize state
    bool finalized = false;
    u64 n_groups = 0;
    std::vector<u64> string_bytes;
    u64* d_pos = nullptr;      // scanned per-block group counts
    u64* d_str_pos = nullptr;  // [n_keys][blocks] scanned per column
    u64 pos_cap = 0, str_pos_cap = 0;
    // partition state
    u32 part_n = 0;
    int part_scheme = 0;
    int part_keys = 0;  // dbg_agg_set_partition_keys: buckets by the first part_keys key columns (0 = all)
    u64 part_nb = 0;  // blocks of the partition histogram
    u64* d_part_pos = nullptr;
    u64* d_part_str_pos = nullptr;
    u64* d_part_str_base = nullptr;
    u64 part_cap = 0, part_str_cap = 0;
    u64* d_lpart = nullptr;   // scheme 2: legacy bucket per slot / group record (u32)
    u64 lpart_cap = 0;
    std::vector<u64> part_counts, part_strings;
    // fused finalize: validity bytes staging
    u8* vbytes = nullptr;
    u64 vbytes_cap = 0;
    // fused finalize in flight (dbg_agg_finalize_into_async)
    FinState fin;
    hipEvent_t switch_ev = nullptr;  // dbg_agg_set_stream hand-off
    // recycle mode (dbg_agg_set_recycle): a small-table finalize_into leaves the table empty
    int recycle = 0;
    bool clean = false;           // table already re-initialised by the last finalize
    // dbg_agg_reset deferred the table's initialisation (counters and the sentinel slot are
    // initialised): table_desc() runs it before any kernel touches the table, except a
    // partitioned insert, whose slice kernel starts every slice EMPTY and writes the whole table
    bool init_pending = false;
    u64 fin_seq = 0;              // sequence number the finalize kernel posts to host_mirror
    bool uploads_pending = false; // descriptor uploads from pinned staging since the last sync
    // radix-partitioned insert (part.hip): sorted mixed keys, slice bounds, rocPRIM scratch
    u64* part_sorted = nullptr;
    u64 part_sorted_cap = 0;
    u64* part_bounds = nullptr;
    u64 part_bounds_cap = 0;
    void* part_temp = nullptr;
    size_t part_temp_cap = 0;
    // A partitioned insert into an empty table in recycle mode holds back its table stage (the
    // keys are sorted already): a finalize_into that comes next runs the direct stage instead —
    // groups into the result columns without the table-wide count and write passes, the slots used
    // as scratch and left to be initialised like a reset table (launch_part_direct);
    // anything else that touches the table launches the regular slice stage first (part_flush).
    bool def_part = false;
    u32 def_part_sb = 0;
    int def_part_kw = 0;
    u64* part_status = nullptr;  // the direct stage's look-back words
    u64 part_status_cap = 0;
    u64 table_rows = 0;  // rows / records inserted into the HBM table since the last reset
    u64 remerged = 0;    // of which records dbg_agg_compact merged back (groups, not input rows)
    int strategy = DBG_STRATEGY_AUTO;
    u64 hint_groups = 0;  // dbg_agg_params.capacity_hint
    // cardinality the last table-mode finalize observed (kept across reset): rows / records
    // inserted and the groups they formed.  A handle reused for the next batch of the same query
    // shape decides its strategy from it instead of probing again (no probe kernel, no host sync)
    u64 obs_rows = 0, obs_groups = 0;

    // ---- partitioned payload (pp.hip): high-cardinality mode ----
    bool pp = false;          // batches go to the radix-partitioned payload, not the HBM table
    double pp_ratio = 1.0;    // estimated groups per selected row (cardinality probe)
    double est_groups = 0;    // the probe's (or the last finalize's) group estimate for this batch
    bool pp_probed = false;   // pp_ratio comes from a probe (not the default upper bound)
    struct Seg {
        u64 base, n;
        std::vector<u64> off;  // level-1 partition offsets (257), relative to base
    };
    struct Kind {  // 0: raw records (add_groups), 1: state records (merge_records)
        u8* l1 = nullptr;
        u64 l1_cap = 0, l1_n = 0;  // records
        u16* dig = nullptr;        // level-2 digits of records [0, dig_n) (fixed-shape raw level 1)
        u64 dig_cap = 0, dig_n = 0;
        std::vector<Seg> segs;
        u8* a = nullptr;  // finalize levels: ping-pong buffers, l1_n records each
        u8* b = nullptr;
        u64 ab_cap = 0;
        u64* part = nullptr;  // final partition offsets (device)
        u64 part_cap = 0;
        u8* fin = nullptr;    // final-level buffer and its alternate (the aggregate's overflow)
        u8* alt = nullptr;
    } ppk[2];
    u32 pp_bits = 0;  // final partition bits
    u32 pp_rc_sub = 0;  // > 0: record-centric aggregation in 2^pp_rc_sub rounds per partition (pp.hip)
    int pp_spec = -1;   // >= 0: the compile-time specialised aggregation's shape (pp_agg_spec_kernel)
    u32 pp_spec_sub = 0;  // its rounds per partition: 2^pp_spec_sub
    u32* pp_spill = nullptr;  // [count, partition ids...] spilled by the specialised / record-centric kernel
    u64 pp_spill_cap = 0;     // ids it holds: one per final partition, so no spill is ever dropped
    u32* pp_cnt = nullptr;
    u64 pp_cnt_cap = 0;
    u64* pp_off = nullptr;
    u64 pp_off_cap = 0;
    u64* pp_scan_tmp = nullptr;  // scan scratch (group totals, block sums)
    u64 pp_scan_tmp_cap = 0;
    u64* pp_last_part = nullptr;  // partition offsets of the last count_scan (read by its scatter)
    u64* pp_mid = nullptr;  // intermediate partition offsets (device)
    u64 pp_mid_cap = 0;
    PPChunk* pp_dchunks = nullptr;
    u64 pp_dchunks_cap = 0;
    PPChunk* pp_hchunks = nullptr;  // pinned staging
    u64 pp_hchunks_cap = 0;
    u32* pp_dc0 = nullptr;
    u64 pp_dc0_cap = 0;
    u32* pp_hc0 = nullptr;
    u64 pp_hc0_cap = 0;
    u64* pp_hpart = nullptr;  // pinned read-back of partition offsets
    u64 pp_hpart_cap = 0;
    u64* pp_tot = nullptr;    // PPT_* (device)
    u64* pp_htot = nullptr;   // pinned
    u64* pp_set = nullptr;    // cardinality probe hash set
    u8* pp_grec = nullptr;    // group records (state record format)
    u64 pp_grec_cap = 0;      // bytes
    u64* pp_blk = nullptr;    // per-block string lengths, scanned
    u64 pp_blk_cap = 0;
    bool pp_grec_ready = false;
    u64 pp_nb = 0;            // blocks of the grec passes
    u64 pp_stat_rounds = 0;   // partitions that took more than one LDS round (last finalize)
    u64* ser_err = nullptr;   // serialized-state ingest error bits (serde.hip)

    // host-block staging (dbg_agg_set_host_staging, host_stage.hpp)
    hstage::Stage stage;
};

// handle helpers abi.hip defines for the other units
int dev_alloc(void** p, size_t bytes);
int build_spec(const dbg_agg_params* p, Spec& S, std::vector<dbg_datatype>& rtypes);
// (defined inside abi.hip's extern "C" block; hidden: not part of the library's interface)
extern "C" __attribute__((visibility("hidden"))) int flush_pending(dbg_agg_handle* h);
