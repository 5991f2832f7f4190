// agg.hpp — host/device shared descriptors of the aggregate hash table.
#pragma once
#include "device.hpp"

// Slot = [entry u64][state words...], `stride_words` u64 per slot, `cap` slots (power of two) plus
// one sentinel slot at index cap (inline keys whose packed value equals EMPTY).
//   inline keys (all group columns fixed-width and packed row-format width <= 8 bytes):
//     entry = packed key bytes (row format of EAGG/payload.rs:100-129: validity bytes, then values)
//   ref keys (strings, Decimal128, wide tuples):
//     entry = salt16 | batch16 | row32 — the reference's Entry (salt | pointer,
//     EAGG/aggregate_hashtable.rs:591-636) with the pointer aimed at the immutable input row
#define SLOT_EMPTY 0xFFFFFFFFFFFFFFFFULL
#define KC_KEY_WORDS 4  // key bytes cached per slot (32) for one non-null String key (Spec::kc_word)

struct Spec {
    int32_t n_keys;
    int32_t inline_keys;
    int32_t inline_width;     // bytes
    int32_t n_aggs;
    int32_t n_words;          // state words (without the entry word)
    int32_t stride_words;     // entry + states, rounded (LDS tables, parked rows, records)
    int32_t tstride;          // HBM table slot words: stride_words, or more with a key cache
    int32_t kc_word;          // 0, or the slot word of the key cache (single non-null String key):
                              // [hdr = hash bits 16..63 | len << 1 | ready][first 32 key bytes]
    int32_t flags_word;       // -1 or word index (1-based, slot word)
    int32_t has_strings;
    uint8_t voff[DBG_MAX_KEYS];  // inline: byte offset of the validity byte
    uint8_t koff[DBG_MAX_KEYS];  // inline: byte offset of the value
    dbg_datatype key_types[DBG_MAX_KEYS];
    // record format (exchange): [hash][key part][state words]
    uint32_t rec_width;
    uint32_t rec_key_off[DBG_MAX_KEYS];  // byte offset of the key value in a record
    uint32_t rec_val_off[DBG_MAX_KEYS];  // byte offset of the validity byte
    uint32_t rec_state_off;
    DAgg aggs[DBG_MAX_AGGS];
    u64 slot_init[DBG_MAX_WORDS];  // initial value of every slot word (EMPTY entry, MIN/MAX identities)
    // partitioned payload (pp.hip): record formats of the radix-partitioned row store
    //   key part: fixed-width keys -> the row format of EAGG/payload.rs:100-129 ([validity bytes]
    //             [values]) padded to 8 bytes; string keys -> [group hash u64][klen u8][blob 39 B]
    //             (blob = per column [validity u8][value | u8 len + bytes]; klen 0xFF = long key,
    //             blob[0..8) = (bid << 32 | row) reference into the retained input)
    //   raw record   = [key part][arg values, each aligned to its width][arg validity bits]
    //   state record = [key part][state words 1..n_words]
    int32_t pp_ok;          // the spec can run partitioned (record widths within bounds)
    int32_t pp_str;         // key part is [hash][klen][blob]
    uint32_t pp_kw;         // key part bytes (multiple of 8)
    uint32_t pp_rw_raw;     // raw record bytes (multiple of 8)
    uint32_t pp_rw_state;   // state record bytes
    uint32_t pp_avoff;      // byte offset of the arg validity bits
    uint32_t pp_sw;         // LDS slot words: [tag][key part][state words]
    u64 pp_klast_mask;      // key bytes of the key part's last word (raw records put args after them)
    uint16_t pp_aoff[DBG_MAX_AGGS];  // raw arg value offset (0: the aggregate takes no argument)
    int16_t pp_avbit[DBG_MAX_AGGS];  // raw arg validity bit (-1: always valid)
    u64* err;               // the handle's CNT_ERR word (device): errors raised inside state updates
    // result-neutral test hooks, read once when the handle is created (host side only):
    // DBG_X_PPSPEC_CAP (a smaller specialised-aggregation LDS table), DBG_X_PPSPEC_DESC=1 (the
    // descriptor kernel for a shape that also has a compile-time instance)
    uint32_t x_pp_cap;      // ~0: none
    int32_t x_pp_desc;
};
#define PP_BLOB 39        // inline blob bytes of a string key part
#define PP_KLEN_LONG 0xFF  // key too long for the blob: reference into the retained input

struct BatchDesc {
    u64 rows;
    int32_t n_fcols, n_nodes;
    int32_t is_records;
    uint32_t rec_width;
    const u8* rec_base;
    // fixed-capacity record segments (dbg_agg_merge_fixed): record i belongs to segment
    // i / seg_records; its record 0 holds [count u64][flags u64], records 1..count are groups
    u64 seg_records;
    DCol keys[DBG_MAX_KEYS];
    DCol args[DBG_MAX_AGGS];
    DCol fcols[DBG_MAX_FCOLS];
    DNode nodes[DBG_MAX_NODES];
};

struct TableDesc {
    u64* slots;
    u64 cap;  // power of two
    u32 stride_words;  // Spec::tstride
    u32 probe_limit;
    u64* counters;  // [0] claims (groups created), [1] overflow rows, [2] overflow records, [3] error bits
    u64* ovf_rows;  // (bid << 32) | row
    u64 ovf_rows_cap;
    u64* ovf_recs;  // [keyref][words...] per record, stride = stride_words
    u64 ovf_recs_cap;
    // per-workgroup parking rows of small LDS tables (merged by the last workgroup of each group,
    // see block_flush in agg.hip): [count u64 x scr_blocks][group tickets u64 x scr_blocks / 2]
    // [group meta u64 x scr_blocks / 2][scr_blocks x SCR_ENTRIES x stride_words]
    // [scr_blocks / SCR_GROUP group rows x SCR_ENTRIES x stride_words] (fused chain)
    u64* scratch;
    u32 scr_blocks;
};
#define SCR_ENTRIES 64
#ifndef SCR_GROUP
#define SCR_GROUP 16  // workgroups per group of the fused chain (C2: 4 / 8 / 16 / 32 / 64 -> 47.1 / 45.5 / 45.0 / 46.0 / 47.8 us)
#endif
#ifndef FLUSH_GROUP
#define FLUSH_GROUP 4  // workgroups per group of the generic insert's parked flush (<= SCR_GROUP)
#endif
inline size_t scr_words(u32 blocks, u32 stride_words) {
    return (size_t)blocks * (2 + (size_t)SCR_ENTRIES * stride_words) + (size_t)(blocks / SCR_GROUP) * SCR_ENTRIES * stride_words;
}
#define DBG_INSERT_MAX_BLOCKS 2048  // grid cap of every insert launch (scratch rows are sized by it)

enum { CNT_CLAIMS = 0, CNT_OVF_ROWS = 1, CNT_OVF_RECS = 2, CNT_ERR = 3, CNT_FIX_FAIL = 4, CNT_FIX_TICKET = 5, CNT_FIN_TICKET = 6,
       CNT_TAIL = 7, CNT_WORDS = 8 };
enum { ERR_DEC_OVERFLOW = 1, ERR_OVF_LOST = 2, ERR_FIXED_INCOMPLETE = 4, ERR_MINMAX_SPIN = 8, ERR_CHAIN_SPIN = 16 };

// ---- device helpers shared by agg.hip and part.hip ----
// Slot placement for inline keys: any good mixer works (placement is not observable); the
// reference hash is recomputed from the key wherever routing needs it.  A bijection of u64
// (xor-shift by 32 and odd multipliers are invertible), so part.hip can sort mixed keys and
// recover the key with slot_unmix.
__host__ __device__ __forceinline__ u64 slot_mix(u64 x) { return hash_prim(x ^ 0x9E3779B97F4A7C15ULL); }
constexpr u64 mul_inverse_u64(u64 c) {
    u64 x = c;  // c * c == 1 (mod 8); each Newton step doubles the correct low bits
    for (int i = 0; i < 6; ++i) x *= 2 - c * x;
    return x;
}
__host__ __device__ __forceinline__ u64 slot_unmix(u64 y) {
    constexpr u64 CI = mul_inverse_u64(0xd6e8feb86659fd93ULL);
    y ^= y >> 32;
    y *= CI;
    y ^= y >> 32;
    y *= CI;
    y ^= y >> 32;
    return y ^ 0x9E3779B97F4A7C15ULL;
}
static_assert(0xd6e8feb86659fd93ULL * mul_inverse_u64(0xd6e8feb86659fd93ULL) == 1, "inverse");

// State updates on an LDS (AS_LDS) or HBM (AS_GLB) slot; the address space is a template
// parameter (see agg.hip: a generic pointer compiles to FLAT atomics).
#define AS_GLB 1
#define AS_LDS 3
template <int AS> using wptr = __attribute__((address_space(AS))) u64*;
template <int AS> using sptr = __attribute__((address_space(AS))) long long*;
template <int AS> using dptr = __attribute__((address_space(AS))) double*;
template <int AS> using vwptr = volatile __attribute__((address_space(AS))) u64*;
template <int AS> __device__ __forceinline__ wptr<AS> asp(u64* p) { return (wptr<AS>)p; }
template <int AS> __device__ __forceinline__ wptr<AS> asp(const u64* p) { return (wptr<AS>)(u64*)p; }
#define AT_SCOPE(AS) ((AS) == AS_LDS ? __HIP_MEMORY_SCOPE_WORKGROUP : __HIP_MEMORY_SCOPE_AGENT)
template <int AS> __device__ __forceinline__ u64 at_add(wptr<AS> p, u64 v) {
    return __hip_atomic_fetch_add(p, v, __ATOMIC_RELAXED, AT_SCOPE(AS));
}
template <int AS> __device__ __forceinline__ void at_addf(wptr<AS> p, double v) {
    __hip_atomic_fetch_add((dptr<AS>)p, v, __ATOMIC_RELAXED, AT_SCOPE(AS));
}
template <int AS> __device__ __forceinline__ void at_or(wptr<AS> p, u64 v) {
    __hip_atomic_fetch_or(p, v, __ATOMIC_RELAXED, AT_SCOPE(AS));
}
template <int AS> __device__ __forceinline__ void at_minmax(wptr<AS> p, u64 v, bool mn, bool sgn) {
    if (sgn) {
        if (mn) __hip_atomic_fetch_min((sptr<AS>)p, (long long)v, __ATOMIC_RELAXED, AT_SCOPE(AS));
        else __hip_atomic_fetch_max((sptr<AS>)p, (long long)v, __ATOMIC_RELAXED, AT_SCOPE(AS));
    } else {
        if (mn) __hip_atomic_fetch_min(p, v, __ATOMIC_RELAXED, AT_SCOPE(AS));
        else __hip_atomic_fetch_max(p, v, __ATOMIC_RELAXED, AT_SCOPE(AS));
    }
}
// i128 MIN/MAX (Decimal128, precision > 18).  CDNA4 has no 128-bit atomics, so the state is
// [seq, lo, hi] under a seqlock: a candidate that does not beat a consistent snapshot is dropped
// (the value only moves one way, so it never will); otherwise the lane that wins the CAS of seq to
// odd writes both words and publishes seq + 2.  The writes and the publish stay INSIDE the loop
// body (no early exit after the CAS): a block that leaves the loop is a loop exit, which the
// structurizer runs only once every lane of the wave has left — a winner whose publish sat there
// would keep the other lanes of its wave spinning on the odd seq forever.
__device__ __forceinline__ bool i128_less(u64 alo, u64 ahi, u64 blo, u64 bhi) {
    return (long long)ahi < (long long)bhi || (ahi == bhi && alo < blo);
}
// A lane still unsettled after 2^20 rounds gives up and raises ERR_MINMAX_SPIN in *err (finalize
// then fails with DBG_ERR_INTERNAL instead of returning a MIN/MAX that missed the candidate).
template <int AS> __device__ __forceinline__ void at_minmax128(wptr<AS> w, u64 lo, u64 hi, bool mn, u64* err) {
    u32 done = 0;
    u32 spins = 0;  // every iteration settles at least one contender; the cap only guards a hang
    do {
        const u64 s1 = __hip_atomic_load(w, __ATOMIC_ACQUIRE, AT_SCOPE(AS));
        const u64 clo = __hip_atomic_load(w + 1, __ATOMIC_RELAXED, AT_SCOPE(AS));
        const u64 chi = __hip_atomic_load(w + 2, __ATOMIC_RELAXED, AT_SCOPE(AS));
        if (AS == AS_LDS) __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        else __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        const u64 s2 = __hip_atomic_load(w, __ATOMIC_RELAXED, AT_SCOPE(AS));
        if (!(s1 & 1) && s1 == s2) {
            if (!(mn ? i128_less(lo, hi, clo, chi) : i128_less(clo, chi, lo, hi))) {
                done = 1;
            } else {
                u64 e = s1;
                if (__hip_atomic_compare_exchange_strong(w, &e, s1 + 1, __ATOMIC_ACQ_REL, __ATOMIC_RELAXED, AT_SCOPE(AS))) {
                    __hip_atomic_store(w + 1, lo, __ATOMIC_RELAXED, AT_SCOPE(AS));
                    __hip_atomic_store(w + 2, hi, __ATOMIC_RELAXED, AT_SCOPE(AS));
                    __hip_atomic_store(w, s1 + 2, __ATOMIC_RELEASE, AT_SCOPE(AS));
                    done = 1;
                }
            }
        }
        // `done` made opaque at the end of the body: every path, the publish included, has to
        // reach the latch, so no branch can jump-thread the winner's writes into the loop exit
        asm volatile("" : "+v"(done));
    } while (!done && ++spins < (1u << 20));
    if (!done) __hip_atomic_fetch_or(err, (u64)ERR_MINMAX_SPIN, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int AS> __device__ __forceinline__ u64 at_cas(wptr<AS> p, u64 expected, u64 desired) {
    __hip_atomic_compare_exchange_strong(p, &expected, desired, __ATOMIC_RELAXED, __ATOMIC_RELAXED, AT_SCOPE(AS));
    return expected;  // the old value (== the expected one iff the exchange happened)
}
template <int AS> __device__ __forceinline__ u64 vld(wptr<AS> p) { return *(vwptr<AS>)p; }

// device-scope (L2-bypassing) load of a word another workgroup of this launch may write
__device__ __forceinline__ u64 ld_sc1(const u64* p) {
    return __hip_atomic_load((wptr<AS_GLB>)(u64*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Phase timestamps inside kernels (experiments only): compiled in by `make TRACE=1`
// (-DDBG_PHASE_TRACE, scripts/gpu_trace_c2.sh); the shipped library carries no trace code.
#ifdef DBG_PHASE_TRACE
constexpr bool kPhaseTrace = true;
#else
constexpr bool kPhaseTrace = false;
#endif

// Experiment knobs (DBG_X_*: ablations, alternative kernels, tile shapes) are read only by a
// library built with `make EXP=1` (-DDBG_EXPERIMENTS).  The shipped library never reads them, so
// a stray environment variable cannot change what it computes; the test hooks it keeps are
// DBG_X_PPSPEC_CAP and DBG_X_PPSPEC_DESC (a smaller LDS table / the descriptor kernel for the
// specialised pp aggregation: same results).
#ifdef DBG_EXPERIMENTS
constexpr bool kExperiments = true;
#define X_ENV(name) getenv(name)
#else
constexpr bool kExperiments = false;
#define X_ENV(name) ((const char*)nullptr)
#endif

struct FusedFin;
// ---- launch wrappers (agg.hip) ----
// part.hip: radix-partitioned COUNT(*) insert for high-cardinality single integer keys
u32 part_slice_bits(const Spec& S, const BatchDesc& hb, u64 rows, u64 cap);  // 0 = not eligible
size_t part_temp_bytes(int width, u64 rows, u32 sb, u64 cap);
hipError_t launch_part_insert(hipStream_t s, const BatchDesc& hb, u64 rows, const TableDesc& t, u32 sb, void* temp,
                              size_t temp_bytes, u64* sorted, u64* bounds, bool table_empty, const char** step);
hipError_t launch_part_sort(hipStream_t s, const BatchDesc& hb, u64 rows, u64 cap, u32 sb, void* temp, size_t temp_bytes,
                            u64* sorted, u64* bounds, const char** step);
hipError_t launch_part_slices(hipStream_t s, const TableDesc& t, u32 sb, const u64* sorted, const u64* bounds, bool table_empty,
                              const char** step);
u64 part_direct_status_words(u64 cap, u32 sb);
hipError_t launch_part_direct(hipStream_t s, const TableDesc& t, u32 sb, const u64* sorted, const u64* bounds, u64* status, int key_width,
                              void* out_key, u64* out_cnt, u64 cap_groups, u64* totals);
void launch_table_init(hipStream_t s, const Spec* dspec, const Spec& hspec, u64* slots, u64 cap, u64* zero_counters = nullptr);
void launch_insert(hipStream_t s, const Spec* dspec, const Spec& hspec, const BatchDesc* batches, u32 bid, u64 rows,
                   bool records, const TableDesc& t, bool use_lds, const BatchDesc* host_batch = nullptr,
                   const FusedFin* fused = nullptr);
void launch_retry(hipStream_t s, const Spec* dspec, const Spec& hspec, const BatchDesc* batches, const TableDesc& t,
                  u64 n_rows, u64 n_recs, const u64* rows_list, const u64* recs_list);
void launch_rehash(hipStream_t s, const Spec* dspec, const Spec& hspec, const BatchDesc* batches, const u64* old_slots,
                   u64 old_cap, const TableDesc& t);
// finalize: counts per block of occupied slots (and string bytes per key col); returns blocks used
u64 finalize_blocks(u64 cap);
// scheme 0: hash % n; 1: radix bits [48 - r, 48); 2: lpart[slot] (legacy buckets, launch_legacy_slot_bucket)
struct LegacyLayout;
void launch_prefix_slot_bucket(hipStream_t s, const Spec* dspec, const BatchDesc* batches, const TableDesc& t, int nk, u32 n_parts,
                               int scheme, u32* out);
void launch_legacy_slot_bucket(hipStream_t s, const Spec* dspec, const BatchDesc* batches, const TableDesc& t, const LegacyLayout& L,
                               u32* out);
void launch_pp_grec_legacy_bucket(hipStream_t s, const Spec* dspec, const BatchDesc* batches, const u8* grec, u64 n,
                                  const LegacyLayout& L, u32* out);
void launch_count_groups(hipStream_t s, const Spec* dspec, const Spec& hspec, const BatchDesc* batches, const TableDesc& t,
                         u32 n_parts, int scheme, const u32* lpart, u64* hist /* [n_parts][blocks] */, u64* str_hist /* [n_parts][n_keys][blocks] */);
void launch_exclusive_scan(hipStream_t s, u64* data, u64 n, u64* total);
struct OutDesc {
    void* key_data[DBG_MAX_KEYS];
    u64* key_offsets[DBG_MAX_KEYS];
    u8* key_valid[DBG_MAX_KEYS];  // bytes (packed later)
    void* agg_data[DBG_MAX_AGGS];
    u8* agg_valid[DBG_MAX_AGGS];  // bytes
    u64 cap_groups;               // rows the output buffers hold
    u64 cap_str[DBG_MAX_KEYS];    // payload bytes the string key buffers hold
    u8* key_bits[DBG_MAX_KEYS];   // bit-packed destinations of key_valid (fused path)
    u8* agg_bits[DBG_MAX_AGGS];
    // serialize mode (dbg_agg_result_serialized): agg_data[a] receives each group's borsh state
    // at row * ser_stride[a], agg_valid[a] its length in bytes
    int32_t ser;
    u32 ser_stride[DBG_MAX_AGGS];
    // aggregates whose every group is valid (non-nullable argument): no validity bytes are
    // written (agg_valid[a] null) and the packers set agg_bits[a] to all ones
    u32 all_valid;
};
// validity bits byte k of an all-valid column of n rows
__host__ __device__ __forceinline__ u8 all_valid_byte(u64 n, u64 k) {
    const u64 i0 = k * 8;
    return i0 + 8 <= n ? (u8)0xFF : (i0 < n ? (u8)((1u << (n - i0)) - 1) : (u8)0);
}
void launch_fill_valid(hipStream_t s, u64 n, u8* bits);
#define FIN_SMALL_SLOTS 16384  // tables up to this many slots finalize in one workgroup
void launch_finalize_small(hipStream_t s, const Spec* dspec, const BatchDesc* batches, const TableDesc& t, const OutDesc& out,
                           u64* totals, u64* host_mirror /* mapped pinned: counters, totals, recycled, seq */,
                           int recycle, u64 seq);
void launch_finish_outputs(hipStream_t s, const OutDesc& out, const u64* totals, int n_keys, int n_aggs);
void launch_ser_compact(hipStream_t s, const u8* lens, const u8* src, u32 stride, u64 n, u64* offs, u8* dst, u64* total);
// finalize_small fused into the fast insert: the last workgroup to finish runs it (one launch per
// batch).  Tables of at most FUSED_FIN_SLOTS slots whose copy fits the insert's LDS.
#define FUSED_FIN_SLOTS 2048
// host mirror words: [0, CNT_WORDS) counters, CNT_WORDS totals (+ string bytes per key), then
// recycled, seq, and the compact word [seq << 25 | recycled << 24 | groups] that the count-only
// fused finalize posts alone when its counters are known (no wait between mirror stores)
#define MIRROR_COMPACT (CNT_WORDS + 3 + DBG_MAX_KEYS)
struct FusedFin {
    OutDesc out;
    u64* totals;
    u64* host_mirror;
    u64 seq;
    int recycle;
    int on;
    int table_empty;  // the HBM table held no group when the launch started (fused chain)
    u64* trace;  // EXPERIMENT (DBG_X_TRACE): phase timestamps of this launch, s_memrealtime ticks
    // direct-mapped hand-off for COUNT(*) over keys of <= 16 bits (fused_dense): dense_n counts then
    // dense_n / 64 bitmap words, all zero between launches; nullptr = the parked-row chain
    u64* dense;
    u32 dense_n;
};
// host side: would launch_insert of this batch take the fast kernel (and so could fuse)?
bool insert_can_fuse(const Spec& S, const BatchDesc& hb, u64 cap);
void launch_write_results(hipStream_t s, const Spec* dspec, const Spec& hspec, const BatchDesc* batches, const TableDesc& t,
                          const u64* pos /* scanned hist */, const u64* str_pos, const OutDesc& out);
void launch_pack_bits(hipStream_t s, const u8* bytes, u64 n, u8* bits);
void launch_export_fixed(hipStream_t s, const Spec* dspec, const BatchDesc* batches, const TableDesc& t, u8* buf, u64 cap_records,
                         int recycle);
void launch_export(hipStream_t s, const Spec* dspec, const Spec& hspec, const BatchDesc* batches, const TableDesc& t,
                   u32 n_parts, int scheme, const u32* lpart, const u64* pos, const u64* str_pos, u8* rec_out, u8* str_out,
                   const u64* part_str_base);

// ---- partitioned payload (pp.hip) ----
// A scatter/count work unit: `n` rows of batch `bid` from row `start` (raw input, level 1) or `n`
// records of a record buffer from index `start` (levels >= 2); `group` = the source partition.
struct PPChunk {
    u64 start;
    u64 n;
    u32 bid;
    u32 group;
};
#define PP_L1_BITS 8
#define PP_CHUNK 262144  // rows / records per scatter work unit
// direct scatter tiles: rows whose records are built in a 32 KiB LDS scratch per step (pp.hip)
#define PP_NT 512  // threads per workgroup of the partitioned-payload kernels
#define PP_SCRATCH_BYTES (32 * 1024)
__host__ __device__ __forceinline__ u32 pp_direct_t(u32 rw) {  // threads with a row per step (0: too wide)
    const u32 t = PP_SCRATCH_BYTES / rw;
    return t >= PP_NT ? PP_NT : (t & ~63u);
}
// sample probe: distinct group hashes among sampled selected rows -> out[0] selected, [1] distinct,
// [2] singletons (f1), [3] doubletons (f2)
void launch_pp_sample(hipStream_t s, const Spec* dspec, const BatchDesc* batches, u32 bid, u64 rows, u64 n_sample,
                      u64* set, u64 set_cap, u64* out);
// level scatter: src = 0 raw batch rows (records built from the batch), 1 records of `src_recs`
void launch_pp_count(hipStream_t s, const Spec* dspec, const BatchDesc* batches, int src, int kind, const u8* src_recs,
                     const PPChunk* chunks, u32 n_chunks, u32 shift, u32 kbits, u32* cnt, u32 wpr = 0);
// off[unit][bucket]: relative start of the unit's run inside partition (group, bucket);
// part_off[g * K + b]: partition starts (G * K + 1 words); scratch: pp_scan_scratch_words
u64 pp_scan_scratch_words(u32 n_groups, u32 kbits);
void launch_pp_scan(hipStream_t s, const u32* cnt, u32 n_chunks, u32 kbits, const u32* group_c0, u32 n_groups, u64* off,
                    u64* part_off, u64* scratch);
void launch_pp_scatter(hipStream_t s, const Spec* dspec, const Spec& hspec, const BatchDesc* batches, int src, int kind,
                       const u8* src_recs, const PPChunk* chunks, u32 n_chunks, u32 shift, u32 kbits, const u64* off,
                       const u64* part_off, u8* dst, u32* cnt_next = nullptr, u32 sh_next = 0, u32 kb_next = 0);
// the next level's counts fused into a records scatter (cnt_next, zeroed: one unit per destination
// partition, cnt_next[(group * K + b) << kb_next | digit]) when this LDS bound holds
#define PP_NEXT_HIST_MAX 8192
// Level 1 from raw columns, specialised (pp.hip): kind 1 = fixed-width non-null keys and
// arguments (<= 8 columns, records <= 64 bytes) with an optional `column <cmp> constant` on a
// fixed-width non-null integer column; kind 2 = one non-null String key, no arguments, optional
// `key <cmp> 'constant'`.
struct PPFast {
    int32_t kind;   // 0 none (generic kernels), 1 fixed, 2 one string key
    u32 ncol, nk;   // loaded columns (keys first), keys
    u32 wpr;        // raw record words
    u32 bid;
    const u8* ptr[8];
    u8 width[8];
    u8 type[8];
    u16 off[8];     // byte offset of the value in the record
    int32_t has_pred, pcmp, ptype;
    u32 pwidth;
    const u8* pptr;
    i64 pconst;
    const u64* soffs;  // kind 2
    const u8* sdata;
    const u8* pstr;
    u64 pstr_len;
    uint16_t* dig;  // kind 1 scatter: the next 16 hash bits below the level-1 digit of each record, at
                    // the record's index (level 2 counts these instead of re-reading the records)
};
// level-2 histograms from the level-1 digit array: bucket = dig >> (16 - kbits)
void launch_pp_count_dig(hipStream_t s, const PPChunk* chunks, u32 n_chunks, const uint16_t* dig, u32 kbits, u32* cnt);
int launch_pp_l1_fast(hipStream_t s, const PPFast& F, int count, const PPChunk* chunks, u32 n_chunks, u32* cnt, const u64* off,
                      const u64* part_off, u8* dst);
// aggregation of the final partitions in LDS; mode 0: result columns (fixed-width keys), mode 1:
// group records (state record format) in `grec`.  counters: [0] row cursor, [1] overflow records
struct PPAggOut {
    OutDesc cols;   // mode 0
    u8* grec;       // mode 1
    u64 grec_cap;
    u64* tot;       // PPT_* words (device)
    u64* trace;     // EXPERIMENT (DBG_X_PPTRACE): summed phase durations of sampled workgroups
};
// device totals of one partitioned finalize: groups, string bytes per key column, extra rounds, errors
enum { PPT_GROUPS = 0, PPT_STR = 1, PPT_ROUNDS = 1 + DBG_MAX_KEYS, PPT_ERR = 2 + DBG_MAX_KEYS, PPT_WORDS = 4 + DBG_MAX_KEYS };
u32 pp_agg_slots(const Spec& hspec);
struct CopyRange {
    u64 src, dst, n;  // byte offsets / length (multiples of 8)
};
void launch_copy_ranges(hipStream_t s, const u8* src, u8* dst, const CopyRange* dranges, u32 n);
// plist (device): [count, partition ids...] — aggregate only those partitions (nullptr: all); plist_cap
// bounds the count (grid size)
void launch_pp_agg(hipStream_t s, const Spec* dspec, const Spec& hspec, const BatchDesc* batches, int mode, u32 n_parts,
                   const u64* raw_off, const u64* st_off, u8* raw, u8* raw_alt, u8* st, u8* st_alt, const PPAggOut& out,
                   const u32* plist = nullptr, u32 plist_cap = 0);
// Record-centric aggregation (raw records only, <= PP_RC_W words): one workgroup per partition,
// aggregated in 2^sub_bits LDS rounds by the hash bits [sub_shift, sub_shift + sub_bits) — a round's
// records in LDS, a table of record indices, states beside the records.  A partition of more than
// PP_RC_MAXN records, or with a round larger than one LDS table, is listed in spill ([count,
// ids...], spill_cap ids at most) for launch_pp_agg.
#define PP_RC_W 4
#define PP_RC_PART 4096  // records per partition the level sizes aim at (PP_RC_MAXN = 8192 at most)
// specialised aggregation (pp.hip pp_agg_spec_kernel): the shape id of a Spec (its raw record
// words), -1 if the Spec is outside the kernel's class; cap = its LDS table slots, max_records =
// records of one partition it holds
int pp_spec_shape(const Spec& hspec, u32* cap, u32* max_records);
void launch_pp_agg_spec(hipStream_t s, const Spec& hspec, int shape, int mode, u32 n_parts, const u64* raw_off, const u8* raw,
                        u32 sub_bits, const PPAggOut& out, u32* spill, u32 spill_cap);
u32 pp_rc_records(const Spec& hspec);  // records one LDS round holds
bool pp_rc_ok(const Spec& hspec);
void launch_pp_agg_rc(hipStream_t s, const Spec* dspec, const Spec& hspec, const BatchDesc* batches, int mode, u32 n_parts,
                      const u64* raw_off, const u8* raw, u32 sub_shift, u32 sub_bits, const PPAggOut& out, u32* spill,
                      u32 spill_cap);
// group records -> result columns (deterministic positions: block sums, scan, write)
void launch_pp_grec_lengths(hipStream_t s, const Spec* dspec, const u8* grec, const u64* n_dev, u64* blk_len /* [n_keys][blocks] */,
                            u64 nblocks, const BatchDesc* batches);
u64 pp_grec_blocks(u64 n);
void launch_pp_grec_write(hipStream_t s, const Spec* dspec, const BatchDesc* batches, const u8* grec, const u64* n_dev,
                          const u64* str_pos /* [n_keys][blocks] scanned */, u64 nblocks, const OutDesc& out, u64* err);
// group records -> exchange records partitioned by hash % n (scheme 0) or radix bits (scheme 1)
void launch_pp_grec_count_parts(hipStream_t s, const Spec* dspec, const BatchDesc* batches, const u8* grec, u64 n,
                                u32 n_parts, int scheme, const u32* lpart, u64* hist /* [n_parts][blocks] */,
                                u64* str_hist /* [n_parts][n_keys][blocks] */, u64 nblocks);
void launch_pp_grec_export(hipStream_t s, const Spec* dspec, const BatchDesc* batches, const u8* grec, u64 n, u32 n_parts,
                           int scheme, const u32* lpart, const u64* pos, const u64* str_pos, u64 nblocks, u8* rec_out, u8* str_out,
                           const u64* part_str_base);
