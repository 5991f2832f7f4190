// agg.hip — gfx950 kernels of the hash GROUP BY path.
//
//   table_init      : slots <- EMPTY entry + per-function initial state words
//   agg_insert      : fused  predicate -> group hash -> LDS-staged partial table -> HBM table
//                     (TransformFilter + AggregateHashTable::add_groups / combine_payload,
//                      EAGG/aggregate_hashtable.rs:128-425)
//   agg_retry       : deferred overflow rows / partial records after the table has grown
//   agg_rehash      : grow the HBM table (AggregateHashTable::resize, :511-561)
//   count / write   : merge_result + flush_column into output columns (:427-451, payload_flush.rs)
//   export          : partial-state records partitioned by hash % n or radix bits
//                     (Payload::scatter, payload.rs:356-391; PartitionedPayload, partitioned_payload.rs)
//
// Bandwidth/atomic-bound integer work: no MFMA.  Every kernel is grid-strided over >= 2048
// workgroups of 256 threads (64-wide waves) or over contiguous row ranges per workgroup.
#include <cstdlib>
#include <cstring>
#include <limits>
#include <type_traits>

#include "legacy.hpp"
#include "agg.hpp"
#include <hip/hip_ext.h>
#include "agg_dev.hpp"

#define BLOCK 256
#define SLOTS_PER_THREAD 8
#define SLOTS_PER_BLOCK (BLOCK * SLOTS_PER_THREAD)
#define LDS_BUDGET_BYTES (32 * 1024)
#define LDS_PROBE_CAP 64
#define FLUSH_ROUND 16  // rounds of BLOCK rows between checks for a full LDS table

// slot_mix (inline-key slot placement) lives in agg.hpp

// ------------------------------------------------------------------------------------------
// Key packing (inline mode): the row format of EAGG/payload.rs:100-129 in <= 8 bytes.
// ------------------------------------------------------------------------------------------

__device__ __forceinline__ u64 pack_key(const Spec& S, const DCol* keys, u64 i) {
    u64 k = 0;
    for (int c = 0; c < S.n_keys; ++c) {
        const DCol& col = keys[c];
        bool v = dcol_valid(col, i);
        if (col.nullable) k |= (u64)(v ? 1 : 0) << (8 * S.voff[c]);
        if (v) {
            u64 b = dcol_bits(col, i);
            if (col.type == DBG_FLOAT32 || col.type == DBG_FLOAT64) b = canon_float_bits(col.type, b);
            k |= (b & width_mask(type_width(col.type))) << (8 * S.koff[c]);
        }
    }
    return k;
}


__device__ __forceinline__ u64 hash_packed(const Spec& S, u64 key, int nk = -1) {
    u64 h = 0;
    if (nk < 0) nk = S.n_keys;
    for (int c = 0; c < nk; ++c) {
        const dbg_datatype& t = S.key_types[c];
        bool v = t.nullable ? ((key >> (8 * S.voff[c])) & 0xff) != 0 : true;
        u64 b = (key >> (8 * S.koff[c])) & width_mask(type_width(t.type));
        u64 x = v ? hash_bits(t.type, b) : NULL_HASH_VAL;
        h = c == 0 ? x : (h * NULL_HASH_VAL) ^ x;
    }
    return h;
}


__device__ __forceinline__ bool ref_equal(const Spec& S, const BatchDesc* batches, const DCol* keys, u64 i, u64 e) {
    const DCol* other = batches[ref_bid(e)].keys;
    u64 j = ref_row(e);
    for (int c = 0; c < S.n_keys; ++c)
        if (!cell_equal(keys[c], i, other[c], j)) return false;
    return true;
}


// Reference group hash of the group an entry stands for.
__device__ __forceinline__ u64 entry_hash(const Spec& S, const BatchDesc* batches, u64 e, bool is_sentinel) {
    if (S.inline_keys) return hash_packed(S, is_sentinel ? SLOT_EMPTY : e);
    return group_hash(batches[ref_bid(e)].keys, S.n_keys, ref_row(e));
}


// ------------------------------------------------------------------------------------------
// Probing
// ------------------------------------------------------------------------------------------
// Find or claim the HBM slot of `key` (inline: packed key; ref: salt|bid|row entry).
// Returns the slot index or ~0 when the probe limit is hit (the caller records an overflow).
template <bool INLINE>
__device__ __forceinline__ u64 g_find(const Spec& S, const BatchDesc* batches, const DCol* keys, u64 i, u64 key,
                                      u64 h, const TableDesc& t, u32 probe_limit, bool& claimed) {
    claimed = false;
    if (INLINE && key == SLOT_EMPTY) {  // only possible for 8-byte packed keys: sentinel slot
        u64 old = at_cas<AS_GLB>(asp<AS_GLB>(t.slots + t.cap * t.stride_words), SLOT_EMPTY, 0ULL);
        claimed = old == SLOT_EMPTY;
        return t.cap;
    }
    u64 mask = t.cap - 1;
    u64 s = (INLINE ? slot_mix(key) : (h >> 16)) & mask;
    for (u32 p = 0; p < probe_limit; ++p) {
        wptr<AS_GLB> e = asp<AS_GLB>(t.slots + s * t.stride_words);
        u64 ev = vld<AS_GLB>(e);
        if (ev == SLOT_EMPTY) {
            u64 old = at_cas<AS_GLB>(e, SLOT_EMPTY, key);
            if (old == SLOT_EMPTY) {
                claimed = true;
                return s;
            }
            ev = old;
        }
        if (INLINE) {
            if (ev == key) return s;
        } else if ((ev >> 48) == (key >> 48) && ref_equal(S, batches, keys, i, ev)) {
            return s;
        }
        s = (s + 1) & mask;
    }
    return ~0ULL;
}

// Same against a table whose entries were claimed from a record/ovf entry that carries a
// foreign key (ref of another batch): compare through the batch table.
template <bool INLINE>
__device__ __forceinline__ u64 g_find_entry(const Spec& S, const BatchDesc* batches, u64 key, u64 h,
                                            const TableDesc& t, u32 probe_limit, bool& claimed) {
    const DCol* keys = INLINE ? nullptr : batches[ref_bid(key)].keys;
    return g_find<INLINE>(S, batches, keys, INLINE ? 0 : ref_row(key), key, h, t, probe_limit, claimed);
}

// LDS partial table: same probing, bounded occupancy; -1 = not staged (use HBM directly).
template <bool INLINE>
__device__ __forceinline__ int lds_find(const Spec& S, const BatchDesc* batches, const DCol* keys, u64 i, u64 key, u64 h,
                                        u64* lds, u32 lmask, u32 sw, u32* lcount, u32 llimit) {
    if (INLINE && key == SLOT_EMPTY) return -1;
    u32 s = (u32)((INLINE ? slot_mix(key) : (h >> 16)) & lmask);
    // Once the table is full (high cardinality), a key found within two probes is staged, any
    // other goes straight to HBM: a long probe through a full table of other keys is wasted LDS
    // traffic.  A key may then hold state both here and in HBM; the flush merges them.
    volatile __attribute__((address_space(3))) u32* lc = (volatile __attribute__((address_space(3))) u32*)lcount;
    const int cap = *lc >= llimit ? 2 : LDS_PROBE_CAP;
    for (int p = 0; p < cap; ++p) {
        wptr<AS_LDS> e = asp<AS_LDS>(lds + (u64)s * sw);
        u64 ev = vld<AS_LDS>(e);
        if (ev == SLOT_EMPTY) {
            if (*lc >= llimit) return -1;
            u64 old = at_cas<AS_LDS>(e, SLOT_EMPTY, key);
            if (old == SLOT_EMPTY) {
                __hip_atomic_fetch_add((__attribute__((address_space(3))) u32*)lcount, 1u, __ATOMIC_RELAXED,
                                       __HIP_MEMORY_SCOPE_WORKGROUP);
                return (int)s;
            }
            ev = old;
        }
        if (INLINE) {
            if (ev == key) return (int)s;
        } else if ((ev >> 48) == (key >> 48) && ref_equal(S, batches, keys, i, ev)) {
            return (int)s;
        }
        s = (s + 1) & lmask;
    }
    return -1;
}

__device__ __forceinline__ void push_ovf_row(const TableDesc& t, u32 bid, u64 row) {
    u64 k = atomicAdd((unsigned long long*)(t.counters + CNT_OVF_ROWS), 1ULL);
    if (k < t.ovf_rows_cap) t.ovf_rows[k] = ((u64)bid << 32) | row;
    else atomicOr((unsigned long long*)(t.counters + CNT_ERR), (unsigned long long)ERR_OVF_LOST);
}
template <bool SC1 = false, int RAS = AS_GLB>
__device__ __forceinline__ void push_ovf_rec(const Spec& S, const TableDesc& t, u64 key, const u64* words) {
    u64 k = atomicAdd((unsigned long long*)(t.counters + CNT_OVF_RECS), 1ULL);
    if (k >= t.ovf_recs_cap) {
        atomicOr((unsigned long long*)(t.counters + CNT_ERR), (unsigned long long)ERR_OVF_LOST);
        return;
    }
    u64* r = t.ovf_recs + k * t.stride_words;
    r[0] = key;
    for (int w = 1; w <= S.n_words; ++w) r[w] = rdw<SC1, RAS>(words + w);
}


// ------------------------------------------------------------------------------------------
// End of an insert launch: merge the workgroup's LDS partial table into the HBM table.
//
// Low cardinality is the hard case for the flush: every workgroup holds the same few hot groups,
// and G workgroups adding into the same HBM slots serialise at the memory side (device-scope
// atomics bypass the per-XCD L2).  So a workgroup whose LDS table holds <= SCR_ENTRIES groups
// parks it, compacted, in its scratch row; the last workgroup to finish (ticket) merges all
// parked rows in its own LDS table and flushes that once.  Larger tables (diverse keys, little
// contention) flush directly.  The combine of partial states follows combine_payload
// (EAGG/aggregate_hashtable.rs:383-425).
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ void st_sc1(u64* p, u64 v) {
    __hip_atomic_store((unsigned long long*)p, (unsigned long long)v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <bool INLINE, bool RECORDS>
__device__ __forceinline__ u64 lds_entry_hash(const Spec& S, const BatchDesc& B, u64 e) {
    if (INLINE) return 0;
    if (RECORDS) return gld<u64>(B.rec_base + (u64)ref_row(e) * B.rec_width);
    return group_hash(B.keys, S.n_keys, ref_row(e));
}

template <bool INLINE, bool RECORDS>
__device__ __forceinline__ void flush_lds_direct(const Spec& S, const BatchDesc* batches, const BatchDesc& B, u64* lds,
                                                 u32 lds_slots, u32 sw, u32 nt, const TableDesc& t, u32& my_claims) {
    for (u32 s = threadIdx.x; s < lds_slots; s += nt) {
        u64* p = lds + (u64)s * sw;
        u64 e = p[0];
        if (e == SLOT_EMPTY) continue;
        u64 h = lds_entry_hash<INLINE, RECORDS>(S, B, e);
        bool claimed;
        u64 gs = g_find<INLINE>(S, batches, B.keys, INLINE ? 0 : ref_row(e), e, h, t, t.probe_limit, claimed);
        if (gs == ~0ULL) {
            push_ovf_rec<false, AS_LDS>(S, t, e, p);
            continue;
        }
        my_claims += claimed ? 1 : 0;
        apply_state<AS_GLB, false, AS_LDS>(S, asp<AS_GLB>(t.slots + gs * t.stride_words), p);
    }
}

__device__ __forceinline__ void lds_table_init(const Spec& S, u64* lds, u32 lds_slots, u32 sw, u32 nt) {
    for (u32 s = threadIdx.x; s < lds_slots; s += nt) {
        u64* p = lds + (u64)s * sw;
        p[0] = SLOT_EMPTY;
        for (u32 w = 1; w < sw; ++w) p[w] = 0;
        for (int a = 0; a < S.n_aggs; ++a)
            if (S.aggs[a].kind == DBG_AGG_MIN || S.aggs[a].kind == DBG_AGG_MAX)
                for (int k = 0; k < S.aggs[a].nwords; ++k) p[S.aggs[a].w0 + k] = state_init_word(S.aggs[a], k);
    }
}

// lcount: [0] LDS claims, [1] HBM claims, [2] parked entries, [3] last-workgroup flag.
// Ends with the workgroup's HBM claims added to the table counter.
template <bool INLINE, bool RECORDS>
__device__ __forceinline__ void block_flush(const Spec& S, const BatchDesc* batches, const BatchDesc& B, u64* lds, u32 lds_slots, u32 sw,
                            u32* lcount, u32 nt, const TableDesc& t, u32 my_claims) {
    const u32 lmask = lds_slots - 1;
    const u32 llimit = lds_slots - lds_slots / 4;
    const bool use_scr = t.scratch != nullptr && gridDim.x > 1 && gridDim.x <= t.scr_blocks;
    if (use_scr) {
        u64* counts = t.scratch;
        u64* tickets = t.scratch + t.scr_blocks;
        u64* rows = t.scratch + 2 * (u64)t.scr_blocks;
        u64* row = rows + (u64)blockIdx.x * SCR_ENTRIES * sw;
        if (lcount[0] <= SCR_ENTRIES) {  // park (uniform: lcount[0] is final after the barrier)
            for (u32 s = threadIdx.x; s < lds_slots; s += nt) {
                const u64* p = lds + (u64)s * sw;
                if (p[0] == SLOT_EMPTY) continue;
                u32 k = atomicAdd(&lcount[2], 1u);
                u64* d = row + (u64)k * sw;
                for (u32 w = 0; w <= (u32)S.n_words; ++w) st_sc1(d + w, p[w]);
            }
            __syncthreads();
            if (threadIdx.x == 0) st_sc1(counts + blockIdx.x, lcount[2]);
        } else {
            if (threadIdx.x == 0) st_sc1(counts + blockIdx.x, 0);
            flush_lds_direct<INLINE, RECORDS>(S, batches, B, lds, lds_slots, sw, nt, t, my_claims);
        }
        // Hand-off without release fences (MI355X_MICROARCH.md, inter-workgroup visibility, valid
        // forms): parked words are stored sc1 (write-through past the XCD's L2); every storing
        // wave drains them and the barrier orders all waves before lane 0's ticket add; the last
        // workgroup of each group of FLUSH_GROUP reads them back with sc1 loads behind one
        // agent-scope acquire.  Groups keep the merge tail short and parallel, and cut the
        // same-address atomics on the HBM table by FLUSH_GROUP (C1, 1464 workgroups of 4 groups:
        // FLUSH_GROUP 2 / 4 / 8 / 16 / 64 -> insert 0.470 / 0.432 / 0.439 / 0.467 / 0.649 ms: a
        // leader's serial merge of many parked tables costs more than the HBM atomics it saves).
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        const u32 g = blockIdx.x / FLUSH_GROUP;
        const u32 gsize = min((u32)FLUSH_GROUP, gridDim.x - g * FLUSH_GROUP);
        if (threadIdx.x == 0) {
            u64 tk = atomicAdd((unsigned long long*)(tickets + g), 1ULL);
            lcount[3] = tk == (u64)gsize - 1 ? 1u : 0u;
        }
        __syncthreads();
        if (lcount[3]) {  // the group's last workgroup: acquire, merge the group's parked rows, flush
            if (threadIdx.x == 0) {
                __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                tickets[g] = 0;  // ready for the next launch on this table (all members have added)
            }
            lds_table_init(S, lds, lds_slots, sw, nt);
            if (threadIdx.x == 0) lcount[0] = 0;
            __syncthreads();
            const u32 total = gsize * SCR_ENTRIES;
            for (u32 f = threadIdx.x; f < total; f += nt) {
                u64 b = (u64)g * FLUSH_GROUP + f / SCR_ENTRIES, k = f % SCR_ENTRIES;
                const u64* r = rows + (b * SCR_ENTRIES + k) * sw;
                u64 cnt = ld_sc1(counts + b);
                u64 e = ld_sc1(r);  // issued with the count: rows are allocated in full
                if (k >= cnt) continue;
                u64 h = lds_entry_hash<INLINE, RECORDS>(S, B, e);
                int ls = lds_find<INLINE>(S, batches, B.keys, INLINE ? 0 : ref_row(e), e, h, lds, lmask, sw, lcount, llimit);
                if (ls >= 0) {
                    apply_state<AS_LDS, true>(S, asp<AS_LDS>(lds + (u64)ls * sw), r);
                    continue;
                }
                bool claimed;
                u64 gs = g_find<INLINE>(S, batches, B.keys, INLINE ? 0 : ref_row(e), e, h, t, t.probe_limit, claimed);
                if (gs == ~0ULL) {
                    push_ovf_rec<true>(S, t, e, r);
                    continue;
                }
                my_claims += claimed ? 1 : 0;
                apply_state<AS_GLB, true>(S, asp<AS_GLB>(t.slots + gs * t.stride_words), r);
            }
            __syncthreads();
            flush_lds_direct<INLINE, RECORDS>(S, batches, B, lds, lds_slots, sw, nt, t, my_claims);
        }
    } else {
        flush_lds_direct<INLINE, RECORDS>(S, batches, B, lds, lds_slots, sw, nt, t, my_claims);
    }
    if (my_claims) atomicAdd(&lcount[1], my_claims);
    __syncthreads();
    if (threadIdx.x == 0 && lcount[1]) atomicAdd((unsigned long long*)(t.counters + CNT_CLAIMS), (unsigned long long)lcount[1]);
}

// ------------------------------------------------------------------------------------------
// table_init
// ------------------------------------------------------------------------------------------
// A memset of the table in 16-byte stores: chunk c is word pair (2k, 2k+1) of slot c / (sw / 2),
// its values from Spec::slot_init (stride_words is even: a power of two >= 2 or a multiple of 8).
typedef unsigned long long v2u64 __attribute__((ext_vector_type(2)));
__global__ void __launch_bounds__(BLOCK) table_init_kernel(const Spec* __restrict__ spec, u64* slots, u64 n_slots, u64* counters) {
    const Spec& S = *spec;
    if (counters && blockIdx.x == 0 && threadIdx.x < CNT_WORDS) counters[threadIdx.x] = 0;  // dbg_agg_reset
    const u32 half = (u32)S.tstride / 2;
    const u64 n_chunks = n_slots * half;
    v2u64 __attribute__((address_space(1)))* out = (v2u64 __attribute__((address_space(1)))*)slots;
    if (half == 1) {
        const v2u64 v = {S.slot_init[0], S.slot_init[1]};
        for (u64 c = blockIdx.x * (u64)BLOCK + threadIdx.x; c < n_chunks; c += (u64)gridDim.x * BLOCK) out[c] = v;
        return;
    }
    for (u64 c = blockIdx.x * (u64)BLOCK + threadIdx.x; c < n_chunks; c += (u64)gridDim.x * BLOCK) {
        u32 k = (u32)(c % half);
        out[c] = v2u64{S.slot_init[2 * k], S.slot_init[2 * k + 1]};
    }
}

void launch_table_init(hipStream_t s, const Spec* dspec, const Spec& hspec, u64* slots, u64 cap, u64* counters) {
    u64 n = (cap + 1) * (u64)(hspec.tstride / 2);
    u64 blocks = (n + BLOCK - 1) / BLOCK;
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL(table_init_kernel, dim3((u32)blocks), dim3(BLOCK), 0, s, dspec, slots, cap + 1, counters);
}

// ------------------------------------------------------------------------------------------
// agg_insert: one workgroup = one contiguous row range; LDS partial table, HBM fallback.
// ------------------------------------------------------------------------------------------
// One selected row (or partial record): group hash -> LDS table -> HBM table -> state update.
template <bool INLINE, bool RECORDS>
__device__ __forceinline__ void insert_one(const Spec& S, const BatchDesc* batches, const BatchDesc& B, u32 bid, u64 i,
                                           u64* lds, u32 lmask, u32 sw, u32* lcount, u32 llimit, const TableDesc& t,
                                           u32& my_claims) {
    u64 h, key;
    if (RECORDS) {
        h = gld<u64>(B.rec_base + i * (u64)B.rec_width);
    } else if (INLINE) {
        h = 0;
    } else {
        h = group_hash(B.keys, S.n_keys, i);
    }
    if (INLINE) key = pack_key(S, B.keys, i);
    else key = (h & 0xFFFF000000000000ULL) | ((u64)bid << 32) | i;

    int ls = lds_find<INLINE>(S, batches, B.keys, i, key, h, lds, lmask, sw, lcount, llimit);
    const u64* rec = RECORDS ? (const u64*)(B.rec_base + i * (u64)B.rec_width + S.rec_state_off) - 1 : nullptr;
    if (ls >= 0) {
        wptr<AS_LDS> st = asp<AS_LDS>(lds + (u64)ls * sw);
        if (RECORDS) apply_state<AS_LDS>(S, st, rec);
        else apply_row<AS_LDS>(S, st, B, i);
        return;
    }
    bool claimed;
    u64 gs = g_find<INLINE>(S, batches, B.keys, i, key, h, t, t.probe_limit, claimed);
    if (gs == ~0ULL) {
        push_ovf_row(t, bid, i);
        return;
    }
    my_claims += claimed ? 1 : 0;
    wptr<AS_GLB> st = asp<AS_GLB>(t.slots + gs * t.stride_words);
    if (RECORDS) apply_state<AS_GLB>(S, st, rec);
    else apply_row<AS_GLB>(S, st, B, i);
}

// Every FLUSH_ROUND rounds: a full LDS table is flushed to HBM and started over (the
// reference's clear_ht of a full partial table, aggregate_hashtable.rs:225-239), so hot keys of
// a skewed stream keep being combined in LDS instead of hammering one HBM slot (not once the HBM
// table overflows: the deferred-overflow lists are sized for two flushes of every workgroup's
// table).  Thread 0 decides, so the branch is uniform.  Called by every thread.
template <bool INLINE, bool RECORDS>
__device__ __forceinline__ void maybe_flush(const Spec& S, const BatchDesc* batches, const BatchDesc& B, u64* lds,
                                            u32 lds_slots, u32 sw, u32* lcount, u32 llimit, const TableDesc& t,
                                            u32& my_claims) {
    __shared__ u32 do_flush;
    if (threadIdx.x == 0)
        do_flush = lcount[0] >= llimit && ld_sc1(t.counters + CNT_OVF_ROWS) == 0 && ld_sc1(t.counters + CNT_OVF_RECS) == 0;
    __syncthreads();
    const bool flush_now = do_flush;
    __syncthreads();  // everyone has read the flag before thread 0 may rewrite it
    if (flush_now) {
        flush_lds_direct<INLINE, RECORDS>(S, batches, B, lds, lds_slots, sw, BLOCK, t, my_claims);
        __syncthreads();
        lds_table_init(S, lds, lds_slots, sw, BLOCK);
        if (threadIdx.x == 0) lcount[0] = 0;
        __syncthreads();
    }
}

template <bool INLINE, bool RECORDS>
__global__ void __launch_bounds__(BLOCK) agg_insert_kernel(const Spec* __restrict__ spec, const BatchDesc* __restrict__ batches,
                                                          u32 bid, u64 rows, u64 rows_per_block, TableDesc t,
                                                          u32 lds_slots, u32 lenq) {
    extern __shared__ __attribute__((aligned(16))) u64 lds[];
    const Spec& S = *spec;
    const BatchDesc& B = batches[bid];
    const u32 sw = S.stride_words;
    u32* lcount = (u32*)(lds + (u64)lds_slots * sw);  // [0] lds claims, [1] hbm claims
    const u32 lmask = lds_slots - 1;
    const u32 llimit = lds_slots - lds_slots / 4;

    lds_table_init(S, lds, lds_slots, sw, BLOCK);
    if (threadIdx.x < 4) lcount[threadIdx.x] = 0;
    __syncthreads();
    auto insert_row = [&](u64 i, u32& my_claims) {
        insert_one<INLINE, RECORDS>(S, batches, B, bid, i, lds, lmask, sw, lcount, llimit, t, my_claims);
    };

    u64 r0 = (u64)blockIdx.x * rows_per_block;
    u64 r1 = r0 + rows_per_block < rows ? r0 + rows_per_block : rows;
    u32 my_claims = 0;
    const u64 n_iter = r1 > r0 ? (r1 - r0 + BLOCK - 1) / BLOCK : 0;
    if (!RECORDS && B.n_nodes && rows_per_block < (1ULL << 32)) {
        // Filtered input (FilterExecutor::select then take, EXP/filter/filter_executor.rs:73-128):
        // every lane evaluates the predicate on its row, the selected rows are queued in LDS (wave
        // ballot + one LDS add per wave), and the hash / probe / state update runs on BLOCK queued
        // rows at a time with every lane busy — at 13% selectivity (ClickBench Q13) the
        // row-per-lane loop would run the long dependent chain of a string key with 1 lane in 8.
        // PU rounds of BLOCK rows are evaluated per step with all their loads issued together (one
        // row per lane per round, a single round in flight left the stream latency-bound: C5's
        // predicate pass ran at ~1.2 TB/s), queued together, and inserted BLOCK at a time.
        // `s <op> ''` on one non-null String column (ClickBench Q13: SearchPhrase <> ''): the
        // selection is a function of the row's length alone, read from the offsets; PU rounds of
        // BLOCK rows are evaluated per step with all their offset loads issued together (one row
        // per lane per round left C5's predicate pass latency-bound, ~1.2 TB/s)
        constexpr int PU = 4;
        static_assert(FLUSH_ROUND % PU == 0, "flush checks fall on step boundaries");
        __shared__ u32 selq[2 * BLOCK];
        __shared__ u32 qn;
        if (threadIdx.x == 0) qn = 0;
        __syncthreads();
        const u32 lane = __lane_id();
        const DNode& n0 = B.nodes[0];
        const DCol& c0 = B.fcols[n0.col];
        // its (PU + 1)-round queue lives in dynamic LDS after the table (lenq entries, host-sized
        // only for such a predicate: the other predicates keep the static 2-round queue and the
        // occupancy it allows — C1: 6 workgroups per CU, all 1464 resident at once)
        const bool lenpred = lenq >= (PU + 1) * BLOCK && B.n_nodes == 1 && n0.op == DBG_PRED_CMP_CONST && n0.str_len == 0 &&
                             c0.type == DBG_STRING && !c0.nullable && c0.layout == LAYOUT_ARROW;
        // the queue in use: the static one, or the multi-round one after the table (lenpred)
        u32* qbuf = lenpred ? (u32*)(lds + (u64)lds_slots * sw + 2) : selq;
        if (lenpred) {
            u32* selq = qbuf;
            const u64* __restrict__ offs = c0.offsets;
            for (u64 it = 0; it < n_iter; it += PU) {
                if (it && (it % FLUSH_ROUND) == 0) maybe_flush<INLINE, RECORDS>(S, batches, B, lds, lds_slots, sw, lcount, llimit, t, my_claims);
                u64 a[PU], b[PU];
#pragma unroll
                for (int k = 0; k < PU; ++k) {
                    const u64 i = r0 + (it + k) * BLOCK + threadIdx.x;
                    const u64 j = i < r1 ? i : r0;
                    a[k] = gld<u64>(offs + j);
                    b[k] = gld<u64>(offs + j + 1);
                }
                bool sel[PU];
                u32 cnt = 0;
                u64 mk[PU];
#pragma unroll
                for (int k = 0; k < PU; ++k) {
                    const u64 i = r0 + (it + k) * BLOCK + threadIdx.x;
                    sel[k] = i < r1 && apply_cmp(n0.cmp, b[k] != a[k] ? 1 : 0);
                    mk[k] = __ballot(sel[k]);
                    cnt += (u32)__popcll(mk[k]);
                }
                if (cnt) {  // queue the step's selected rows: one LDS add per wave
                    u32 wbase = 0;
                    if (lane == 0) wbase = atomicAdd(&qn, cnt);
                    wbase = __shfl(wbase, 0);
                    const u64 lt = (1ULL << lane) - 1;
#pragma unroll
                    for (int k = 0; k < PU; ++k) {
                        if (sel[k]) selq[wbase + (u32)__popcll(mk[k] & lt)] = (u32)((it + k) * BLOCK + threadIdx.x);
                        wbase += (u32)__popcll(mk[k]);
                    }
                }
                __syncthreads();
                const u32 n = qn;  // < (PU + 1) * BLOCK
                if (n >= BLOCK) {
                    const u32 full = n / BLOCK;
                    for (u32 c = 0; c < full; ++c) insert_row(r0 + selq[c * BLOCK + threadIdx.x], my_claims);
                    const u32 rem = n - full * BLOCK;  // < BLOCK: moved to the front
                    const u32 mv = threadIdx.x < rem ? selq[full * BLOCK + threadIdx.x] : 0u;
                    __syncthreads();
                    if (threadIdx.x < rem) selq[threadIdx.x] = mv;
                    if (threadIdx.x == 0) qn = rem;
                }
                __syncthreads();  // the queue is settled before the next step appends
            }
        } else {
            for (u64 it = 0; it < n_iter; ++it) {
                if (it && (it % FLUSH_ROUND) == 0) maybe_flush<INLINE, RECORDS>(S, batches, B, lds, lds_slots, sw, lcount, llimit, t, my_claims);
                const u64 i = r0 + it * BLOCK + threadIdx.x;
                const bool sel = i < r1 && eval_pred(B.nodes, B.n_nodes, B.fcols, i);
                const u64 m = __ballot(sel);
                if (m) {
                    u32 wbase = 0;
                    if (lane == 0) wbase = atomicAdd(&qn, (u32)__popcll(m));
                    wbase = __shfl(wbase, 0);
                    if (sel) selq[wbase + (u32)__popcll(m & ((1ULL << lane) - 1))] = (u32)(i - r0);
                }
                __syncthreads();
                const u32 n = qn;  // < 2 * BLOCK
                if (n >= BLOCK) {
                    const u32 off = selq[threadIdx.x];
                    const u32 rem = n - BLOCK;  // < BLOCK
                    const u32 mv = threadIdx.x < rem ? selq[BLOCK + threadIdx.x] : 0u;
                    __syncthreads();
                    if (threadIdx.x < rem) selq[threadIdx.x] = mv;
                    if (threadIdx.x == 0) qn = rem;
                    insert_row(r0 + off, my_claims);
                }
                __syncthreads();  // the queue is settled before the next round appends
            }
        }
        const u32 n = qn;  // < BLOCK
        if (threadIdx.x < n)
            insert_row(r0 + qbuf[threadIdx.x], my_claims);
    } else {
        for (u64 it = 0; it < n_iter; ++it) {
            if (it && (it % FLUSH_ROUND) == 0) maybe_flush<INLINE, RECORDS>(S, batches, B, lds, lds_slots, sw, lcount, llimit, t, my_claims);
            const u64 i = r0 + it * BLOCK + threadIdx.x;
            if (i >= r1) continue;
            if (!RECORDS && B.n_nodes && !eval_pred(B.nodes, B.n_nodes, B.fcols, i)) continue;
            if (RECORDS && B.seg_records) {  // fixed-capacity segments: record 0 is [count][flags]
                const u64 q = i % B.seg_records;
                const u8* hdr = B.rec_base + (i - q) * (u64)B.rec_width;
                if (q == 0) {
                    if (gld<u64>(hdr + 8)) atomicOr((unsigned long long*)(t.counters + CNT_ERR), (unsigned long long)ERR_FIXED_INCOMPLETE);
                    continue;
                }
                if (q > gld<u64>(hdr)) continue;
            }
            insert_row(i, my_claims);
        }
    }
    __syncthreads();
    block_flush<INLINE, RECORDS>(S, batches, B, lds, lds_slots, sw, lcount, BLOCK, t, my_claims);
}

// ------------------------------------------------------------------------------------------
// agg_insert_str1: one non-null Arrow String key (ClickBench Q13: SearchPhrase), filtered by
// `key <op> ''` or not at all, into a table whose slots cache the key (Spec::kc_word).
//
// The generic kernel compares every probe against the representative row in global memory: an
// LDS hit reads that row's offsets and bytes, an LDS miss reads the HBM slot, then the row's
// offsets and bytes — three dependent random reads before the atomic (C5: 6x the algorithmic
// bytes).  Here the key's first 32 bytes and a header (hash bits 16..63, length, ready bit) sit
// beside the entry in LDS and HBM slots alike, so a probe decides inside the slot: an LDS hit
// touches no global memory, an HBM miss reads its slot's line and adds.  The stream reads two
// offsets per lane per 16-B load, keeps the selected rows' (byte offset, row, length) in an LDS
// queue and inserts them 256 at a time with every lane busy.
//
// Exactness: a different header means a different key (hash or length differ).  An equal header
// with equal cached bytes and a length <= 32 is the same key.  Anything else — a header not yet
// published (a claim in flight on this or another XCD, whose L2s are not coherent), equal headers
// with different bytes, a key longer than 32 bytes — compares against the representative row
// (ref_equal), as the generic kernel always does.  A claimer writes the key words with sc1 stores,
// drains them, then publishes the header sc1 (MI355X_MICROARCH.md, inter-workgroup visibility);
// readers load the slot with sc1 loads.  In LDS a slot whose header is not yet published is
// passed over (the row goes to HBM; the flush merges both states), so no lane ever waits.
// ------------------------------------------------------------------------------------------
typedef volatile __attribute__((address_space(3))) u64 vlds_u64;
typedef volatile __attribute__((address_space(3))) u32 vlds_u32;
// STR1_NT threads per workgroup, STR1_ROUNDS rounds of 2 x STR1_NT rows per stream step
#ifndef STR1_NT
#define STR1_NT 512
#endif
#ifndef STR1_ROUNDS
#define STR1_ROUNDS 2
#endif
#define STR1_QCAP ((2 * STR1_ROUNDS + 1) * STR1_NT)
#define STR1_LDS_BUDGET (56 * 1024)  // the key-caching LDS table (1024 slots for COUNT)

struct KcKey {
    u64 k[KC_KEY_WORDS];  // first 32 bytes, little-endian, zero-padded
    u64 h;                // group hash (hash_bytes)
    u64 hdr;              // (h & ~0xFFFF) | (len & 0x7FFF) << 1 | 1
    u32 len;
};

__device__ __forceinline__ void kc_key(const u8* p, u32 len, KcKey& q) {
    q.len = len;
    const u32 n = len < 8 * KC_KEY_WORDS ? len : 8 * KC_KEY_WORDS;
    const uintptr_t a = (uintptr_t)p;
    const u32 sh = (u32)(a & 7);
    const u64* base = (const u64*)(a - sh);
    const u32 nw = n ? (sh + n + 7) >> 3 : 0;  // aligned words covering [p, p + n): <= 5
    u64 w[KC_KEY_WORDS + 1];
#pragma unroll
    for (int j = 0; j <= KC_KEY_WORDS; ++j) w[j] = (u32)j < nw ? gld<u64>(base + j) : 0;
#pragma unroll
    for (int j = 0; j < KC_KEY_WORDS; ++j) {
        u64 v = sh ? (w[j] >> (8 * sh)) | (w[j + 1] << (64 - 8 * sh)) : w[j];
        const int rem = (int)n - 8 * j;
        q.k[j] = rem >= 8 ? v : (rem <= 0 ? 0 : v & ((1ULL << (8 * rem)) - 1));
    }
    if (len <= 8 * KC_KEY_WORDS) {  // hash_bytes over the register words (device.hpp)
        const u64 M = 0xc6a4a7935bd1e995ULL, R = 47;
        u64 h = 0xe17a1465ULL ^ ((u64)len * M);
        const u32 nb = len >> 3, tl = len & 7;
        u64 tail = 0;
#pragma unroll
        for (u32 i = 0; i < KC_KEY_WORDS; ++i) {
            if (i < nb) {
                u64 x = q.k[i] * M;
                x ^= x >> R;
                x *= M;
                h ^= x;
                h *= M;
            }
            if (i == nb) tail = q.k[i];
        }
        if (tl) h ^= __builtin_bswap64(tail) >> (8 * (8 - tl));
        h ^= h >> R;
        h *= M;
        h ^= h >> R;
        q.h = h;
    } else {
        q.h = hash_bytes(p, len);
    }
    q.hdr = (q.h & ~0xFFFFULL) | ((u64)(len < 0x7FFF ? len : 0x7FFF) << 1) | 1;
}

// LDS probe of the key-caching table; -1 = not staged here (use HBM).
__device__ __forceinline__ int lds_find_kc(u64* lds, u32 lmask, u32 lsw, u32 kc, u32* lcount, u32 llimit, u64 key, const KcKey& q) {
    if (q.len > 8 * KC_KEY_WORDS) return -1;
    vlds_u32* lc = (vlds_u32*)lcount;
    u32 s = (u32)(q.h >> 16) & lmask;
    const int cap = *lc >= llimit ? 2 : LDS_PROBE_CAP;
    for (int p = 0; p < cap; ++p) {
        vlds_u64* e = (vlds_u64*)(lds + (u64)s * lsw);
        u64 ev = e[0];
        if (ev == SLOT_EMPTY) {
            if (*lc >= llimit) return -1;
            u64 old = at_cas<AS_LDS>(asp<AS_LDS>(lds + (u64)s * lsw), SLOT_EMPTY, key);
            if (old == SLOT_EMPTY) {
                __hip_atomic_fetch_add((__attribute__((address_space(3))) u32*)lcount, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
#pragma unroll
                for (int j = 0; j < KC_KEY_WORDS; ++j) e[kc + 1 + j] = q.k[j];
                e[kc] = q.hdr;  // volatile LDS accesses stay in order: the words are visible first
                return (int)s;
            }
            ev = old;
        }
        if ((ev >> 48) == (key >> 48)) {
            const u64 hv = e[kc];
            if (!(hv & 1)) return -1;  // a claim in flight: not waited for
            if (hv == q.hdr) {
                bool eq = true;
#pragma unroll
                for (int j = 0; j < KC_KEY_WORDS; ++j) eq &= e[kc + 1 + j] == q.k[j];
                if (eq) return (int)s;
            }
        }
        s = (s + 1) & lmask;
    }
    return -1;
}

// HBM probe with the slot's key cache; exact (see above).  ~0 = probe limit reached.  The slot's
// entry and its cache words are loaded together (16-B loads of one 64-B slot); a stale copy (this
// CU's L1 or this XCD's L2 holding the line from before a claim) can only show EMPTY — the CAS
// then returns the real entry — or an unpublished header, which takes the representative row.
__device__ __forceinline__ u64 g_find_kc(const Spec& S, const BatchDesc* batches, const DCol* keys, u64 i, u64 key, const KcKey& q,
                                         const TableDesc& t, u32 probe_limit, bool& claimed) {
    claimed = false;
    const u32 kc = (u32)S.kc_word, kp = kc >> 1;
    const bool odd = kc & 1;
    const u64 mask = t.cap - 1;
    u64 s = (q.h >> 16) & mask;
    for (u32 p = 0; p < probe_limit; ++p) {
        u64* slot = t.slots + s * t.stride_words;
        const v2u64 __attribute__((address_space(1)))* sp = (const v2u64 __attribute__((address_space(1)))*)slot;
        const v2u64 p0 = sp[0], pa = sp[kp], pb = sp[kp + 1], pc = sp[kp + 2];
        u64 ev = p0[0];
        u64 hv = odd ? pa[1] : pa[0];
        u64 w[KC_KEY_WORDS] = {odd ? pb[0] : pa[1], odd ? pb[1] : pb[0], odd ? pc[0] : pb[1], odd ? pc[1] : pc[0]};
        if (ev == SLOT_EMPTY) {
            u64 old = at_cas<AS_GLB>(asp<AS_GLB>(slot), SLOT_EMPTY, key);
            if (old == SLOT_EMPTY) {
                claimed = true;
#pragma unroll
                for (int j = 0; j < KC_KEY_WORDS; ++j) st_sc1(slot + kc + 1 + j, q.k[j]);
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                st_sc1(slot + kc, q.hdr);
                return s;
            }
            ev = old;
            hv = ld_sc1(slot + kc);  // the line was read before the claim: the cache again
#pragma unroll
            for (int j = 0; j < KC_KEY_WORDS; ++j) w[j] = ld_sc1(slot + kc + 1 + j);
        }
        if ((ev >> 48) == (key >> 48)) {
            if ((hv & 1) && hv != q.hdr) {  // published and different: another key
                s = (s + 1) & mask;
                continue;
            }
            bool eq = (hv & 1) && q.len <= 8 * KC_KEY_WORDS;
#pragma unroll
            for (int j = 0; j < KC_KEY_WORDS; ++j) eq = eq && w[j] == q.k[j];
            if (eq || ref_equal(S, batches, keys, i, ev)) return s;
        }
        s = (s + 1) & mask;
    }
    return ~0ULL;
}

// The key-caching LDS table into HBM (end of block, and whenever it fills: maybe_flush's rule).
__device__ __forceinline__ void flush_kc(const Spec& S, const BatchDesc* batches, const BatchDesc& B, u64* lds, u32 lds_slots, u32 lsw,
                                         u32 kc, const TableDesc& t, u32& my_claims) {
    for (u32 s = threadIdx.x; s < lds_slots; s += STR1_NT) {
        u64* p = lds + (u64)s * lsw;
        const u64 e = p[0];
        if (e == SLOT_EMPTY) continue;
        KcKey q;
        const u64 hv = p[kc];
        const u64 i = ref_row(e);
        u64 gs;
        bool claimed;
        if (hv & 1) {  // every claim has published its header before the flush's barrier
            q.hdr = hv;
            q.len = (u32)((hv >> 1) & 0x7FFF);
            for (int j = 0; j < KC_KEY_WORDS; ++j) q.k[j] = p[kc + 1 + j];
            // the slot index uses hash bits 16..: the header holds them; the salt is in the entry
            q.h = (hv & ~0xFFFFULL);
            gs = g_find_kc(S, batches, B.keys, i, e, q, t, t.probe_limit, claimed);
        } else {
            gs = g_find<false>(S, batches, B.keys, i, e, group_hash(B.keys, S.n_keys, i), t, t.probe_limit, claimed);
        }
        if (gs == ~0ULL) {
            push_ovf_rec<false, AS_LDS>(S, t, e, p);
            continue;
        }
        my_claims += claimed ? 1 : 0;
        apply_state<AS_GLB, false, AS_LDS>(S, asp<AS_GLB>(t.slots + gs * t.stride_words), p);
    }
}

__device__ __forceinline__ void lds_init_kc(const Spec& S, u64* lds, u32 lds_slots, u32 lsw) {
    for (u32 s = threadIdx.x; s < lds_slots; s += STR1_NT) {
        u64* p = lds + (u64)s * lsw;
        p[0] = SLOT_EMPTY;
        for (u32 w = 1; w < lsw; ++w) p[w] = w < (u32)S.kc_word ? S.slot_init[w] : 0;
    }
}

template <bool PRED>
__global__ void __launch_bounds__(STR1_NT) agg_insert_str1_kernel(const Spec* __restrict__ spec, const BatchDesc* __restrict__ batches,
                                                               u32 bid, u64 rows, u64 rows_per_block, TableDesc t, u32 lds_slots,
                                                               u32 fper, u32 xmode) {
    extern __shared__ __attribute__((aligned(16))) u64 lds[];
    const Spec& S = *spec;
    const BatchDesc& B = batches[bid];
    const u32 kc = (u32)S.kc_word, lsw = kc + 1 + KC_KEY_WORDS;
    // [0] LDS claims, [1] HBM claims, [2] queue length, [3] flush flag, [4] LDS hits, [5] misses
    u32* lcount = (u32*)(lds + (u64)lds_slots * lsw);
    u32* qoff = lcount + 8;       // queue: key byte offset - offs[r0]
    u32* qrl = qoff + STR1_QCAP;  // (row - r0) << 6 | min(len, 63)
    const u32 lmask = lds_slots - 1, llimit = lds_slots - lds_slots / 4;
    lds_init_kc(S, lds, lds_slots, lsw);
    if (threadIdx.x < 8) lcount[threadIdx.x] = 0;
    __syncthreads();
    const DCol& kcol = B.keys[0];
    const u64* __restrict__ offs = kcol.offsets;
    const u8* __restrict__ data = kcol.data;
    const int pcmp = PRED ? B.nodes[0].cmp : 0;
    const u64 r0 = (u64)blockIdx.x * rows_per_block;
    const u64 r1 = r0 + rows_per_block < rows ? r0 + rows_per_block : rows;
    const u32 lane = __lane_id();
    const u64 lt = (1ULL << lane) - 1;
    const u64 off0 = r0 < rows ? gld<u64>(offs + r0) : 0;
    u32 my_claims = 0;

    auto insert = [&](u32 offr, u32 rl) {
        const u64 i = r0 + (rl >> 6);
        u64 off = off0 + offr;
        u32 len = rl & 63;
        if (len == 63 || offr == ~0u) {  // long key or far offset: read the row's offsets again
            off = gld<u64>(offs + i);
            len = (u32)(gld<u64>(offs + i + 1) - off);
        }
        // timing ablations (EXP=1 builds only, DBG_X_STR1): 1 stream + queue only, 2 + key loads
        // and hash, 4 misses dropped, 8 no LDS table
        if (kExperiments && (xmode & 1)) {
            if (off == ~0ULL) atomicAdd(&lcount[1], 1u);
            return;
        }
        KcKey q;
        kc_key(data + off, len, q);
        if (kExperiments && (xmode & 2)) {
            if (q.h == 0x1234567ULL) atomicAdd(&lcount[1], 1u);
            return;
        }
        const u64 key = (q.h & 0xFFFF000000000000ULL) | ((u64)bid << 32) | i;
        const int ls = (kExperiments && (xmode & 8)) ? -1 : lds_find_kc(lds, lmask, lsw, kc, lcount, llimit, key, q);
        const u64 hm = __ballot(ls >= 0), mm = __ballot(ls < 0);
        if (lane == 0) {  // the flush rule's hit rate: one LDS add per wave
            atomicAdd(&lcount[4], (u32)__popcll(hm));
            atomicAdd(&lcount[5], (u32)__popcll(mm));
        }
        if (ls >= 0) {
            apply_row<AS_LDS>(S, asp<AS_LDS>(lds + (u64)ls * lsw), B, i);
            return;
        }
        if (kExperiments && (xmode & 4)) return;
        bool claimed;
        const u64 gs = g_find_kc(S, batches, B.keys, i, key, q, t, t.probe_limit, claimed);
        if (gs == ~0ULL) {
            push_ovf_row(t, bid, i);
            return;
        }
        my_claims += claimed ? 1 : 0;
        apply_row<AS_GLB>(S, asp<AS_GLB>(t.slots + gs * t.stride_words), B, i);
    };

    // A full LDS table is flushed to HBM and started over only while it serves few rows (hit rate
    // below 1/4 since the last check): with Zipf keys (ClickBench Q13) the first keys a workgroup
    // meets are the hot ones and flushing them every few rounds cost more than it saved (C5 insert
    // 15.3 -> 13.0 ms without periodic flushes), while clustered input (a key's rows together)
    // would otherwise send a hot key's rows to one HBM slot for good.
    auto maybe_flush_kc = [&]() {
        if (threadIdx.x == 0) {
            lcount[3] = lcount[0] >= llimit && 3 * lcount[4] < lcount[5] && ld_sc1(t.counters + CNT_OVF_ROWS) == 0 &&
                        ld_sc1(t.counters + CNT_OVF_RECS) == 0;
            lcount[4] = lcount[5] = 0;
        }
        __syncthreads();
        const bool now = lcount[3];
        __syncthreads();
        if (now) {
            flush_kc(S, batches, B, lds, lds_slots, lsw, kc, t, my_claims);
            __syncthreads();
            lds_init_kc(S, lds, lds_slots, lsw);
            if (threadIdx.x == 0) lcount[0] = 0;
            __syncthreads();
        }
    };

    // the stream: two rows per lane per round, offs[i], offs[i + 1] in one 16-B load (i even,
    // offsets 16-B aligned: host-checked), offs[i + 2] from the next lane — or loaded, by the
    // wave's last lane and wherever the next lane's pair runs past the batch's last offset.  The
    // next step's loads are issued before this step's rows are queued and inserted.
    constexpr u64 STEP = (u64)STR1_ROUNDS * 2 * STR1_NT;
    u64 nv[STR1_ROUNDS][3];
    auto load_step = [&](u64 base) {
#pragma unroll
        for (int k = 0; k < STR1_ROUNDS; ++k) {
            const u64 i = base + (u64)k * 2 * STR1_NT + 2 * threadIdx.x;
            const u64 j = i + 1 <= rows ? i : 0;
            const v2u64 v = *(const v2u64 __attribute__((address_space(1)))*)(offs + j);
            nv[k][0] = v[0];
            nv[k][1] = v[1];
            nv[k][2] = ((lane == 63 || i + 3 > rows) && i + 2 <= rows) ? gld<u64>(offs + i + 2) : 0;
        }
    };
    if (r0 < r1) load_step(r0);
    u32 step = 0;
    for (u64 base = r0; base < r1; base += STEP, ++step) {
        if (fper && step && (step % fper) == 0) maybe_flush_kc();
        u64 a[STR1_ROUNDS][3];
#pragma unroll
        for (int k = 0; k < STR1_ROUNDS; ++k)
            for (int r = 0; r < 3; ++r) a[k][r] = nv[k][r];
        if (base + STEP < r1) load_step(base + STEP);
        u64 mk[STR1_ROUNDS][2];
        u32 cnt = 0;
#pragma unroll
        for (int k = 0; k < STR1_ROUNDS; ++k) {
            const u64 i = base + (u64)k * 2 * STR1_NT + 2 * threadIdx.x;
            const u64 nx = __shfl_down(a[k][0], 1);
            if (lane != 63 && i + 3 <= rows) a[k][2] = nx;
#pragma unroll
            for (int r = 0; r < 2; ++r) {
                const u64 len = a[k][r + 1] - a[k][r];
                bool sel = i + r < r1;
                if (PRED) sel = sel && apply_cmp(pcmp, len != 0 ? 1 : 0);
                mk[k][r] = __ballot(sel);
                cnt += (u32)__popcll(mk[k][r]);
            }
        }
        if (cnt) {  // queue the step's selected rows: one LDS add per wave
            u32 wb = 0;
            if (lane == 0) wb = atomicAdd(&lcount[2], cnt);
            wb = __shfl(wb, 0);
#pragma unroll
            for (int k = 0; k < STR1_ROUNDS; ++k) {
                const u64 i = base + (u64)k * 2 * STR1_NT + 2 * threadIdx.x;
#pragma unroll
                for (int r = 0; r < 2; ++r) {
                    if ((mk[k][r] >> lane) & 1) {
                        const u32 q = wb + (u32)__popcll(mk[k][r] & lt);
                        const u64 d = a[k][r] - off0, len = a[k][r + 1] - a[k][r];
                        qoff[q] = d < 0xFFFFFFFFULL ? (u32)d : ~0u;
                        qrl[q] = (u32)(i + r - r0) << 6 | (u32)(len < 63 ? len : 63);
                    }
                    wb += (u32)__popcll(mk[k][r]);
                }
            }
        }
        __syncthreads();
        const u32 n = lcount[2];  // < STR1_QCAP
        if (n >= STR1_NT) {
            const u32 full = n / STR1_NT;
            for (u32 c = 0; c < full; ++c) insert(qoff[c * STR1_NT + threadIdx.x], qrl[c * STR1_NT + threadIdx.x]);
            const u32 rem = n - full * STR1_NT;  // < STR1_NT: moved to the front
            u32 mo = 0, mr = 0;
            if (threadIdx.x < rem) {
                mo = qoff[full * STR1_NT + threadIdx.x];
                mr = qrl[full * STR1_NT + threadIdx.x];
            }
            __syncthreads();
            if (threadIdx.x < rem) {
                qoff[threadIdx.x] = mo;
                qrl[threadIdx.x] = mr;
            }
            if (threadIdx.x == 0) lcount[2] = rem;
        }
        __syncthreads();  // the queue is settled before the next step appends
    }
    const u32 n = lcount[2];  // < STR1_NT
    if (threadIdx.x < n) insert(qoff[threadIdx.x], qrl[threadIdx.x]);
    __syncthreads();
    flush_kc(S, batches, B, lds, lds_slots, lsw, kc, t, my_claims);
    if (my_claims) atomicAdd(&lcount[1], my_claims);
    __syncthreads();
    if (threadIdx.x == 0 && lcount[1]) atomicAdd((unsigned long long*)(t.counters + CNT_CLAIMS), (unsigned long long)lcount[1]);
}

// ------------------------------------------------------------------------------------------
// agg_insert_short: the generic insert specialised for short String keys and COUNT / SUM / AVG over
// non-nullable arguments (TPC-H Q1: GROUP BY l_returnflag, l_linestatus — 1-byte strings — with
// seven Decimal128 SUM / AVG).  The generic kernel's chain per queued row is: predicate -> LDS
// queue -> key offsets -> key bytes -> hash -> LDS probe -> the representative row's offsets ->
// its bytes -> the arguments -> LDS atomics, seven dependent global round trips.  Here the rows
// stay on their lanes (no queue): a row's key offsets and argument values are loaded together,
// then its key bytes with the predicate's column (fetching a row ahead, SHORT_PIPE=1, costs two
// waves per SIMD of occupancy and measured slower: C1 insert 0.26 -> 0.32 ms).  Each key of <= 7 bytes is packed with its length into
// one word, and the LDS probe compares the packed words against a side array beside the table —
// the representative row is read only by the lane that claims a slot (for the group hash the HBM
// entry needs).
//
// Decimal SUM / AVG arguments of precision p with rows_per_block * 10^p < 2^63 (`narrow`, bit per
// aggregate) accumulate in the low state word alone, as a signed 64-bit partial (no carry, so a
// non-returning LDS add instead of add128's returning add + dependent high add); before the flush
// the high word is set to the partial's sign.  Slots are therefore either "short" (claimed here,
// packed keys in the side array, narrow representation) or "generic" (claimed by the fallback
// for longer keys or a full probe, marked PK_GEN, standard representation); each path matches only
// its own slots, so the two never mix (a key may hold a slot of each: the flush merges them).
// The end-of-block flush is the generic one.
// ------------------------------------------------------------------------------------------
#define SHORT_MAXA 8
#define SHORT_MAX_SLOTS 65536  // HBM table slots up to which the short-key insert is taken
#ifndef SHORT_PIPE
#define SHORT_PIPE 0
#endif
#define PK_NONE (~0ULL)
#define PK_GEN (~0ULL - 1)
typedef __attribute__((address_space(3))) u64 lds_u64;
typedef volatile __attribute__((address_space(3))) u64 vlds_u64;
typedef volatile __attribute__((address_space(3))) u32 vlds_u32;
struct ShortRow {
    u64 o[4];               // key offsets [k0 begin, k0 end, k1 begin, k1 end]
    u64 lo[SHORT_MAXA];     // argument low words (or the whole value)
    u64 hi[SHORT_MAXA];     // Decimal128 high words of wide sums
};
// End of the short-key insert: a merge tree over parked tables, fan-in SHORT_FANIN per level.
// block_flush parks each workgroup's table and lets the last of every FLUSH_GROUP merge them and
// flush to HBM, so G / FLUSH_GROUP leaders still add into the same few HBM slots, serialised at
// the memory side (C1: 366 leaders x 4 groups).  Here a level's leader parks its merged table
// again, one level up, until one root flushes: the HBM table sees one add per group.  Parked rows
// carry the slot's packed keys (words n_words+1, n_words+2), so a merge compares them in LDS and
// never reads a representative row.  Node n of level L parks in the scratch row of workgroup
// n * FANIN^L (read by its own leader before), its tickets sit at a per-level offset.  Hand-off
// as in block_flush: sc1 stores, vmcnt drain + barrier before the ticket add, acquire + sc1 loads.
// A table with a generic slot or more than SCR_ENTRIES short slots flushes directly and parks an
// empty row.
#ifndef SHORT_FANIN_LOG
#define SHORT_FANIN_LOG 2  // 4 parked tables per leader (16: 3 levels instead of 6 for C1, the same 0.274 ms step)
#endif
#define SHORT_FANIN (1u << SHORT_FANIN_LOG)
__device__ __forceinline__ void short_tree_flush(const Spec& S, const BatchDesc* batches, const BatchDesc& B, u64* lds, u32 lds_slots,
                                                 u32 sw, u32* lcount, u64* pk0, u64* pk1, const TableDesc& t, u32 my_claims) {
    const u32 lmask = lds_slots - 1;
    const u32 llimit = lds_slots - lds_slots / 4;
    const u32 nw = (u32)S.n_words;
    u64* counts = t.scratch;
    u64* tickets = t.scratch + t.scr_blocks;
    u64* rows = t.scratch + 2 * (u64)t.scr_blocks;
    u32 node = blockIdx.x, n_nodes = gridDim.x, shift = 0, toff = 0;
    for (;;) {
        // the table in LDS: count slots; [4] generic slots, [5] short slots
        if (threadIdx.x == 0) lcount[4] = lcount[5] = 0;
        __syncthreads();
        for (u32 s = threadIdx.x; s < lds_slots; s += BLOCK) {
            const u64 e = lds[(u64)s * sw];
            if (e == SLOT_EMPTY) continue;
            atomicAdd(&lcount[pk0[s] == PK_GEN || pk0[s] == PK_NONE ? 4 : 5], 1u);
        }
        __syncthreads();
        const bool root = n_nodes == 1;
        const bool direct = root || lcount[4] != 0 || lcount[5] > SCR_ENTRIES;
        const u64 b = (u64)node << shift;  // this node's scratch row
        if (direct) {
            flush_lds_direct<false, false>(S, batches, B, lds, lds_slots, sw, BLOCK, t, my_claims);
            if (!root && threadIdx.x == 0) st_sc1(counts + b, 0);
        } else {
            if (threadIdx.x == 0) lcount[2] = 0;
            __syncthreads();
            u64* row = rows + b * SCR_ENTRIES * sw;
            for (u32 s = threadIdx.x; s < lds_slots; s += BLOCK) {
                const u64* p = lds + (u64)s * sw;
                if (p[0] == SLOT_EMPTY) continue;
                const u32 k = atomicAdd(&lcount[2], 1u);
                u64* d = row + (u64)k * sw;
                for (u32 w = 0; w <= nw; ++w) st_sc1(d + w, p[w]);
                st_sc1(d + nw + 1, pk0[s]);
                st_sc1(d + nw + 2, pk1[s]);
            }
            __syncthreads();
            if (threadIdx.x == 0) st_sc1(counts + b, lcount[2]);
        }
        if (root) break;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        const u32 g = node / SHORT_FANIN;
        const u32 gsize = min((u32)SHORT_FANIN, n_nodes - g * SHORT_FANIN);
        if (threadIdx.x == 0) {
            const u64 tk = atomicAdd((unsigned long long*)(tickets + toff + g), 1ULL);
            lcount[3] = tk == (u64)gsize - 1 ? 1u : 0u;
        }
        __syncthreads();
        if (!lcount[3]) break;
        // this workgroup leads node g one level up: merge the members' parked rows
        if (threadIdx.x == 0) {
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            tickets[toff + g] = 0;  // ready for the next launch (all members have added)
        }
        lds_table_init(S, lds, lds_slots, sw, BLOCK);
        for (u32 j = threadIdx.x; j < lds_slots; j += BLOCK) pk0[j] = pk1[j] = PK_NONE;
        if (threadIdx.x == 0) lcount[0] = 0;
        __syncthreads();
        for (u32 f = threadIdx.x; f < gsize * SCR_ENTRIES; f += BLOCK) {
            const u64 mb = ((u64)g * SHORT_FANIN + f / SCR_ENTRIES) << shift, k = f % SCR_ENTRIES;
            const u64* r = rows + (mb * SCR_ENTRIES + k) * sw;
            const u64 cnt = ld_sc1(counts + mb);
            const u64 e = ld_sc1(r);
            if (k >= cnt) continue;
            const u64 q0 = ld_sc1(r + nw + 1), q1 = ld_sc1(r + nw + 2);
            u32 pos = (u32)slot_mix(q0 ^ slot_mix(q1)) & lmask;
            int ls = -1;
            for (int p = 0; p < LDS_PROBE_CAP; ++p) {
                wptr<AS_LDS> ep = asp<AS_LDS>(lds + (u64)pos * sw);
                u64 ev = vld<AS_LDS>(ep);
                if (ev == SLOT_EMPTY) {
                    if (*(vlds_u32*)lcount >= llimit) break;
                    const u64 old = at_cas<AS_LDS>(ep, SLOT_EMPTY, e);
                    if (old == SLOT_EMPTY) {
                        ((vlds_u64*)pk0)[pos] = q0;
                        ((vlds_u64*)pk1)[pos] = q1;
                        __hip_atomic_fetch_add((__attribute__((address_space(3))) u32*)lcount, 1u, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_WORKGROUP);
                        ls = (int)pos;
                        break;
                    }
                }
                if (((vlds_u64*)pk0)[pos] == q0 && ((vlds_u64*)pk1)[pos] == q1) {
                    ls = (int)pos;
                    break;
                }
                pos = (pos + 1) & lmask;
            }
            if (ls >= 0) {
                apply_state<AS_LDS, true>(S, asp<AS_LDS>(lds + (u64)ls * sw), r);
                continue;
            }
            // the merge table is full: this row goes to HBM by itself
            bool claimed;
            const u64 h = group_hash(B.keys, S.n_keys, ref_row(e));
            const u64 gs = g_find<false>(S, batches, B.keys, ref_row(e), e, h, t, t.probe_limit, claimed);
            if (gs == ~0ULL) {
                push_ovf_rec<true>(S, t, e, r);
                continue;
            }
            my_claims += claimed ? 1 : 0;
            apply_state<AS_GLB, true>(S, asp<AS_GLB>(t.slots + gs * t.stride_words), r);
        }
        __syncthreads();
        toff += (n_nodes + SHORT_FANIN - 1) / SHORT_FANIN;
        node = g;
        n_nodes = (n_nodes + SHORT_FANIN - 1) / SHORT_FANIN;
        shift += SHORT_FANIN_LOG;
    }
    if (my_claims) atomicAdd(&lcount[1], my_claims);
    __syncthreads();
    if (threadIdx.x == 0 && lcount[1]) atomicAdd((unsigned long long*)(t.counters + CNT_CLAIMS), (unsigned long long)lcount[1]);
}

__global__ void __launch_bounds__(BLOCK) __attribute__((amdgpu_waves_per_eu(6))) agg_insert_short_kernel(const Spec* __restrict__ spec, const BatchDesc* __restrict__ batches,
                                                                u32 bid, u64 rows, u64 rows_per_block, TableDesc t, u32 lds_slots,
                                                                u32 rep_mask, int xmode, u32 narrow, int tree_ok, u64* trace) {
    extern __shared__ __attribute__((aligned(16))) u64 lds[];
    // EXPERIMENT (TRACE=1 builds, DBG_X_TRACE_SHORT): [0] first workgroup start, [1] / [2] first /
    // last row loop end, [3] last flush start, [4] last workgroup end (s_memrealtime, 100 MHz)
    auto tmark = [&](int k, bool mx) {
        if (kPhaseTrace && trace && threadIdx.x == 0) {
            const unsigned long long v = __builtin_amdgcn_s_memrealtime();
            if (mx) atomicMax((unsigned long long*)trace + k, v);
            else atomicMin((unsigned long long*)trace + k, v);
        }
    };
    tmark(0, false);
    const Spec& S = *spec;
    const BatchDesc& B = batches[bid];
    const u32 sw = S.stride_words;
    u32* lcount = (u32*)(lds + (u64)lds_slots * sw);  // [0] lds claims, [1] hbm claims, [2..5] flush
    u64* pk0 = lds + (u64)lds_slots * sw + 4;          // packed keys of short slots (PK_NONE / PK_GEN)
    u64* pk1 = pk0 + lds_slots;
    const u32 lmask = lds_slots - 1;
    const u32 llimit = lds_slots - lds_slots / 4;
    lds_table_init(S, lds, lds_slots, sw, BLOCK);
    for (u32 j = threadIdx.x; j < lds_slots; j += BLOCK) pk0[j] = pk1[j] = PK_NONE;
    if (threadIdx.x < 8) lcount[threadIdx.x] = 0;
    __syncthreads();
    const u64 r0 = (u64)blockIdx.x * rows_per_block;
    const u64 r1 = r0 + rows_per_block < rows ? r0 + rows_per_block : rows;
    u32 my_claims = 0;
    const int nk = S.n_keys;
    const int na = S.n_aggs;
    vlds_u32* lc = (vlds_u32*)lcount;
    auto fetch = [&](u64 i, ShortRow& r) __attribute__((always_inline)) {
        r.o[0] = gld<u64>(B.keys[0].offsets + i);
        r.o[1] = gld<u64>(B.keys[0].offsets + i + 1);
        r.o[2] = r.o[3] = 0;
        if (nk > 1) {
            r.o[2] = gld<u64>(B.keys[1].offsets + i);
            r.o[3] = gld<u64>(B.keys[1].offsets + i + 1);
        }
#pragma unroll
        for (int a = 0; a < SHORT_MAXA; ++a) {
            r.lo[a] = r.hi[a] = 0;
            if (a < na && S.aggs[a].arg_type >= 0 && S.aggs[a].kind != DBG_AGG_COUNT) {
                r.lo[a] = dcol_bits(B.args[a], i);
                if (S.aggs[a].sumk == SUMK_I128 && !((narrow >> a) & 1)) r.hi[a] = dcol_hi(B.args[a], i);
            }
        }
    };
    // the fallback: a generic slot (PK_GEN) of this workgroup's table, else the HBM table
    auto generic_row = [&](u64 i) __attribute__((always_inline)) {
        const u64 h = group_hash(B.keys, nk, i);
        const u64 key = (h & 0xFFFF000000000000ULL) | ((u64)bid << 32) | i;
        u32 s = (u32)((h >> 16) & lmask);
        const int cap = *lc >= llimit ? 2 : LDS_PROBE_CAP;
        int ls = -1;
        for (int p = 0; p < cap; ++p) {
            wptr<AS_LDS> e = asp<AS_LDS>(lds + (u64)s * sw);
            u64 ev = vld<AS_LDS>(e);
            if (ev == SLOT_EMPTY) {
                if (*lc >= llimit) break;
                const u64 old = at_cas<AS_LDS>(e, SLOT_EMPTY, key);
                if (old == SLOT_EMPTY) {
                    ((vlds_u64*)pk0)[s] = PK_GEN;
                    __hip_atomic_fetch_add((__attribute__((address_space(3))) u32*)lcount, 1u, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_WORKGROUP);
                    ls = (int)s;
                    break;
                }
                ev = old;
            }
            // a slot whose marker is not written yet reads as not generic: at worst a second slot
            if (((vlds_u64*)pk0)[s] == PK_GEN && (ev >> 48) == (key >> 48) && ref_equal(S, batches, B.keys, i, ev)) {
                ls = (int)s;
                break;
            }
            s = (s + 1) & lmask;
        }
        if (ls >= 0) {
            apply_row<AS_LDS>(S, asp<AS_LDS>(lds + (u64)ls * sw), B, i);
            return;
        }
        bool claimed;
        const u64 gs = g_find<false>(S, batches, B.keys, i, key, h, t, t.probe_limit, claimed);
        if (gs == ~0ULL) {
            push_ovf_row(t, bid, i);
            return;
        }
        my_claims += claimed ? 1 : 0;
        apply_row<AS_GLB>(S, asp<AS_GLB>(t.slots + gs * t.stride_words), B, i);
    };
    auto process = [&](u64 i, const ShortRow& r) __attribute__((always_inline)) {
        const u64 l0 = r.o[1] - r.o[0], l1 = r.o[3] - r.o[2];
        const bool shortk = l0 <= 7 && l1 <= 7;
        // key bytes and the predicate's column: issued together, one wait
        u64 b0 = 0, b1 = 0;
        if (shortk && l0) b0 = load_partial(B.keys[0].data + r.o[0], l0);
        if (shortk && l1) b1 = load_partial(B.keys[1].data + r.o[2], l1);
        const bool pass = B.n_nodes == 0 || eval_pred(B.nodes, B.n_nodes, B.fcols, i);
        if (!pass) return;
        // timing ablation (EXP=1 builds only): the loads and the predicate alone (no probe, adds
        // or flush); the key bytes stay live through an improbable compare
        if (kExperiments && xmode == 5 && (b0 ^ b1) != 0x5A5A5A5A5A5A5A5AULL) return;
        if (!shortk) {
            generic_row(i);
            return;
        }
        const u64 k0 = (l0 << 56) | (b0 & width_mask((u32)l0));
        u64 k1 = nk > 1 ? ((l1 << 56) | (b1 & width_mask((u32)l1))) : 0;
        if (rep_mask && *lc < lds_slots / 8)
            k1 |= (u64)((threadIdx.x & rep_mask) + 1) << 59;  // a replica of the key's slot: fewer lanes per LDS address
        u32 pos = (u32)slot_mix(k0 ^ slot_mix(k1)) & lmask;
        int ls = -1;
        for (int p = 0; p < LDS_PROBE_CAP; ++p) {
            wptr<AS_LDS> e = asp<AS_LDS>(lds + (u64)pos * sw);
            u64 ev = vld<AS_LDS>(e);
            if (ev == SLOT_EMPTY) {
                if (*lc >= llimit) break;  // full: the generic path
                const u64 h = group_hash(B.keys, nk, i);
                const u64 key = (h & 0xFFFF000000000000ULL) | ((u64)bid << 32) | i;
                const u64 old = at_cas<AS_LDS>(e, SLOT_EMPTY, key);
                if (old == SLOT_EMPTY) {
                    ((vlds_u64*)pk0)[pos] = k0;
                    ((vlds_u64*)pk1)[pos] = k1;
                    __hip_atomic_fetch_add((__attribute__((address_space(3))) u32*)lcount, 1u, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_WORKGROUP);
                    ls = (int)pos;
                    break;
                }
                ev = old;
            }
            // packed keys not written yet (or a generic slot) do not match: at worst a second slot
            if (((vlds_u64*)pk0)[pos] == k0 && ((vlds_u64*)pk1)[pos] == k1) {
                ls = (int)pos;
                break;
            }
            pos = (pos + 1) & lmask;
        }
        if (ls < 0) {
            generic_row(i);
            return;
        }
        if (kExperiments && (xmode == 2 || xmode == 4)) return;  // timing ablation (EXP=1 builds only)
        wptr<AS_LDS> st = asp<AS_LDS>(lds + (u64)ls * sw);
#pragma unroll
        for (int a = 0; a < SHORT_MAXA; ++a) {
            if (a >= na) break;
            const DAgg& A = S.aggs[a];
            wptr<AS_LDS> w = st + A.w0;
            if (A.kind == DBG_AGG_COUNT) {
                at_add<AS_LDS>(w, 1ULL);
                continue;
            }
            if (A.sumk == SUMK_I64) {
                u64 v = r.lo[a];
                switch (A.arg_type) {
                    case DBG_INT8: v = (u64)(i64)(int8_t)v; break;
                    case DBG_INT16: v = (u64)(i64)(int16_t)v; break;
                    case DBG_INT32: case DBG_DATE: v = (u64)(i64)(int32_t)v; break;
                    default: break;
                }
                at_add<AS_LDS>(w, v);
            } else if (A.sumk == SUMK_F64) {
                at_addf<AS_LDS>(w, A.arg_type == DBG_FLOAT32 ? (double)__uint_as_float((u32)r.lo[a]) : __longlong_as_double((long long)r.lo[a]));
            } else if ((narrow >> a) & 1) {
                at_add<AS_LDS>(w, r.lo[a]);  // signed 64-bit partial, widened before the flush
            } else {
                add128<AS_LDS>(w, r.lo[a], r.hi[a]);
            }
            if (A.kind == DBG_AGG_AVG) at_add<AS_LDS>(w + (A.sumk == SUMK_I128 ? 2 : 1), 1ULL);
        }
    };
    static_assert(SHORT_PIPE == 0 || SHORT_PIPE == 1, "");
    u64 i = r0 + threadIdx.x;
    if (SHORT_PIPE && i < r1) {  // loads one row ahead (measured slower: occupancy 6 -> 4 waves)
        ShortRow cur;
        fetch(i, cur);
        for (; i < r1; i += BLOCK) {
            ShortRow nxt;
            const u64 in = i + BLOCK;
            if (in < r1) fetch(in, nxt);
            process(i, cur);
            cur = nxt;
        }
    } else {
        for (; i < r1; i += BLOCK) {
            ShortRow cur;
            fetch(i, cur);
            process(i, cur);
        }
    }
    __syncthreads();
    tmark(1, false);
    tmark(2, true);
    if (kExperiments && xmode >= 3) return;  // timing ablation (EXP=1 builds only: no flush)
    if (narrow) {  // short slots: narrow partials -> Decimal128 state (high word = sign)
        for (u32 s = threadIdx.x; s < lds_slots; s += BLOCK) {
            const u64 pk = pk0[s];
            if (pk == PK_NONE || pk == PK_GEN) continue;
            u64* st = lds + (u64)s * sw;
            for (int a = 0; a < na; ++a)
                if ((narrow >> a) & 1) st[S.aggs[a].w0 + 1] = (u64)((i64)st[S.aggs[a].w0] >> 63);
        }
        __syncthreads();
    }
    const bool tree = tree_ok && t.scratch != nullptr && gridDim.x > 1 && gridDim.x <= t.scr_blocks;  // uniform
    tmark(3, true);
    if (tree) short_tree_flush(S, batches, B, lds, lds_slots, sw, lcount, pk0, pk1, t, my_claims);
    else block_flush<false, false>(S, batches, B, lds, lds_slots, sw, lcount, BLOCK, t, my_claims);
    tmark(4, true);
}

// host: the short-key specialisation applies (hb = host copy of the batch descriptor)
static bool short_eligible(const Spec& S, const BatchDesc& hb) {
    if (S.inline_keys || S.n_keys < 1 || S.n_keys > 2 || S.n_aggs > SHORT_MAXA || S.flags_word >= 0 || hb.is_records) return false;
    for (int c = 0; c < S.n_keys; ++c)
        if (S.key_types[c].type != DBG_STRING || S.key_types[c].nullable || hb.keys[c].layout != LAYOUT_ARROW) return false;
    for (int a = 0; a < S.n_aggs; ++a) {
        const DAgg& A = S.aggs[a];
        if (A.kind != DBG_AGG_COUNT && A.kind != DBG_AGG_SUM && A.kind != DBG_AGG_AVG) return false;
        if (A.arg_type >= 0 && A.arg_nullable) return false;
    }
    return true;
}

// agg_insert_str1_kernel: one non-null Arrow String key (the Spec's key cache), no predicate or
// `key <op> ''` on that same column, offsets 16-B aligned, row offsets below 2^32 per workgroup.
static bool str1_eligible(const Spec& S, const BatchDesc& hb, u64 rows) {
    if (!S.kc_word || hb.is_records || S.n_keys != 1) return false;
    const DCol& k = hb.keys[0];
    if (k.type != DBG_STRING || k.nullable || k.layout != LAYOUT_ARROW || ((uintptr_t)k.offsets & 15)) return false;
    if (rows >= (1ULL << 32)) return false;  // queue entries hold (row - r0) << 6 in 32 bits: < 2^26 per workgroup
    if (hb.n_nodes == 0) return true;
    if (hb.n_nodes != 1) return false;
    const DNode& n = hb.nodes[0];
    const DCol& c = hb.fcols[n.col];
    return n.op == DBG_PRED_CMP_CONST && n.str_len == 0 && c.type == DBG_STRING && !c.nullable && c.layout == LAYOUT_ARROW &&
           c.offsets == k.offsets && c.data == k.data;
}

static u32 lds_slots_for(const Spec& S, u32 budget = LDS_BUDGET_BYTES) {
    u32 bytes_per = (u32)S.stride_words * 8;
    u32 n = 1;
    while ((n * 2) * bytes_per + 16 <= budget) n *= 2;
    return n;
}

// ------------------------------------------------------------------------------------------
// Deferred overflow: rows (bid,row) and partial records [entry][words] re-inserted after growth.
// ------------------------------------------------------------------------------------------
template <bool INLINE>
__global__ void __launch_bounds__(BLOCK) agg_retry_kernel(const Spec* __restrict__ spec, const BatchDesc* __restrict__ batches,
                                                         TableDesc t, u64 n_rows, u64 n_recs, const u64* rows_list,
                                                         const u64* recs_list) {
    const Spec& S = *spec;
    u64 total = n_rows + n_recs;
    for (u64 k = blockIdx.x * (u64)BLOCK + threadIdx.x; k < total; k += (u64)gridDim.x * BLOCK) {
        bool claimed;
        u64 gs;
        if (k < n_rows) {
            u64 it = rows_list[k];
            u32 bid = (u32)(it >> 32);
            u64 i = (u32)it;
            const BatchDesc& B = batches[bid];
            u64 h, key;
            if (B.is_records) h = gld<u64>(B.rec_base + i * (u64)B.rec_width);
            else h = INLINE ? 0 : group_hash(B.keys, S.n_keys, i);
            key = INLINE ? pack_key(S, B.keys, i) : ((h & 0xFFFF000000000000ULL) | ((u64)bid << 32) | i);
            gs = g_find<INLINE>(S, batches, B.keys, i, key, h, t, (u32)(t.cap < 0xFFFFFFFFull ? t.cap : 0xFFFFFFFFull), claimed);
            if (gs == ~0ULL) {
                atomicOr((unsigned long long*)(t.counters + CNT_ERR), (unsigned long long)ERR_OVF_LOST);
                continue;
            }
            wptr<AS_GLB> st = asp<AS_GLB>(t.slots + gs * t.stride_words);
            if (B.is_records) apply_state<AS_GLB>(S, st, (const u64*)(B.rec_base + i * (u64)B.rec_width + S.rec_state_off) - 1);
            else apply_row<AS_GLB>(S, st, B, i);
        } else {
            const u64* r = recs_list + (k - n_rows) * t.stride_words;
            u64 key = r[0];
            if (INLINE && key == SLOT_EMPTY) continue;  // consumed by part_fixup (never a record key)
            u64 h = 0;
            if (!INLINE) {
                const BatchDesc& B = batches[ref_bid(key)];
                h = B.is_records ? gld<u64>(B.rec_base + (u64)ref_row(key) * B.rec_width) : group_hash(B.keys, S.n_keys, ref_row(key));
            }
            gs = g_find_entry<INLINE>(S, batches, key, h, t, (u32)(t.cap < 0xFFFFFFFFull ? t.cap : 0xFFFFFFFFull), claimed);
            if (gs == ~0ULL) {
                atomicOr((unsigned long long*)(t.counters + CNT_ERR), (unsigned long long)ERR_OVF_LOST);
                continue;
            }
            apply_state<AS_GLB>(S, asp<AS_GLB>(t.slots + gs * t.stride_words), r);
        }
        if (claimed) atomicAdd((unsigned long long*)(t.counters + CNT_CLAIMS), 1ULL);
    }
}

void launch_retry(hipStream_t s, const Spec* dspec, const Spec& S, const BatchDesc* batches, const TableDesc& t, u64 n_rows,
                  u64 n_recs, const u64* rows_list, const u64* recs_list) {
    u64 total = n_rows + n_recs;
    if (!total) return;
    u64 blocks = (total + BLOCK - 1) / BLOCK;
    if (blocks > 4096) blocks = 4096;
    if (S.inline_keys)
        hipLaunchKernelGGL(agg_retry_kernel<true>, dim3((u32)blocks), dim3(BLOCK), 0, s, dspec, batches, t, n_rows, n_recs, rows_list, recs_list);
    else
        hipLaunchKernelGGL(agg_retry_kernel<false>, dim3((u32)blocks), dim3(BLOCK), 0, s, dspec, batches, t, n_rows, n_recs, rows_list, recs_list);
}

// ------------------------------------------------------------------------------------------
// Rehash into a larger table (groups are distinct: claim the first empty slot, copy the words).
// ------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(BLOCK) agg_rehash_kernel(const Spec* __restrict__ spec, const BatchDesc* __restrict__ batches,
                                                          const u64* old_slots, u64 old_cap, TableDesc t) {
    const Spec& S = *spec;
    u64 sw = t.stride_words;
    u64 mask = t.cap - 1;
    for (u64 s = blockIdx.x * (u64)BLOCK + threadIdx.x; s <= old_cap; s += (u64)gridDim.x * BLOCK) {
        const u64* o = old_slots + s * sw;
        u64 e = o[0];
        if (e == SLOT_EMPTY) continue;
        u64 ns;
        if (s == old_cap) {
            ns = t.cap;  // sentinel slot
        } else {
            u64 h = S.inline_keys ? 0 : entry_hash(S, batches, e, false);
            ns = (S.inline_keys ? slot_mix(e) : (h >> 16)) & mask;
            for (;;) {
                u64 old = atomicCAS((unsigned long long*)(t.slots + ns * sw), SLOT_EMPTY, (unsigned long long)e);
                if (old == SLOT_EMPTY) break;
                ns = (ns + 1) & mask;
            }
        }
        u64* d = t.slots + ns * sw;
        if (s == old_cap) d[0] = e;
        for (u64 w = 1; w < sw; ++w) d[w] = o[w];
    }
}

void launch_rehash(hipStream_t s, const Spec* dspec, const Spec& S, const BatchDesc* batches, const u64* old_slots, u64 old_cap,
                   const TableDesc& t) {
    u64 blocks = (old_cap + 1 + BLOCK - 1) / BLOCK;
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL(agg_rehash_kernel, dim3((u32)blocks), dim3(BLOCK), 0, s, dspec, batches, old_slots, old_cap, t);
}

// ------------------------------------------------------------------------------------------
// Finalize / partition: per-block histograms over slot ranges.
// ------------------------------------------------------------------------------------------
u64 finalize_blocks(u64 cap) { return (cap + 1 + SLOTS_PER_BLOCK - 1) / SLOTS_PER_BLOCK; }

// scheme 2: the slot's legacy bucket, computed beforehand by legacy_slot_bucket_kernel
__device__ __forceinline__ u32 part_of(u64 h, u32 n_parts, int scheme, const u32* lpart, u64 s) {
    if (n_parts <= 1) return 0;
    if (scheme == 2) return lpart[s];
    if (scheme == 0) return (u32)(h % n_parts);  // Payload::scatter: hash % n (payload.rs:383)
    u32 rb = 31 - __clz(n_parts);                // radix bits [48 - r, 48) (partitioned_payload.rs:121)
    return (u32)((h >> (48 - rb)) & (n_parts - 1));
}

__device__ __forceinline__ u64 key_str_len(const Spec& S, const BatchDesc* batches, u64 e, int c) {
    StrRef r = dcol_str(batches[ref_bid(e)].keys[c], ref_row(e));
    return r.len;
}
// The same from slot s's key cache when it holds the key (published header, length <= 32): no
// read of the representative row.
__device__ __forceinline__ u64 slot_str_len(const Spec& S, const BatchDesc* batches, const TableDesc& t, u64 s, u64 e, int c) {
    if (S.kc_word && s < t.cap) {
        const u64 hv = t.slots[s * t.stride_words + S.kc_word];
        if ((hv & 1) && ((hv >> 1) & 0x7FFF) <= 8 * KC_KEY_WORDS) return (hv >> 1) & 0x7FFF;
    }
    return key_str_len(S, batches, e, c);
}

#define MAX_PARTS_LDS 256

__global__ void __launch_bounds__(BLOCK) count_groups_kernel(const Spec* __restrict__ spec, const BatchDesc* __restrict__ batches,
                                                            TableDesc t, u32 n_parts, int scheme, const u32* __restrict__ lpart,
                                                            u64* hist, u64* str_hist, u64 nblocks) {
    const Spec& S = *spec;
    __shared__ unsigned long long lh[MAX_PARTS_LDS];
    __shared__ unsigned long long ls[DBG_MAX_KEYS][MAX_PARTS_LDS];
    for (u32 p = threadIdx.x; p < n_parts; p += BLOCK) lh[p] = 0;
    if (S.has_strings && !S.inline_keys)
        for (u32 p = threadIdx.x; p < (u32)S.n_keys * MAX_PARTS_LDS; p += BLOCK) ls[p / MAX_PARTS_LDS][p % MAX_PARTS_LDS] = 0;
    __syncthreads();
    u64 base = (u64)blockIdx.x * SLOTS_PER_BLOCK;
    u32 mine = 0;  // n_parts == 1: count in registers, reduce once (no LDS atomics on one word)
    for (u32 k = threadIdx.x; k < SLOTS_PER_BLOCK; k += BLOCK) {
        u64 s = base + k;
        if (s > t.cap) break;
        u64 e = t.slots[s * t.stride_words];
        if (e == SLOT_EMPTY) continue;
        u32 p = 0;
        if (n_parts > 1) {
            p = part_of(scheme == 2 ? 0 : entry_hash(S, batches, e, s == t.cap), n_parts, scheme, lpart, s);
            atomicAdd(&lh[p], 1ULL);
        } else {
            mine++;
        }
        if (S.has_strings && !S.inline_keys)
            for (int c = 0; c < S.n_keys; ++c)
                if (S.key_types[c].type == DBG_STRING) atomicAdd(&ls[c][p], (unsigned long long)slot_str_len(S, batches, t, s, e, c));
    }
    if (n_parts == 1) {
        for (int off = 32; off > 0; off >>= 1) mine += __shfl_xor(mine, off, 64);
        if ((threadIdx.x & 63) == 0 && mine) atomicAdd(&lh[0], (unsigned long long)mine);
    }
    __syncthreads();
    for (u32 p = threadIdx.x; p < n_parts; p += BLOCK) {
        hist[(u64)p * nblocks + blockIdx.x] = lh[p];
        if (S.has_strings && !S.inline_keys)
            for (int c = 0; c < S.n_keys; ++c)
                if (S.key_types[c].type == DBG_STRING) str_hist[((u64)p * S.n_keys + c) * nblocks + blockIdx.x] = ls[c][p];
    }
}

void launch_count_groups(hipStream_t s, const Spec* dspec, const Spec& S, const BatchDesc* batches, const TableDesc& t, u32 n_parts,
                         int scheme, const u32* lpart, u64* hist, u64* str_hist) {
    u64 nb = finalize_blocks(t.cap);
    hipLaunchKernelGGL(count_groups_kernel, dim3((u32)nb), dim3(BLOCK), 0, s, dspec, batches, t, n_parts, scheme, lpart, hist, str_hist, nb);
}

// Legacy bucket of every occupied slot (enable_experimental_aggregate_hashtable = 0): the
// FastHash of the group's FixedKeys / SingleBinary key (legacy.hpp), hash2bucket<bits, true>.
__global__ void __launch_bounds__(BLOCK) legacy_slot_bucket_kernel(const Spec* __restrict__ spec, const BatchDesc* __restrict__ batches,
                                                                  TableDesc t, LegacyLayout L, u32* __restrict__ out) {
    const Spec& S = *spec;
    __shared__ u32 tab[256];
    crc_table_init(tab);
    for (u64 s = blockIdx.x * (u64)BLOCK + threadIdx.x; s <= t.cap; s += (u64)gridDim.x * BLOCK) {
        const u64 e = t.slots[s * t.stride_words];
        if (e == SLOT_EMPTY) continue;
        u64 h;
        if (L.binary) {
            const StrRef sr = dcol_str(batches[ref_bid(e)].keys[0], ref_row(e));
            h = legacy_bytes_hash(tab, sr.p, sr.len);
        } else if (L.serializer) {
            SerCrc sc;
            const u64 key = s == t.cap ? SLOT_EMPTY : e;
            for (int c = 0; c < S.n_keys; ++c) {
                const dbg_datatype& ty = S.key_types[c];
                bool v;
                u64 lo = 0, hi = 0;
                StrRef sr{nullptr, 0};
                if (S.inline_keys) {
                    v = !ty.nullable || ((key >> (8 * S.voff[c])) & 0xff) != 0;
                    lo = (key >> (8 * S.koff[c])) & width_mask(type_width(ty.type));
                } else {
                    const DCol& kc = batches[ref_bid(e)].keys[c];
                    const u64 row = ref_row(e);
                    v = dcol_valid(kc, row);
                    if (v && ty.type == DBG_STRING) sr = dcol_str(kc, row);
                    else if (v) {
                        lo = dcol_bits(kc, row);
                        if (ty.type == DBG_DECIMAL128) hi = dcol_hi(kc, row);
                    }
                }
                sc.column(tab, ty.type, ty.nullable, v, lo, hi, sr.p, sr.len);
            }
            h = sc.finish(tab);
        } else {
            u64 k[4] = {0, 0, 0, 0};
            const u64 key = s == t.cap ? SLOT_EMPTY : e;
            for (int c = 0; c < S.n_keys; ++c) {
                const dbg_datatype& ty = S.key_types[c];
                const u32 w = type_width(ty.type);
                bool v;
                u64 lo, hi = 0;
                if (S.inline_keys) {
                    v = !ty.nullable || ((key >> (8 * S.voff[c])) & 0xff) != 0;
                    lo = (key >> (8 * S.koff[c])) & width_mask(w);
                } else {
                    const DCol& kc = batches[ref_bid(e)].keys[c];
                    const u64 row = ref_row(e);
                    v = dcol_valid(kc, row);
                    lo = dcol_bits(kc, row);
                    if (w == 16) hi = dcol_hi(kc, row);
                }
                if (!v) {  // null byte 1, value bytes 0
                    const u32 o = (u32)L.null_off[c];
                    k[o >> 3] |= 1ULL << (8 * (o & 7));
                } else {
                    legacy_put(k, L.off[c], lo, hi, w);
                }
            }
            h = legacy_fixed_crc(tab, k, L.words);
        }
        out[s] = legacy_bucket(h, L.bits);
    }
}

// Bucket (scheme 0 or 1) of every occupied slot by the group hash of its first `nk` key columns: a
// DISTINCT aggregate's pair table (keys..., x) is bucketed by its group's keys alone, so each of
// its buckets holds exactly the pairs of the groups the same bucket of the main table holds
// (AggregateDistinctCombinator's set travels inside its group's state in the reference,
// FUN/aggregate_combinator_distinct.rs:94-105).
__global__ void __launch_bounds__(BLOCK) prefix_slot_bucket_kernel(const Spec* __restrict__ spec, const BatchDesc* __restrict__ batches,
                                                                  TableDesc t, int nk, u32 n_parts, int scheme, u32* __restrict__ out) {
    const Spec& S = *spec;
    for (u64 s = blockIdx.x * (u64)BLOCK + threadIdx.x; s <= t.cap; s += (u64)gridDim.x * BLOCK) {
        const u64 e = t.slots[s * t.stride_words];
        if (e == SLOT_EMPTY) continue;
        const u64 h = S.inline_keys ? hash_packed(S, s == t.cap ? SLOT_EMPTY : e, nk) : group_hash(batches[ref_bid(e)].keys, nk, ref_row(e));
        out[s] = part_of(h, n_parts, scheme, nullptr, s);
    }
}

void launch_prefix_slot_bucket(hipStream_t s, const Spec* dspec, const BatchDesc* batches, const TableDesc& t, int nk, u32 n_parts,
                               int scheme, u32* out) {
    u64 blocks = (t.cap + 1 + BLOCK - 1) / BLOCK;
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL(prefix_slot_bucket_kernel, dim3((u32)blocks), dim3(BLOCK), 0, s, dspec, batches, t, nk, n_parts, scheme, out);
}

void launch_legacy_slot_bucket(hipStream_t s, const Spec* dspec, const BatchDesc* batches, const TableDesc& t, const LegacyLayout& L,
                               u32* out) {
    u64 blocks = (t.cap + 1 + BLOCK - 1) / BLOCK;
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL(legacy_slot_bucket_kernel, dim3((u32)blocks), dim3(BLOCK), 0, s, dspec, batches, t, L, out);
}

// Single-workgroup exclusive scan (in place) over n u64; *total = sum.
__global__ void __launch_bounds__(1024) exclusive_scan_kernel(u64* data, u64 n, u64* total) {
    __shared__ u64 sums[1024];
    u64 per = (n + 1023) / 1024;
    u64 a = threadIdx.x * per, b = a + per < n ? a + per : n;
    u64 acc = 0;
    for (u64 k = a; k < b; ++k) acc += data[k];
    sums[threadIdx.x] = acc;
    __syncthreads();
    for (int off = 1; off < 1024; off <<= 1) {
        u64 v = threadIdx.x >= (u32)off ? sums[threadIdx.x - off] : 0;
        __syncthreads();
        sums[threadIdx.x] += v;
        __syncthreads();
    }
    u64 run = threadIdx.x ? sums[threadIdx.x - 1] : 0;
    for (u64 k = a; k < b; ++k) {
        u64 v = data[k];
        data[k] = run;
        run += v;
    }
    if (threadIdx.x == 1023 && total) *total = sums[1023];
}

void launch_exclusive_scan(hipStream_t s, u64* data, u64 n, u64* total) {
    hipLaunchKernelGGL(exclusive_scan_kernel, dim3(1), dim3(1024), 0, s, data, n, total);
}

// ------------------------------------------------------------------------------------------
// Results (merge_result + flush_column): deterministic order inside a workgroup via block scan.
// ------------------------------------------------------------------------------------------

// flush_column of one group (slot s, entry e, state words st) into output row p; sp[c] = string
// write cursor of key column c (advanced).
__device__ __forceinline__ void write_group(const Spec& S, const BatchDesc* batches, const TableDesc& t, u64 s, const u64* st,
                                           u64 e, u64 p, u64* sp, const OutDesc& out) {
    // group columns
    if (S.inline_keys) {
        u64 key = s == t.cap ? SLOT_EMPTY : e;
        for (int c = 0; c < S.n_keys; ++c) {
            const dbg_datatype& ty = S.key_types[c];
            u32 w = type_width(ty.type);
            u64 b = (key >> (8 * S.koff[c])) & width_mask(w);
            bool v = ty.nullable ? ((key >> (8 * S.voff[c])) & 0xff) != 0 : true;
            write_bytes(out.key_data[c], p, w, b, 0);
            if (out.key_valid[c]) out.key_valid[c][p] = v ? 1 : 0;
        }
    } else if (S.kc_word && s < t.cap && (st[S.kc_word] & 1) && ((st[S.kc_word] >> 1) & 0x7FFF) <= 8 * KC_KEY_WORDS) {
        // one String key held by the slot's key cache: no read of the representative row
        const u32 len = (u32)((st[S.kc_word] >> 1) & 0x7FFF);
        u64 w[KC_KEY_WORDS];
#pragma unroll
        for (int j = 0; j < KC_KEY_WORDS; ++j) w[j] = st[S.kc_word + 1 + j];
        out.key_offsets[0][p] = sp[0];
        if (out.key_valid[0]) out.key_valid[0][p] = 1;
        if (sp[0] + len <= out.cap_str[0]) {
            u8* d = (u8*)out.key_data[0] + sp[0];
#pragma unroll
            for (u32 j = 0; j < 8 * KC_KEY_WORDS; ++j)
                if (j < len) d[j] = (u8)(w[j >> 3] >> (8 * (j & 7)));
        }
        sp[0] += len;
    } else {
        const BatchDesc& RB = batches[ref_bid(e)];
        u64 row = ref_row(e);
        for (int c = 0; c < S.n_keys; ++c) {
            const DCol& kc = RB.keys[c];
            bool v = dcol_valid(kc, row);
            if (out.key_valid[c]) out.key_valid[c][p] = v ? 1 : 0;
            if (kc.type == DBG_STRING) {
                StrRef r = dcol_str(kc, row);
                out.key_offsets[c][p] = sp[c];
                if (sp[c] + r.len <= out.cap_str[c]) {
                    u8* d = (u8*)out.key_data[c] + sp[c];
                    for (u64 j = 0; j < r.len; ++j) d[j] = r.p[j];
                }
                sp[c] += r.len;
            } else {
                u32 w = type_width(kc.type);
                write_bytes(out.key_data[c], p, w, dcol_bits(kc, row), w == 16 ? dcol_hi(kc, row) : 0);
            }
        }
    }
    for (int a = 0; a < S.n_aggs; ++a) write_agg(S, a, st, p, out, t.counters + CNT_ERR);
}

// Slot order within the block: iteration k covers slots base + k*BLOCK + tid (coalesced entry
// reads); positions come from a block-wide exclusive scan per iteration (wave shuffles + one
// LDS exchange), with running totals carried across iterations.  Same per-block ownership of
// slots as count_groups, so the scanned block offsets line up.
__global__ void __launch_bounds__(BLOCK) write_results_kernel(const Spec* __restrict__ spec, const BatchDesc* __restrict__ batches,
                                                             TableDesc t, const u64* pos, const u64* str_pos, u64 nblocks,
                                                             OutDesc out) {
    const Spec& S = *spec;
    // double-buffered per-wave sums: iteration k writes buffer k & 1, so one barrier per iteration
    // orders both its reads and the next iteration's writes
    __shared__ u64 wsum2[2][BLOCK / 64][1 + DBG_MAX_KEYS];
    const bool ref_strings = S.has_strings && !S.inline_keys;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const u64 base = (u64)blockIdx.x * SLOTS_PER_BLOCK;
    u64 run = pos[blockIdx.x];
    u64 srun[DBG_MAX_KEYS];
    if (ref_strings)
        for (int c = 0; c < S.n_keys; ++c)
            srun[c] = S.key_types[c].type == DBG_STRING ? str_pos[(u64)c * nblocks + blockIdx.x] : 0;
    auto wave_incl = [&](u64 v) {
        for (int off = 1; off < 64; off <<= 1) {
            u64 o = __shfl_up(v, off, 64);
            if (lane >= off) v += o;
        }
        return v;
    };
    // the next iteration's entry is loaded before this iteration's barrier
    auto entry_at = [&](u32 k) -> u64 {
        const u64 s = base + (u64)k * BLOCK + threadIdx.x;
        return s <= t.cap ? t.slots[s * t.stride_words] : SLOT_EMPTY;
    };
    u64 e_next = entry_at(0);
    for (u32 k = 0; k < SLOTS_PER_THREAD; ++k) {
        if (base + (u64)k * BLOCK > t.cap) break;  // uniform
        u64 (*wsum)[1 + DBG_MAX_KEYS] = wsum2[k & 1];
        const u64 s = base + (u64)k * BLOCK + threadIdx.x;
        const bool in = s <= t.cap;
        const u64* st = t.slots + (in ? s : 0) * t.stride_words;
        const u64 e = e_next;
        if (k + 1 < SLOTS_PER_THREAD) e_next = entry_at(k + 1);
        const u64 cnt = e != SLOT_EMPTY ? 1 : 0;
        u64 sb[DBG_MAX_KEYS];
        // inclusive count within the wave from one ballot (cnt is 0 / 1)
        const u64 ic = (u64)__popcll(__ballot(cnt != 0) & (lane == 63 ? ~0ULL : ((2ULL << lane) - 1)));
        if (lane == 63) wsum[wave][0] = ic;
        if (ref_strings)
            for (int c = 0; c < S.n_keys; ++c) {
                sb[c] = (cnt && S.key_types[c].type == DBG_STRING) ? slot_str_len(S, batches, t, s, e, c) : 0;
                u64 is = wave_incl(sb[c]);
                if (lane == 63) wsum[wave][1 + c] = is;
                sb[c] = is - sb[c];  // exclusive within the wave
            }
        __syncthreads();
        u64 p = run + ic - cnt, tot = 0;
        for (int w = 0; w < BLOCK / 64; ++w) {
            if (w < wave) p += wsum[w][0];
            tot += wsum[w][0];
        }
        u64 sp[DBG_MAX_KEYS];
        if (ref_strings)
            for (int c = 0; c < S.n_keys; ++c) {
                sp[c] = srun[c] + sb[c];
                u64 stot = 0;
                for (int w = 0; w < BLOCK / 64; ++w) {
                    if (w < wave) sp[c] += wsum[w][1 + c];
                    stot += wsum[w][1 + c];
                }
                srun[c] += stot;
            }
        run += tot;
        if (cnt && p < out.cap_groups) write_group(S, batches, t, s, st, e, p, sp, out);
    }
}

// ------------------------------------------------------------------------------------------
// finalize_small: count + scan + write + validity bits + string offsets in ONE workgroup, for
// tables of at most FIN_SMALL_SLOTS slots (low-cardinality queries: the four-launch finalize
// costs more than the work).  totals: [0] groups, [1 + c] string bytes of key column c.
//
// Each thread owns FIN_MAXPER consecutive slots whose entries it loads once, all in flight
// together, and keeps in registers for the write pass.  recycle != 0 (dbg_agg_set_recycle):
// the table is left re-initialised for the next batch (this kernel already holds every slot, so
// the reset costs no extra launch), unless an insert overflowed (the host then grows the table
// and finalizes again).  host_mirror (mapped pinned memory) receives the counters, the totals and
// finally `seq`, which the host polls instead of synchronising the stream.
// ------------------------------------------------------------------------------------------
#define FIN_NT 1024
#define FIN_MAXPER (FIN_SMALL_SLOTS / FIN_NT)
// The body, run by FIN_NT threads of one workgroup: the standalone kernel below, or the last
// workgroup of a fused insert (agg_insert_fast with FusedFin::on).  `view` holds the slots to
// read (t.slots, or a copy in LDS); the re-initialisation of a recycled table writes t.slots.
template <int MAXPER>
__device__ __forceinline__ bool finalize_small_body(const Spec& S, const BatchDesc* batches, const TableDesc& t, const u64* view,
                                                    const OutDesc& out, u64* totals, u64* host_mirror, int recycle, u64 seq,
                                                    u64* trace = nullptr, bool writeback = false, int xfin = 0) {
    __shared__ u64 wsum[FIN_NT / 64][1 + DBG_MAX_KEYS];
    __shared__ u64 cnts[CNT_WORDS];
    auto mark = [&](int k) { if (kPhaseTrace && trace && threadIdx.x == 0) trace[k] = __builtin_amdgcn_s_memrealtime(); };
    // Barriers here are LDS-only (no wait for this workgroup's global stores) unless a later
    // phase reads what other threads stored to global memory: every __syncthreads costs a
    // store round trip (vmcnt 0, ~1 us).
    auto lds_barrier = [] { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); };
    const u64 n_slots = t.cap + 1;
    const u32 per = (u32)((n_slots + FIN_NT - 1) / FIN_NT);  // <= MAXPER (host checks cap)
    const u64 base = (u64)threadIdx.x * per;
    const bool ref_strings = S.has_strings && !S.inline_keys;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    bool has_bits = false, dec_err = false;  // uniform
    for (int c = 0; c < S.n_keys; ++c) has_bits |= out.key_valid[c] && out.key_bits[c];
    for (int a = 0; a < S.n_aggs; ++a) {
        has_bits |= (out.agg_valid[a] || ((out.all_valid >> a) & 1)) && out.agg_bits[a];
        dec_err |= S.aggs[a].dec_check || (S.aggs[a].kind == DBG_AGG_AVG && S.aggs[a].sumk == SUMK_I128);
    }
    // the table counters, in flight while the table is scanned (final: every inserting workgroup
    // has finished; write_group may still set decimal-overflow bits, reloaded below)
    u64 myc = threadIdx.x < CNT_WORDS ? ld_sc1(t.counters + threadIdx.x) : 0;
    u64 ent[MAXPER];
#pragma unroll
    for (u32 k = 0; k < MAXPER; ++k) {
        u64 s = base + k;
        ent[k] = (k < per && s < n_slots) ? view[s * t.stride_words] : SLOT_EMPTY;
    }
    u64 cnt = 0, sb[DBG_MAX_KEYS];
    u32 occ = 0;  // occupied owned slots (bit k = slot base + k)
    for (int c = 0; c < DBG_MAX_KEYS; ++c) sb[c] = 0;
#pragma unroll
    for (u32 k = 0; k < MAXPER; ++k) {
        if (ent[k] == SLOT_EMPTY) continue;
        cnt++;
        occ |= 1u << k;
        if (ref_strings)
            for (int c = 0; c < S.n_keys; ++c)
                if (S.key_types[c].type == DBG_STRING) sb[c] += key_str_len(S, batches, ent[k], c);
    }
    // block exclusive scan of cnt (and of the string bytes of each key column)
    auto wave_incl = [&](u64 v) {
        for (int off = 1; off < 64; off <<= 1) {
            u64 o = __shfl_up(v, off, 64);
            if (lane >= off) v += o;
        }
        return v;
    };
    u64 ic = wave_incl(cnt);
    u64 isb[DBG_MAX_KEYS];
    if (ref_strings)
        for (int c = 0; c < S.n_keys; ++c) isb[c] = wave_incl(sb[c]);
    if (lane == 63) {
        wsum[wave][0] = ic;
        if (ref_strings)
            for (int c = 0; c < S.n_keys; ++c) wsum[wave][1 + c] = isb[c];
    }
    lds_barrier();
    u64 p = ic - cnt, sp[DBG_MAX_KEYS];
    for (int w = 0; w < wave; ++w) p += wsum[w][0];
    if (ref_strings)
        for (int c = 0; c < S.n_keys; ++c) {
            sp[c] = isb[c] - sb[c];
            for (int w = 0; w < wave; ++w) sp[c] += wsum[w][1 + c];
        }
    u64 total = 0, stot[DBG_MAX_KEYS];
    for (int w = 0; w < FIN_NT / 64; ++w) total += wsum[w][0];
    for (int c = 0; c < S.n_keys; ++c) {
        stot[c] = 0;
        if (ref_strings)
            for (int w = 0; w < FIN_NT / 64; ++w) stot[c] += wsum[w][1 + c];
    }
    mark(7);
    // write pass over the occupied slots only (one write_group instance in the code; the entry
    // is re-read from the cache rather than indexed out of the register array)
    const u32 occ_all = occ;
    if (kExperiments && (xfin & 1)) occ = 0;  // timing ablation (EXP=1 builds only)
    while (occ && p < out.cap_groups) {
        const u32 k = __builtin_ctz(occ);
        occ &= occ - 1;
        const u64 s = base + k;
        const u64* st = view + s * t.stride_words;
        write_group(S, batches, t, s, st, st[0], p, sp, out);
        p++;
    }
    mark(8);
    u64 n = total < out.cap_groups ? total : out.cap_groups;
    if (has_bits && !(kExperiments && (xfin & 2))) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();  // validity bytes of every row are in global memory
        const u32 ncols = (u32)(S.n_keys + S.n_aggs);
        for (u64 f = threadIdx.x; f < (n + 7) / 8 * ncols; f += FIN_NT) {  // one (byte, column) per thread
            const u64 k = f / ncols;
            const int c = (int)(f % ncols);
            {
                const u8* bytes = c < S.n_keys ? out.key_valid[c] : out.agg_valid[c - S.n_keys];
                u8* bits = c < S.n_keys ? out.key_bits[c] : out.agg_bits[c - S.n_keys];
                if (!bytes && bits && c >= S.n_keys && ((out.all_valid >> (c - S.n_keys)) & 1)) {
                    bits[k] = all_valid_byte(n, k);
                    continue;
                }
                if (!bytes || !bits) continue;
                u8 b = 0;
                for (int j = 0; j < 8; ++j) {
                    u64 i = k * 8 + j;
                    if (i < n && bytes[i]) b |= (u8)(1u << j);
                }
                bits[k] = b;
            }
        }
    }
    if (threadIdx.x == 0) {
        totals[0] = total;
        for (int c = 0; c < S.n_keys; ++c) {
            totals[1 + c] = stot[c];
            if (out.key_offsets[c] && total <= out.cap_groups) out.key_offsets[c][total] = stot[c];
        }
    }
    if (dec_err) {
        __syncthreads();  // decimal-overflow bits of write_group are in the counters
        if (threadIdx.x == CNT_ERR) myc = ld_sc1(t.counters + CNT_ERR);
    }
    if (threadIdx.x < CNT_WORDS) cnts[threadIdx.x] = myc;
    lds_barrier();
    mark(9);
    // recycle only when the caller got every group (short buffers: the table must stay intact
    // for the retry with larger ones) and no insert overflowed (the host grows and finalizes again)
    bool rc = recycle && cnts[CNT_OVF_ROWS] == 0 && cnts[CNT_OVF_RECS] == 0 && total <= out.cap_groups;
    for (int c = 0; c < S.n_keys; ++c)
        if (ref_strings && S.key_types[c].type == DBG_STRING && stot[c] > out.cap_str[c]) rc = false;
    if (rc && threadIdx.x < CNT_WORDS) t.counters[threadIdx.x] = 0;  // dbg_agg_reset
    // zero-copy read-back: the table counters and the totals go straight to mapped pinned host
    // memory ([0, CNT_WORDS) counters, then totals), so finalize needs no copy launches
    // (system-scope stores: written through to host memory, never parked in the L2)
    auto put = [&](int w, u64 v) { __hip_atomic_store(host_mirror + w, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM); };
    if (threadIdx.x == 0) {
        if (host_mirror) {
            for (int w = 0; w < CNT_WORDS; ++w) put(w, cnts[w]);
            put(CNT_WORDS, total);
            for (int c = 0; c < S.n_keys; ++c) put(CNT_WORDS + 1 + c, stot[c]);
            put(CNT_WORDS + 1 + DBG_MAX_KEYS, rc ? 1 : 0);  // recycled
        }
    }
    mark(10);
    if (!rc && writeback)  // `view` is an LDS table the HBM table does not hold yet
        for (u64 i = threadIdx.x; i < n_slots * t.stride_words; i += FIN_NT) t.slots[i] = view[i];
    if (rc) {  // table_init of the owned slots that were claimed (an EMPTY slot is still in its
               // initial state: state words are only written after the entry is claimed)
        const u32 sw = (u32)t.stride_words;
        u32 o = occ_all;
        while (o) {
            const u32 k = __builtin_ctz(o);
            o &= o - 1;
            u64* d = t.slots + (base + k) * sw;
            for (u32 w = 0; w < sw; ++w) d[w] = S.slot_init[w];
        }
    }
    // `seq` last: thread 0 waits for its write-through mirror stores to complete before posting it.  No system-scope release: that would write
    // back the whole L2; the output columns are consumed in stream order on the device.
    if (host_mirror && threadIdx.x == 0) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_store(host_mirror + CNT_WORDS + 2 + DBG_MAX_KEYS, seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
    return rc;
}

__global__ void __launch_bounds__(FIN_NT) finalize_small_kernel(const Spec* __restrict__ spec, const BatchDesc* __restrict__ batches,
                                                                TableDesc t, OutDesc out, u64* totals, u64* host_mirror,
                                                                int recycle, u64 seq, int xfin) {
    if (kExperiments && (xfin & 8)) return;  // timing ablation (EXP=1 builds only)
    finalize_small_body<FIN_MAXPER>(*spec, batches, t, t.slots, out, totals, host_mirror, recycle, seq, nullptr, false, xfin);
}

void launch_finalize_small(hipStream_t s, const Spec* dspec, const BatchDesc* batches, const TableDesc& t, const OutDesc& out,
                           u64* totals, u64* host_mirror, int recycle, u64 seq) {
    static const int xfin = X_ENV("DBG_X_FIN") ? atoi(X_ENV("DBG_X_FIN")) : 0;
    hipLaunchKernelGGL(finalize_small_kernel, dim3(1), dim3(FIN_NT), 0, s, dspec, batches, t, out, totals, host_mirror, recycle,
                       seq, xfin);
}

// The last workgroup of an insert launch finalizes the table (FusedFin).  Hand-off
// (MI355X_MICROARCH.md, inter-workgroup visibility, valid forms: agent atomics / sc1 stores on
// the producer side, the workgroup whose ticket add came last as the consumer, sc1 global loads
// of every handed-off byte): every table word of this launch was written by agent-scope atomics
// (g_find's CAS, apply_row / apply_state) and read back only by sc1 loads (g_find's volatile
// entry loads, ld_sc1 here); every wave drains its memory operations and the barrier orders
// them before lane 0's ticket add.  The last workgroup copies the table into LDS with sc1 loads
// and runs the finalize_small body on the copy (recycle re-initialises t.slots directly).
__device__ __forceinline__ void fused_finalize(const Spec& S, const BatchDesc* batches, const TableDesc& t, u64* lds,
                                               const FusedFin& ff) {
    __shared__ u32 is_last;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        u64 tk = atomicAdd((unsigned long long*)(t.counters + CNT_FIN_TICKET), 1ULL);
        is_last = tk == (u64)gridDim.x - 1 ? 1u : 0u;
    }
    __syncthreads();
    if (!is_last) return;
    if (kPhaseTrace && ff.trace && threadIdx.x == 0) ff.trace[4] = __builtin_amdgcn_s_memrealtime();
    const u64 n = (t.cap + 1) * t.stride_words;  // host: <= the launch's dynamic LDS
    for (u64 i = threadIdx.x; i < n; i += FIN_NT) lds[i] = ld_sc1(t.slots + i);
    if (threadIdx.x == 0) atomicExch((unsigned long long*)(t.counters + CNT_FIN_TICKET), 0ULL);
    __syncthreads();
    if (kPhaseTrace && ff.trace && threadIdx.x == 0) ff.trace[5] = __builtin_amdgcn_s_memrealtime();
    finalize_small_body<FUSED_FIN_SLOTS / FIN_NT>(S, batches, t, lds, ff.out, ff.totals, ff.host_mirror, ff.recycle, ff.seq,
                                                  ff.trace);
    if (kPhaseTrace && ff.trace && threadIdx.x == 0) ff.trace[6] = __builtin_amdgcn_s_memrealtime();
}

// merge_states of a parked partial state (sc1 loads) into a slot; COUNT(*) alone (CO): one add
template <int AS, bool CO>
__device__ __forceinline__ void merge_parked(const Spec& S, u64* st, const u64* r, u64 c1) {
    if constexpr (CO) {  // c1: the parked count, loaded with the entry
        if (c1) at_add<AS>(asp<AS>(st + 1), c1);
    } else {
        apply_state<AS, true>(S, asp<AS>(st), r);
    }
}

// finalize_small_body for the COUNT(*)-only fast kernel (one non-null integer key of type T,
// slots [key][count]): the same outputs, counters, recycle and host mirror in a fraction of the
// code — this tail runs once per launch on whichever CU finishes last, from a cold instruction
// cache, so its length is latency.
template <typename T>
__device__ __forceinline__ void finalize_count_only(const TableDesc& t, const u64* view, const FusedFin& ff, bool known,
                                                    u32 view_claims, bool hbm_clean = false) {
    __shared__ u64 wsum[FIN_NT / 64];
    __shared__ u64 cnts[CNT_WORDS];
    auto lds_barrier = [] { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); };
    const OutDesc& out = ff.out;
    const u64 n_slots = t.cap + 1;
    constexpr u32 PER = FUSED_FIN_SLOTS / FIN_NT;
    const u64 base = (u64)threadIdx.x * PER;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    u64 myc = (!known && threadIdx.x < CNT_WORDS) ? ld_sc1(t.counters + threadIdx.x) : 0;
    u64 ent[PER];
    u32 occ = 0, cnt = 0;
#pragma unroll
    for (u32 k = 0; k < PER; ++k) {
        const u64 s = base + k;
        ent[k] = s < n_slots ? view[s * 2] : SLOT_EMPTY;
        if (ent[k] != SLOT_EMPTY) {
            occ |= 1u << k;
            cnt++;
        }
    }
    u64 ic = cnt;
    for (int off = 1; off < 64; off <<= 1) {
        const u64 o = __shfl_up(ic, off, 64);
        if (lane >= off) ic += o;
    }
    if (lane == 63) wsum[wave] = ic;
    lds_barrier();
    u64 p = ic - cnt, total = 0;
    for (int w = 0; w < FIN_NT / 64; ++w) {
        if (w < wave) p += wsum[w];
        total += wsum[w];
    }
#pragma unroll
    for (u32 k = 0; k < PER; ++k) {
        if (!((occ >> k) & 1) || p >= out.cap_groups) continue;
        const u64 s = base + k;
        ((T*)out.key_data[0])[p] = (T)(s == t.cap ? SLOT_EMPTY : ent[k]);
        ((u64*)out.agg_data[0])[p] = view[s * 2 + 1];
        p++;
    }
    if (threadIdx.x == 0) ff.totals[0] = total;
    // known: every group of the table was claimed in this launch, nothing overflowed
    if (known) myc = threadIdx.x == CNT_CLAIMS ? total : 0;
    if (threadIdx.x < CNT_WORDS) cnts[threadIdx.x] = myc;
    lds_barrier();
    const bool rc = ff.recycle && cnts[CNT_OVF_ROWS] == 0 && cnts[CNT_OVF_RECS] == 0 && total <= out.cap_groups;
    if (rc && threadIdx.x < CNT_WORDS) t.counters[threadIdx.x] = 0;  // dbg_agg_reset
    // known counters: the view's claims were not added yet (fused_chain); a table that outlives
    // this finalize needs them
    if (known && !rc && threadIdx.x == 0 && view_claims)
        atomicAdd((unsigned long long*)(t.counters + CNT_CLAIMS), (unsigned long long)view_claims);
    u64* hm = ff.host_mirror;
    auto put = [&](int w, u64 v) { __hip_atomic_store(hm + w, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM); };
    // known counters: one self-validating word ([seq | recycled | groups], MIRROR_COMPACT) instead
    // of the counter words and a seq posted behind a wait for them
    const bool compact = known && total < (1u << 24);
    if (hm && compact && threadIdx.x == 0)
        put(MIRROR_COMPACT, (ff.seq << 25) | ((rc ? 1ULL : 0ULL) << 24) | total);
    if (hm && !compact && threadIdx.x == 0) {
        for (int w = 0; w < CNT_WORDS; ++w) put(w, cnts[w]);
        put(CNT_WORDS, total);
        put(CNT_WORDS + 1, 0);  // string bytes of the (integer) key column
        put(CNT_WORDS + 1 + DBG_MAX_KEYS, rc ? 1 : 0);
    }
    if (!rc)  // the table outlives this finalize: the view holds groups the HBM table does not
        for (u64 i = threadIdx.x; i < n_slots * 2; i += FIN_NT) t.slots[i] = view[i];
    if (rc && !hbm_clean)  // table_init of the claimed slots of the view (the HBM copy may hold fewer: same
                           // values); hbm_clean: empty at launch and never written since — nothing to undo
#pragma unroll
        for (u32 k = 0; k < PER; ++k)
            if ((occ >> k) & 1) {
                u64* d = t.slots + (base + k) * 2;
                d[0] = SLOT_EMPTY;
                d[1] = 0;
            }
    if (hm && !compact && threadIdx.x == 0) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __hip_atomic_store(hm + CNT_WORDS + 2 + DBG_MAX_KEYS, ff.seq, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    }
}

// Find or claim `key` (inline) in an LDS copy of the HBM table (same slots, same probing as
// g_find).  false: the probe limit was hit.
__device__ __forceinline__ bool view_find(u64* view, const TableDesc& t, u64 key, u32& claims, u64& slot) {
    const u32 sw = t.stride_words;
    if (key == SLOT_EMPTY) {  // the all-ones 8-byte key: sentinel slot, entry 0 once claimed
        slot = t.cap;
        claims += at_cas<AS_LDS>(asp<AS_LDS>(view + t.cap * sw), SLOT_EMPTY, 0ULL) == SLOT_EMPTY ? 1u : 0u;
        return true;
    }
    const u64 mask = t.cap - 1;
    u64 s = slot_mix(key) & mask;
    for (u32 p = 0; p < t.probe_limit; ++p) {
        wptr<AS_LDS> e = asp<AS_LDS>(view + s * sw);
        u64 ev = vld<AS_LDS>(e);
        if (ev == SLOT_EMPTY) {
            const u64 old = at_cas<AS_LDS>(e, SLOT_EMPTY, key);
            if (old == SLOT_EMPTY) {
                claims++;
                slot = s;
                return true;
            }
            ev = old;
        }
        if (ev == key) {
            slot = s;
            return true;
        }
        s = (s + 1) & mask;
    }
    return false;
}

// The end of a fused COUNT(*) launch over keys of <= 16 bits (ClickBench Q8: Int16 AdvEngineID):
// a direct-mapped hand-off instead of the parked-row tree.  Every workgroup adds its LDS table's
// counts into a dense array indexed by the key (device atomics without return, issued as soon as
// it has streamed its share — overlapping the workgroups still streaming) and sets the key's bit
// in a presence bitmap, then takes the launch ticket; the last arrival reads the bitmap and the
// counts of the set bits (zeroing both behind it for the next launch), merges them into an LDS
// view of the table and runs the count-only finalize.  The critical path after the last workgroup
// streams is one atomic drain, one ticket and two dependent loads — against the tree's two park /
// ticket / reload levels — and the merge no longer grows with the grid.
template <typename T>
__device__ __forceinline__ void fused_dense(const Spec& S, const BatchDesc* batches, const BatchDesc& B, u64* lds, u32 lds_slots,
                                            u32 sw, u32* lcount, u32 nt, const TableDesc& t, u32 my_claims, u32 my_ovf,
                                            const FusedFin& ff) {
    __shared__ u32 role, bad, vcl, wg_ovf;
    __shared__ u64 hbm_claims, ovf_seen;
    const u32 dn = ff.dense_n, dmask = dn - 1;
    u64* dcnt = ff.dense;
    u64* dbits = ff.dense + dn;
    if (threadIdx.x == 0) wg_ovf = 0;
    // 1. the LDS table into the dense array (no return values: the stores drain before the ticket)
    for (u32 s = threadIdx.x; s < lds_slots; s += nt) {
        const u64* p = lds + (u64)s * sw;
        const u64 e = p[0];
        if (e == SLOT_EMPTY) continue;
        const u32 idx = (u32)e & dmask;
        __hip_atomic_fetch_add(dcnt + idx, p[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_fetch_or(dbits + (idx >> 6), 1ULL << (idx & 63), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    if (my_claims) atomicAdd(&lcount[1], my_claims);
    if (my_ovf) atomicAdd(&wg_ovf, my_ovf);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (threadIdx.x == 0) {
        if (lcount[1]) {
            atomicAdd((unsigned long long*)(t.counters + CNT_CLAIMS), (unsigned long long)lcount[1]);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        const u64 add = 1 + ((u64)lcount[1] << 16) + ((u64)wg_ovf << 40);
        const u64 tk = atomicAdd((unsigned long long*)(t.counters + CNT_FIN_TICKET), (unsigned long long)add) + add;
        role = (tk & 0xFFFF) == gridDim.x ? 1u : 0u;
        hbm_claims = (tk >> 16) & 0xFFFFFF;
        ovf_seen = tk >> 40;
    }
    __syncthreads();
    if (kPhaseTrace && ff.trace && threadIdx.x == 0) atomicMax((unsigned long long*)ff.trace + 3, (unsigned long long)__builtin_amdgcn_s_memrealtime());
    if (!role) return;
    // 2. the last arrival: view of the table, the dense groups merged into it, finalize
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        atomicExch((unsigned long long*)(t.counters + CNT_FIN_TICKET), 0ULL);
        atomicExch((unsigned long long*)(t.counters + CNT_TAIL), 0ULL);  // every workgroup has left its tail
        bad = 0;
        vcl = 0;
        lcount[2] = 0;
        if (kPhaseTrace && ff.trace) ff.trace[4] = __builtin_amdgcn_s_memrealtime();
    }
    const u64 n = (t.cap + 1) * sw;  // host: <= the launch's dynamic LDS
    if (ff.table_empty && hbm_claims == 0)
        for (u64 i = threadIdx.x; i < n; i += nt) lds[i] = S.slot_init[i % sw];
    else
        for (u64 i = threadIdx.x; i < n; i += nt) lds[i] = ld_sc1(t.slots + i);
    __syncthreads();
    u32 vclaims = 0;
    for (u32 w = threadIdx.x; w < (dn >> 6); w += nt) {
        u64 b = ld_sc1(dbits + w);
        if (!b) continue;
        st_sc1(dbits + w, 0);
        while (b) {
            const u32 j = (u32)__builtin_ctzll(b);
            b &= b - 1;
            const u32 idx = (w << 6) | j;
            const u64 c = ld_sc1(dcnt + idx);
            st_sc1(dcnt + idx, 0);
            const u64 key = (u64)idx;  // the inline packed key of a <= 16-bit column: its raw bits
            u64 slot;
            if (view_find(lds, t, key, vclaims, slot)) {
                lds[slot * sw + 1] += c;  // one thread per key
            } else {  // an overflow record (the host grows the table and finalizes again)
                const u64 k = atomicAdd((unsigned long long*)(t.counters + CNT_OVF_RECS), 1ULL);
                if (k < t.ovf_recs_cap) {
                    u64* r = t.ovf_recs + k * t.stride_words;
                    r[0] = key;
                    r[1] = c;
                } else {
                    atomicOr((unsigned long long*)(t.counters + CNT_ERR), (unsigned long long)ERR_OVF_LOST);
                }
                bad = 1;
            }
        }
    }
    if (vclaims) atomicAdd(&vcl, vclaims);
    __syncthreads();
    const bool known = ff.table_empty && ovf_seen == 0 && !bad;
    if (threadIdx.x == 0 && vcl && !known) {
        atomicAdd((unsigned long long*)(t.counters + CNT_CLAIMS), (unsigned long long)vcl);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    if (kPhaseTrace && ff.trace && threadIdx.x == 0) ff.trace[5] = __builtin_amdgcn_s_memrealtime();
    finalize_count_only<T>(t, lds, ff, known, vcl);
    if (kPhaseTrace && ff.trace && threadIdx.x == 0) ff.trace[6] = __builtin_amdgcn_s_memrealtime();
}

// The low-cardinality end of a fused insert + finalize launch (ClickBench Q8: 32 groups in every
// workgroup's LDS table).  The HBM table is not written on the way: partial tables travel as
// parked rows up a two-level tree and are merged in LDS, and the last workgroup finalizes from
// an LDS view of the table with the group tables merged in.
//   1. every workgroup parks its LDS table (<= SCR_ENTRIES groups; a larger one flushes into the
//      HBM table as block_flush does) and takes its group's ticket;
//   2. the last workgroup of each group of SCR_GROUP merges the group's parked rows in LDS,
//      parks the merged table in the group's row and takes the launch ticket;
//   3. the last group leader copies the HBM table (groups of earlier launches and direct flushes)
//      into LDS, merges every group row into that view and runs the finalize body on it.  The
//      view goes back to HBM only when the table outlives the finalize (no recycle) or a key did
//      not fit the view (overflow record: the host grows the table and finalizes again).
// Each hand-off is a store drain + one ticket + sc1 loads (MI355X_MICROARCH.md, inter-workgroup
// visibility); against block_flush + fused_finalize this saves the HBM probe / CAS / atomic
// round trips of the group leaders' flush and one barrier + ticket level.
template <typename T, bool CO>
__device__ __forceinline__ void fused_chain(const Spec& S, const BatchDesc* batches, const BatchDesc& B, u64* lds, u32 lds_slots,
                                            u32 sw, u32* lcount, u32 nt, const TableDesc& t, u32 my_claims, u32 my_ovf,
                                            const FusedFin& ff) {
    __shared__ u32 role, bad, vcl, wg_ovf;  // (the view overwrites lcount: the table copy extends past lds_slots)
    const u32 lmask = lds_slots - 1;
    const u32 llimit = lds_slots - lds_slots / 4;
    u64* counts = t.scratch;
    u64* tickets = t.scratch + t.scr_blocks;
    u64* gmeta = tickets + t.scr_blocks / 2;  // [group] parked entries of the group row
    u64* rows = t.scratch + 2 * (u64)t.scr_blocks;
    u64* grows = rows + (u64)t.scr_blocks * SCR_ENTRIES * sw;
    const u32 n_groups = (gridDim.x + SCR_GROUP - 1) / SCR_GROUP;
    const u32 g = blockIdx.x / SCR_GROUP;
    const u32 gsize = min((u32)SCR_GROUP, gridDim.x - g * SCR_GROUP);
    if (threadIdx.x == 0) wg_ovf = 0;
    __syncthreads();
    // park the LDS table (compacted) in `dst` with sc1 stores, or flush it into the HBM table when
    // it holds more than a row takes (counted as a possible overflow: the flush may push
    // records); returns the parked entries (uniform)
    auto park = [&](u64* dst) -> u64 {
        if (lcount[0] > SCR_ENTRIES) {
            flush_lds_direct<true, false>(S, batches, B, lds, lds_slots, sw, nt, t, my_claims);
            my_ovf += threadIdx.x == 0 ? 1u : 0u;
            return 0;
        }
        for (u32 s = threadIdx.x; s < lds_slots; s += nt) {
            const u64* p = lds + (u64)s * sw;
            if (p[0] == SLOT_EMPTY) continue;
            const u32 k = atomicAdd(&lcount[2], 1u);
            u64* d = dst + (u64)k * sw;
            for (u32 w = 0; w <= (u32)S.n_words; ++w) st_sc1(d + w, p[w]);
        }
        __syncthreads();
        return lcount[2];
    };
    // HBM claims of this workgroup into the table counter, then a ticket (thread 0; both device
    // atomics complete in order: the ticket's taker sees the claims)
    // A ticket word carries, besides the arrivals (bits [0, 16)), the HBM claims (bits [16, 40))
    // and the possible overflow pushes (bits [40, 64)) of the workgroups that took it, so the last
    // arrival knows without another load whether this launch created groups in HBM or pushed
    // overflow records (the finalize then needs neither the table nor the counters).
    auto claims_and_ticket = [&](u64* ticket, u64 carried_claims, u64 carried_ovf) -> u64 {
        if (my_claims) atomicAdd(&lcount[1], my_claims);
        if (my_ovf) atomicAdd(&wg_ovf, my_ovf);
        my_claims = my_ovf = 0;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        u64 tk = 0;
        if (threadIdx.x == 0) {
            if (lcount[1]) {
                atomicAdd((unsigned long long*)(t.counters + CNT_CLAIMS), (unsigned long long)lcount[1]);
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            const u64 add = 1 + ((carried_claims + lcount[1]) << 16) + ((carried_ovf + wg_ovf) << 40);
            tk = atomicAdd((unsigned long long*)ticket, (unsigned long long)add) + add;  // inclusive
        }
        return tk;
    };
    // 1. park, group ticket
    const u64 np = park(rows + (u64)blockIdx.x * SCR_ENTRIES * sw);
    if (threadIdx.x == 0) st_sc1(counts + blockIdx.x, np);
    __shared__ u64 hbm_claims, ovf_seen;  // this launch's HBM claims / possible overflow pushes: the
                                          // group's (leader), all (last leader)
    {
        const u64 tk = claims_and_ticket(tickets + g, 0, 0);
        if (threadIdx.x == 0) {
            role = (tk & 0xFFFF) == gsize ? 1u : 0u;
            hbm_claims = (tk >> 16) & 0xFFFFFF;
            ovf_seen = tk >> 40;
            wg_ovf = 0;
        }
    }
    __syncthreads();
    if (!role) return;
    // 2. group leader: merge the group's parked rows in LDS, park the result in the group row
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        tickets[g] = 0;  // ready for the next launch on this table (all members have added)
        lcount[0] = lcount[1] = lcount[2] = 0;
    }
    lds_table_init(S, lds, lds_slots, sw, nt);
    __syncthreads();
    for (u32 f = threadIdx.x; f < gsize * SCR_ENTRIES; f += nt) {
        const u64 b = (u64)g * SCR_GROUP + f / SCR_ENTRIES, k = f % SCR_ENTRIES;
        const u64* r = rows + (b * SCR_ENTRIES + k) * sw;
        const u64 cnt = ld_sc1(counts + b);
        const u64 e = ld_sc1(r);  // issued with the count: rows are allocated in full
        const u64 c1 = CO ? ld_sc1(r + 1) : 0;  // COUNT(*): the whole state, in the same round trip
        if (k >= cnt) continue;
        const int ls = lds_find<true>(S, batches, B.keys, 0, e, 0, lds, lmask, sw, lcount, llimit);
        if (ls >= 0) {
            merge_parked<AS_LDS, CO>(S, lds + (u64)ls * sw, r, c1);
            continue;
        }
        bool claimed;
        const u64 gs = g_find<true>(S, batches, B.keys, 0, e, 0, t, t.probe_limit, claimed);
        if (gs == ~0ULL) {
            push_ovf_rec<true>(S, t, e, r);
            my_ovf++;
            continue;
        }
        my_claims += claimed ? 1 : 0;
        merge_parked<AS_GLB, CO>(S, t.slots + gs * t.stride_words, r, c1);
    }
    __syncthreads();
    const u64 gp = park(grows + (u64)g * SCR_ENTRIES * sw);
    if (threadIdx.x == 0) st_sc1(gmeta + g, gp);
    {
        const u64 tk = claims_and_ticket(t.counters + CNT_FIN_TICKET, hbm_claims, ovf_seen);
        if (threadIdx.x == 0) {
            role = (tk & 0xFFFF) == n_groups ? 2u : 0u;
            hbm_claims = (tk >> 16) & 0xFFFFFF;
            ovf_seen = tk >> 40;
        }
    }
    __syncthreads();
    if (kPhaseTrace && ff.trace && threadIdx.x == 0) atomicMax((unsigned long long*)ff.trace + 3, (unsigned long long)__builtin_amdgcn_s_memrealtime());
    if (role != 2) return;
    // 3. the last group leader: view of the HBM table, group rows merged into it, finalize
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        atomicExch((unsigned long long*)(t.counters + CNT_FIN_TICKET), 0ULL);
        atomicExch((unsigned long long*)(t.counters + CNT_TAIL), 0ULL);  // every workgroup has left its tail
        bad = 0;
        vcl = 0;
        if (kPhaseTrace && ff.trace) ff.trace[4] = __builtin_amdgcn_s_memrealtime();
    }
    // the view: the HBM table, or its initial state when it was empty at launch start (recycled
    // by the previous finalize) and no workgroup of this launch created a group in it
    const u64 n = (t.cap + 1) * sw;  // host: <= the launch's dynamic LDS
    if (ff.table_empty && hbm_claims == 0)
        for (u64 i = threadIdx.x; i < n; i += nt) lds[i] = S.slot_init[i % sw];
    else
        for (u64 i = threadIdx.x; i < n; i += nt) lds[i] = ld_sc1(t.slots + i);
    __syncthreads();
    u32 vclaims = 0;
    for (u32 f = threadIdx.x; f < n_groups * SCR_ENTRIES; f += nt) {
        const u64 gg = f / SCR_ENTRIES, k = f % SCR_ENTRIES;
        const u64* r = grows + (gg * SCR_ENTRIES + k) * sw;
        const u64 cnt = ld_sc1(gmeta + gg);
        const u64 e = ld_sc1(r);
        const u64 c1 = CO ? ld_sc1(r + 1) : 0;
        if (k >= cnt) continue;
        u64 slot;
        if (view_find(lds, t, e, vclaims, slot)) {
            merge_parked<AS_LDS, CO>(S, lds + slot * sw, r, c1);
        } else {
            push_ovf_rec<true>(S, t, e, r);
            bad = 1;
        }
    }
    if (vclaims) atomicAdd(&vcl, vclaims);
    __syncthreads();
    const bool known = ff.table_empty && ovf_seen == 0 && !bad;
    // the view's claims into the table counter: before the finalize reads the counters, or — when
    // they are known (count-only) — only if the table outlives the finalize (finalize_count_only)
    if (threadIdx.x == 0 && vcl && !(CO && known)) {
        atomicAdd((unsigned long long*)(t.counters + CNT_CLAIMS), (unsigned long long)vcl);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    if (kPhaseTrace && ff.trace && threadIdx.x == 0) ff.trace[5] = __builtin_amdgcn_s_memrealtime();
    // the finalize writes the view back when the table outlives it (no recycle: short buffers, an
    // overflow record, or a caller that keeps the table)
    // counters known without a load: an empty table at launch start, no overflow anywhere
    if constexpr (CO) finalize_count_only<T>(t, lds, ff, known, vcl);
    else finalize_small_body<FUSED_FIN_SLOTS / FIN_NT>(S, batches, t, lds, ff.out, ff.totals, ff.host_mirror, ff.recycle, ff.seq,
                                                       ff.trace, true);
    if (kPhaseTrace && ff.trace && threadIdx.x == 0) ff.trace[6] = __builtin_amdgcn_s_memrealtime();
}

// The fused chain for COUNT(*) over a key of <= 16 bits (ClickBench Q8's Int16 AdvEngineID), with
// self-validating parked rows so that every hand-off costs one round trip instead of three.  The
// chain above parks a table, drains the stores, takes a ticket, and the last arrival then loads
// the rows: store drain + ticket + loads on the critical path at both levels.  Here a workgroup
// takes its ticket FIRST and parks only if it is not the last: the last arrival merges its own
// table in place (no park, no reload) and loads the others' rows while they may still be landing.
// A parked entry is one word, [key 16 b | count 24 b (level 2: 28 b) | tag 24 b (level 2: 20 b)],
// the tag the launch's sequence number, so an entry is accepted only once this launch's word is
// visible; the row's entry count is posted as [seq 44 b | entries 20 b] after the entries.  A
// reader spins (bounded) on an item until both are current — no acquire / release pair, no
// second round trip.  (A workgroup covers < 2^24 rows, a group of 16 < 2^28: the host launches
// at most 256 workgroups over < 2^32 rows, and a grid below 256 covers <= 32768 rows each.)
#ifndef CHAIN_TAGGED
#define CHAIN_TAGGED 1  // 0: the generic chain for these launches too (A/B builds: make EXP=1 EXTRA=-DCHAIN_TAGGED=0)
#endif
constexpr bool kChainTagged = CHAIN_TAGGED != 0;
#define TAG1_BITS 24
#define TAG2_BITS 20
__device__ __forceinline__ u64 chain_pack(u64 key, u64 cnt, u64 seq, int level) {
    const int tb = level == 1 ? TAG1_BITS : TAG2_BITS;
    return key | (cnt << 16) | ((seq & ((1ULL << tb) - 1)) << (64 - tb));
}

template <typename T>
__device__ __forceinline__ void fused_chain_tagged(const Spec& S, const BatchDesc* batches, const BatchDesc& B, u64* lds, u32 lds_slots,
                                                   u32 sw, u32* lcount, u32 nt, const TableDesc& t, u32 my_claims, u32 my_ovf,
                                                   const FusedFin& ff) {
    constexpr int OWN = 4;  // own slots per thread the last leader holds in registers (lds_slots <= 4 x nt, host-checked)
    __shared__ u32 role, bad, vcl, wg_ovf;
    __shared__ u64 hbm_claims, ovf_seen;
    const u32 lmask = lds_slots - 1;
    const u32 llimit = lds_slots - lds_slots / 4;
    u64* counts = t.scratch;
    u64* tickets = t.scratch + t.scr_blocks;
    u64* gmeta = tickets + t.scr_blocks / 2;
    u64* rows = t.scratch + 2 * (u64)t.scr_blocks;  // SCR_ENTRIES words per workgroup (one word per entry)
    u64* grows = rows + (u64)t.scr_blocks * SCR_ENTRIES * sw;
    const u32 n_groups = (gridDim.x + SCR_GROUP - 1) / SCR_GROUP;
    const u32 g = blockIdx.x / SCR_GROUP;
    const u32 gsize = min((u32)SCR_GROUP, gridDim.x - g * SCR_GROUP);
    const u64 seq = ff.seq & ((1ULL << 44) - 1);
    if (threadIdx.x == 0) wg_ovf = 0;
    __syncthreads();
    // A table too large for a row goes to the HBM table before the ticket, so its claims and
    // possible overflow pushes ride on the ticket (uniform: lcount[0] is final).
    auto flush_if_large = [&]() -> bool {
        if (lcount[0] <= SCR_ENTRIES) return false;
        flush_lds_direct<true, false>(S, batches, B, lds, lds_slots, sw, nt, t, my_claims);
        my_ovf += threadIdx.x == 0 ? 1u : 0u;
        return true;
    };
    auto claims_and_ticket = [&](u64* ticket, u64 carried_claims, u64 carried_ovf) -> u64 {
        if (my_claims) atomicAdd(&lcount[1], my_claims);
        if (my_ovf) atomicAdd(&wg_ovf, my_ovf);
        my_claims = my_ovf = 0;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        u64 tk = 0;
        if (threadIdx.x == 0) {
            if (lcount[1]) {
                atomicAdd((unsigned long long*)(t.counters + CNT_CLAIMS), (unsigned long long)lcount[1]);
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            }
            const u64 add = 1 + ((carried_claims + lcount[1]) << 16) + ((carried_ovf + wg_ovf) << 40);
            tk = atomicAdd((unsigned long long*)ticket, (unsigned long long)add) + add;
        }
        return tk;
    };
    // park the LDS table as packed words (sc1), then post the entry count (sc1, after the drain)
    auto park_tagged = [&](u64* dst, u64* meta, int level) {
        if (threadIdx.x == 0) lcount[2] = 0;
        __syncthreads();
        for (u32 s = threadIdx.x; s < lds_slots; s += nt) {
            const u64* p = lds + (u64)s * sw;
            if (p[0] == SLOT_EMPTY) continue;
            const u32 k = atomicAdd(&lcount[2], 1u);
            st_sc1(dst + k, chain_pack(p[0], p[1], seq, level));
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (threadIdx.x == 0) st_sc1(meta, (seq << 20) | lcount[2]);
    };
    // an overflow record [key][count] (the host grows the table and finalizes again)
    auto push_kc = [&](u64 key, u64 c) {
        const u64 k = atomicAdd((unsigned long long*)(t.counters + CNT_OVF_RECS), 1ULL);
        if (k >= t.ovf_recs_cap) {
            atomicOr((unsigned long long*)(t.counters + CNT_ERR), (unsigned long long)ERR_OVF_LOST);
            return;
        }
        u64* r = t.ovf_recs + k * t.stride_words;
        r[0] = key;
        r[1] = c;
    };
    // item k of a parked row: spins until the row's count and (k < count) the entry are this
    // launch's; false = no entry k.  A spin that does not settle raises ERR_CHAIN_SPIN.
    auto read_item = [&](const u64* meta, const u64* row, u32 k, int level, u64& key, u64& cnt) -> bool {
        const int tb = level == 1 ? TAG1_BITS : TAG2_BITS;
        const u64 tag = seq & ((1ULL << tb) - 1);
        for (u32 it = 0; it < (1u << 22); ++it) {
            const u64 m = ld_sc1(meta);
            const u64 w = ld_sc1(row + k);
            if ((m >> 20) == seq) {
                if (k >= (m & 0xFFFFF)) return false;
                if ((w >> (64 - tb)) == tag) {
                    key = w & 0xFFFF;
                    cnt = (w << tb) >> (tb + 16);
                    return true;
                }
            }
            __builtin_amdgcn_s_sleep(1);
        }
        atomicOr((unsigned long long*)(t.counters + CNT_ERR), (unsigned long long)ERR_CHAIN_SPIN);
        bad = 1;
        return false;
    };
    // 1. ticket first; a workgroup that is not its group's last parks
    bool flushed = flush_if_large();
    {
        const u64 tk = claims_and_ticket(tickets + g, 0, 0);
        if (threadIdx.x == 0) {
            role = (tk & 0xFFFF) == gsize ? 1u : 0u;
            hbm_claims = (tk >> 16) & 0xFFFFFF;
            ovf_seen = tk >> 40;
            wg_ovf = 0;
            bad = 0;
        }
    }
    __syncthreads();
    if (!role) {
        if (flushed) {
            if (threadIdx.x == 0) st_sc1(counts + blockIdx.x, seq << 20);
        } else {
            park_tagged(rows + (u64)blockIdx.x * SCR_ENTRIES * sw, counts + blockIdx.x, 1);
        }
        return;
    }
    // 2. group leader: the members' rows merged into its own LDS table (emptied first when it went
    //    to the HBM table above); its level-1 claims are on the ticket already
    if (threadIdx.x == 0) {
        tickets[g] = 0;  // all members have added
        lcount[1] = 0;
        if (flushed) lcount[0] = 0;
    }
    if (flushed) lds_table_init(S, lds, lds_slots, sw, nt);
    __syncthreads();
    for (u32 f = threadIdx.x; f < gsize * SCR_ENTRIES; f += nt) {
        const u64 b = (u64)g * SCR_GROUP + f / SCR_ENTRIES;
        if (b == blockIdx.x) continue;
        u64 key, c;
        if (!read_item(counts + b, rows + b * SCR_ENTRIES * sw, f % SCR_ENTRIES, 1, key, c)) continue;
        const int ls = lds_find<true>(S, batches, B.keys, 0, key, 0, lds, lmask, sw, lcount, llimit);
        if (ls >= 0) {
            at_add<AS_LDS>(asp<AS_LDS>(lds + (u64)ls * sw + 1), c);
            continue;
        }
        bool claimed;
        const u64 gs = g_find<true>(S, batches, B.keys, 0, key, 0, t, t.probe_limit, claimed);
        if (gs == ~0ULL) {
            push_kc(key, c);
            my_ovf++;
            continue;
        }
        my_claims += claimed ? 1 : 0;
        at_add<AS_GLB>(asp<AS_GLB>(t.slots + gs * t.stride_words + 1), c);
    }
    __syncthreads();
    // 3. level 2: ticket first again; a leader that is not the last parks its group's table
    flushed = flush_if_large();
    {
        const u64 tk = claims_and_ticket(t.counters + CNT_FIN_TICKET, hbm_claims, ovf_seen);
        if (threadIdx.x == 0) {
            role = (tk & 0xFFFF) == n_groups ? 2u : 0u;
            hbm_claims = (tk >> 16) & 0xFFFFFF;
            ovf_seen = tk >> 40;
        }
    }
    __syncthreads();
    if (kPhaseTrace && ff.trace && threadIdx.x == 0) atomicMax((unsigned long long*)ff.trace + 3, (unsigned long long)__builtin_amdgcn_s_memrealtime());
    if (role != 2) {
        if (flushed) {
            if (threadIdx.x == 0) st_sc1(gmeta + g, seq << 20);
        } else {
            park_tagged(grows + (u64)g * SCR_ENTRIES * sw, gmeta + g, 2);
        }
        return;
    }
    // 4. the last leader: its own table into registers, the view of the HBM table, own entries
    //    and the other group rows merged into the view, finalize
    if (threadIdx.x == 0) {
        atomicExch((unsigned long long*)(t.counters + CNT_FIN_TICKET), 0ULL);
        atomicExch((unsigned long long*)(t.counters + CNT_TAIL), 0ULL);
        vcl = 0;
        if (kPhaseTrace && ff.trace) ff.trace[4] = __builtin_amdgcn_s_memrealtime();
    }
    u64 okey[OWN], ocnt[OWN];
#pragma unroll
    for (int j = 0; j < OWN; ++j) {
        const u32 s = threadIdx.x + (u32)j * nt;
        okey[j] = SLOT_EMPTY;
        ocnt[j] = 0;
        if (!flushed && s < lds_slots) {
            okey[j] = lds[(u64)s * sw];
            ocnt[j] = lds[(u64)s * sw + 1];
        }
    }
    __syncthreads();  // the view overwrites the table
    const u64 n = (t.cap + 1) * sw;  // host: <= the launch's dynamic LDS
    const bool hbm_clean = ff.table_empty && hbm_claims == 0;
    if (hbm_clean)  // COUNT(*) slots start [EMPTY][0]: no load of the Spec's initial slot
        for (u64 i = threadIdx.x; i < n; i += nt) lds[i] = (i % sw) == 0 ? SLOT_EMPTY : 0ULL;
    else
        for (u64 i = threadIdx.x; i < n; i += nt) lds[i] = ld_sc1(t.slots + i);
    __syncthreads();
    u32 vclaims = 0;
    auto to_view = [&](u64 key, u64 c) {
        u64 slot;
        if (view_find(lds, t, key, vclaims, slot)) {
            at_add<AS_LDS>(asp<AS_LDS>(lds + slot * sw + 1), c);
        } else {
            push_kc(key, c);
            bad = 1;
        }
    };
#pragma unroll
    for (int j = 0; j < OWN; ++j)
        if (okey[j] != SLOT_EMPTY) to_view(okey[j], ocnt[j]);
    for (u32 f = threadIdx.x; f < n_groups * SCR_ENTRIES; f += nt) {
        const u64 gg = f / SCR_ENTRIES;
        if (gg == g) continue;
        u64 key, c;
        if (read_item(gmeta + gg, grows + gg * SCR_ENTRIES * sw, f % SCR_ENTRIES, 2, key, c)) to_view(key, c);
    }
    if (vclaims) atomicAdd(&vcl, vclaims);
    __syncthreads();
    const bool known = ff.table_empty && ovf_seen == 0 && !bad;
    if (threadIdx.x == 0 && vcl && !known) {
        atomicAdd((unsigned long long*)(t.counters + CNT_CLAIMS), (unsigned long long)vcl);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    if (kPhaseTrace && ff.trace && threadIdx.x == 0) ff.trace[5] = __builtin_amdgcn_s_memrealtime();
    finalize_count_only<T>(t, lds, ff, known, vcl, hbm_clean && !bad);
    if (kPhaseTrace && ff.trace && threadIdx.x == 0) ff.trace[6] = __builtin_amdgcn_s_memrealtime();
}

// ------------------------------------------------------------------------------------------
// agg_insert_fast: one non-null integer key column, optional `key <cmp> constant` predicate on
// that same column (GROUP BY x WHERE x <> c: ClickBench Q8; or no predicate: Q16).  Streams the
// key column with 16-byte loads (FAST_UNROLL per lane per grid round, the next round's issued
// before this one is filtered), evaluates the predicate on every value, and stages the selected
// rows in the LDS table exactly like agg_insert.
// ------------------------------------------------------------------------------------------
#ifndef FAST_UNROLL
// 16-byte loads per lane and round: C2 kernel (200 steps, three alternating rounds,
// scripts/gpu_c2_variants.sh) 1 / 2 / 3 / 4 / 8 -> 45.5 / 40.6 / 41.9 / 43.4 / 55 us: two rounds
// of two in flight keep each wave's window of the column to 2 x 2 grid strides
#define FAST_UNROLL 2
#endif
#ifndef TAIL_ON
// dynamic stream tail of fused-chain launches: measured and not kept (C2 step 45.7 -> 51.3 us,
// profiles/r04/c2_tail_ab.json); make TAIL=1 builds it for A/B runs
#define TAIL_ON 0
#endif
typedef unsigned int v4u __attribute__((ext_vector_type(4)));
// Column data reached through a descriptor is a generic pointer to the compiler, which then
// emits flat loads: those count against lgkmcnt too and retire out of order, so every LDS wait
// (and every use of a loaded value) drains ALL loads in flight and the prefetch pipeline
// collapses.  Streams read through this address-space-1 view compile to global_load.
typedef const v4u __attribute__((address_space(1)))* gv4p;

template <typename T>
__device__ __forceinline__ bool fast_pred(T v, int op, i64 c) {
    // the constant is in the column's domain (signed / unsigned by T)
    T k = (T)c;
    switch (op) {
        case DBG_CMP_EQ: return v == k;
        case DBG_CMP_NE: return v != k;
        case DBG_CMP_LT: return v < k;
        case DBG_CMP_LE: return v <= k;
        case DBG_CMP_GT: return v > k;
        default: return v >= k;
    }
}

// Element j of a 16-byte vector viewed as T[16 / sizeof(T)], from registers (no address taken).
template <typename T>
__device__ __forceinline__ T vget(const v4u& y, int j) {
    constexpr int W = sizeof(T);
    if constexpr (W == 8) {
        u32 lo = j ? y.z : y.x, hi = j ? y.w : y.y;
        return (T)(((u64)hi << 32) | lo);
    } else {
        int wi = (j * W) >> 2;
        u32 word = wi == 0 ? y.x : (wi == 1 ? y.y : (wi == 2 ? y.z : y.w));
        return (T)(word >> (((j * W) & 3) * 8));
    }
}

// Selected rows are appended to a per-wave LDS queue (ballot + mbcnt) and staged 64 at a time
// with every lane active: at low selectivity (Q8: 0.63 %) a lane-divergent insert per row would
// leave 63 of 64 lanes idle on every LDS round trip.
#define WQ 128  // queue entries per wave
#define WQW 384  // u64 words of per-wave queue space: rows (2 x WQ) or candidate vectors (WQ x (16 + 8) B)

template <typename T, bool PRED, int NT, bool CO>
__global__ void __launch_bounds__(NT) agg_insert_fast_kernel(const Spec* __restrict__ spec, const BatchDesc* __restrict__ batches,
                                                               u32 bid, u64 rows, TableDesc t, u32 lds_slots,
                                                               T lo, T hi, int negate, FusedFin ff) {
    extern __shared__ __attribute__((aligned(16))) u64 lds[];
    constexpr int V = 16 / sizeof(T);
    const Spec& S = *spec;
    const BatchDesc& B = batches[bid];
    const T* __restrict__ col = (const T*)B.keys[0].data;
    const u32 sw = S.stride_words;
    u32* lcount = (u32*)(lds + (u64)lds_slots * sw);
    const u32 lmask = lds_slots - 1;
    const u32 llimit = lds_slots - lds_slots / 4;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    // per-wave queue (keys and rows) after the table and its 16 bytes of counters
    u64* qkey = lds + (u64)lds_slots * sw + 2 + (u64)wave * WQW;
    u64* qrow = qkey + WQ;
    // candidate-vector queue (the `<> c` path below) over the same per-wave space
    v4u* vq = (v4u*)qkey;
    u64* vqb = qkey + 2 * WQ;
    if (kPhaseTrace && ff.trace && threadIdx.x == 0) atomicMin((unsigned long long*)ff.trace, (unsigned long long)__builtin_amdgcn_s_memrealtime());
    lds_table_init(S, lds, lds_slots, sw, NT);
    if (threadIdx.x < 4) lcount[threadIdx.x] = 0;
    __syncthreads();
    u32 my_claims = 0;
    u32 my_ovf = 0;  // overflow rows pushed (the fused chain reports them through its tickets)

    // predicate in range form: lo <= v <= hi, xor negate (host maps =, <>, <, <=, >, >=)
    auto pass = [&](T v) -> bool { return ((v >= lo) & (v <= hi)) ^ (negate != 0); };

    // stage one selected row (key bits, row index) — all callers have full or near-full lanes
    auto process = [&](u64 key, u64 i) {
        int ls = lds_find<true>(S, batches, nullptr, i, key, 0, lds, lmask, sw, lcount, llimit);
        if (ls >= 0) {
            wptr<AS_LDS> st = asp<AS_LDS>(lds + (u64)ls * sw);
            if (CO) at_add<AS_LDS>(st + 1, 1ULL);
            else apply_row<AS_LDS>(S, st, B, i);
            return;
        }
        bool claimed;
        u64 gs = g_find<true>(S, batches, nullptr, i, key, 0, t, t.probe_limit, claimed);
        if (gs == ~0ULL) {
            push_ovf_row(t, bid, i);
            my_ovf++;
            return;
        }
        my_claims += claimed ? 1 : 0;
        wptr<AS_GLB> gst = asp<AS_GLB>(t.slots + gs * t.stride_words);
        if (CO) at_add<AS_GLB>(gst + 1, 1ULL);
        else apply_row<AS_GLB>(S, gst, B, i);
    };

    u32 qn = 0;  // wave-uniform queue length
    auto drain64 = [&]() {  // process entries [0, 64), shift [64, qn) down
        vwptr<AS_LDS> qk = (vwptr<AS_LDS>)qkey, qr = (vwptr<AS_LDS>)qrow;
        u64 k = qk[lane], r = qr[lane];
        u64 k2 = 0, r2 = 0;
        bool mv = lane + 64 < (int)qn;
        if (mv) {
            k2 = qk[lane + 64];
            r2 = qr[lane + 64];
        }
        __builtin_amdgcn_wave_barrier();
        if (mv) {
            qk[lane] = k2;
            qr[lane] = r2;
        }
        __builtin_amdgcn_wave_barrier();
        qn -= 64;
        process(k, r);
    };

    // `key <> c` (ClickBench Q8: AdvEngineID <> 0) as a two-level compaction.  A row-level
    // queue pays the per-row mask + ballot-prefix VALU work on every lane (SQ counters: ~350
    // VALU per 32-row round, VALU ~60 % busy); instead each 16-byte vector is tested whole —
    // "some element differs from c" is three ORs of XORs — and only candidate vectors (4.9 % at
    // Q8's selectivity) are appended, whole, to a per-wave LDS queue; 64 at a time they are
    // expanded with every lane busy.  ~10 VALU per 8-row vector instead of ~90.
    const bool neq_fast = PRED && negate && lo == hi;
    u32 cc_lo, cc_hi;
    {
        typedef typename std::make_unsigned<T>::type UT;
        const u64 c = (u64)(UT)lo;
        if (sizeof(T) == 8) { cc_lo = (u32)c; cc_hi = (u32)(c >> 32); }
        else if (sizeof(T) == 4) { cc_lo = cc_hi = (u32)c; }
        else if (sizeof(T) == 2) { cc_lo = cc_hi = (u32)(c | (c << 16)); }
        else { cc_lo = cc_hi = (u32)(c * 0x01010101u); }
    }
    u32 vqn = 0;  // wave-uniform candidate count
    // expand candidate vectors [0, n) (n <= 64, one per lane), shift [64, vqn) down
    auto drain_vec = [&](u32 n) {
        v4u v = {0, 0, 0, 0};
        u64 bs = 0;
        const bool have = lane < (int)n;
        if (have) {
            v = ((volatile v4u*)vq)[lane];
            bs = ((volatile u64*)vqb)[lane];
        }
        const bool mv = lane + 64 < (int)vqn;
        v4u v2 = {0, 0, 0, 0};
        u64 b2 = 0;
        if (mv) {
            v2 = ((volatile v4u*)vq)[lane + 64];
            b2 = ((volatile u64*)vqb)[lane + 64];
        }
        __builtin_amdgcn_wave_barrier();
        if (mv) {
            ((volatile v4u*)vq)[lane] = v2;
            ((volatile u64*)vqb)[lane] = b2;
        }
        __builtin_amdgcn_wave_barrier();
        vqn -= n;
        u32 mm = 0;
        if (have)
#pragma unroll
            for (int j = 0; j < V; ++j) mm |= (pass(vget<T>(v, j)) ? 1u : 0u) << j;
        while (mm) {
            const int j = __builtin_ctz(mm);
            mm &= mm - 1;
            // element j of v from registers (j is lane-varying here): select over the dwords
            const int W = (int)sizeof(T);
            const int wi = (j * W) >> 2;
            const u32 w0 = wi == 0 ? v.x : (wi == 1 ? v.y : (wi == 2 ? v.z : v.w));
            u64 key;
            if (W == 8) {
                const u32 w1 = wi == 0 ? v.y : v.w;
                key = ((u64)w1 << 32) | w0;
            } else {
                const u32 sh = (u32)((j * W) & 3) * 8;
                key = (u64)((w0 >> sh) & (W == 4 ? 0xFFFFFFFFu : ((1u << (8 * W)) - 1u)));
            }
            process(key, bs + j);
        }
    };
    const u64 ltmask = (1ULL << lane) - 1;
    auto key_of = [&](const v4u& y, int j) -> u64 { return (u64)(typename std::make_unsigned<T>::type)vget<T>(y, j); };
    // Stage the selected rows of a group of NV vectors (one per lane and slot u), all lanes
    // together.  A lane's vector slots hold rows base[u] .. base[u] + V - 1.
    auto handle_group = [&](const v4u* y, const u64* base, int nv, u32 actm) {
        if (!PRED) {
            for (int u = 0; u < nv; ++u)
                if ((actm >> u) & 1)
#pragma unroll
                    for (int j = 0; j < V; ++j) process(key_of(y[u], j), base[u] + j);
            return;
        }
        if (neq_fast) {
#pragma unroll
            for (int u = 0; u < FAST_UNROLL; ++u) {
                const v4u& v = y[u];
                const bool any = (((v.x ^ cc_lo) | (v.y ^ cc_hi) | (v.z ^ cc_lo) | (v.w ^ cc_hi)) != 0) && ((actm >> u) & 1);
                const u64 b = __ballot(any);
                if (b == 0) continue;
                if (any) {
                    const u32 pos = vqn + (u32)__popcll(b & ltmask);
                    vq[pos] = v;
                    vqb[pos] = base[u];
                }
                vqn += (u32)__popcll(b);
                if (vqn >= 64) {
                    __builtin_amdgcn_wave_barrier();
                    drain_vec(64);
                }
            }
            return;
        }
        u32 m[FAST_UNROLL];
        u32 cnt = 0;
#pragma unroll
        for (int u = 0; u < FAST_UNROLL; ++u) {
            m[u] = 0;
            if (u < nv) {
#pragma unroll
                for (int j = 0; j < V; ++j) m[u] |= (pass(vget<T>(y[u], j)) ? 1u : 0u) << j;
            }
            if (!((actm >> u) & 1)) m[u] = 0;
            cnt += __popc(m[u]);
        }
        if (__ballot(cnt != 0) == 0) return;
        // exclusive prefix and wave total of cnt (<= 32 = 6 bits) from one ballot per bit
        u32 pre = 0, tot = 0;
#pragma unroll
        for (int bb = 0; bb < 6; ++bb) {
            u64 bal = __ballot((cnt >> bb) & 1);
            pre += (u32)__popcll(bal & ltmask) << bb;
            tot += (u32)__popcll(bal) << bb;
        }
        if (qn + tot <= WQ) {
            u32 pos = qn + pre;
#pragma unroll
            for (int u = 0; u < FAST_UNROLL; ++u) {
                u32 mm = m[u];
                while (mm) {
                    int j = __builtin_ctz(mm);
                    mm &= mm - 1;
                    qkey[pos] = key_of(y[u], j);
                    qrow[pos] = base[u] + j;
                    pos++;
                }
            }
            qn += tot;
            while (qn >= 64) {
                __builtin_amdgcn_wave_barrier();
                drain64();
            }
        } else {  // dense selection: lanes already busy, insert directly
#pragma unroll
            for (int u = 0; u < FAST_UNROLL; ++u) {
                u32 mm = m[u];
                while (mm) {
                    int j = __builtin_ctz(mm);
                    mm &= mm - 1;
                    process(key_of(y[u], j), base[u] + j);
                }
            }
        }
    };

    // Grid-strided stream (all waves of the chip sweep one window of the column together: DRAM
    // rows stay open, scripts/micro/stream.hip): FAST_UNROLL unconditional 16-byte loads per lane
    // per round (an index past the end is clamped and its lane-slot masked off), so no branch
    // sits around the loads; other waves of the CU keep HBM busy while one filters.  The loop
    // condition is wave-uniform (ballot) because the queue needs all 64 lanes.
    const u64 nvec = rows / V;
    gv4p vp = (gv4p)col;
    const u64 gstride = (u64)gridDim.x * NT;
    u64 k = (u64)blockIdx.x * NT + threadIdx.x;
    const u64 step = (u64)FAST_UNROLL * gstride;
    const u64 lastv = nvec ? nvec - 1 : 0;
    // Dynamic tail (fused-chain launches): the grid-strided static part covers ~80 % of the
    // vectors in whole rounds of the grid; the rest is cut into chunks of NT x FAST_UNROLL vectors
    // that workgroups done with their static share take from a device counter — so the chip's
    // fast CUs absorb the end of the stream instead of waiting for its slow ones (workgroups
    // finished streaming between 27.8 and 35.0 us of a C2 launch).  The counter
    // (CNT_TAIL) is reset by the launch's last group leader.
    constexpr u64 TAIL_CH = (u64)NT * FAST_UNROLL;
    const bool dyn = TAIL_ON && ff.on && t.scratch != nullptr && gridDim.x > 1 && gridDim.x <= t.scr_blocks;
    u64 nstat = nvec, nch = 0;
    if (dyn) {
        nstat = ((nvec * 4 / 5) / step) * step;
        nch = (nvec - nstat + TAIL_CH - 1) / TAIL_CH;
    }
    u64 tail_grab = 0;  // thread 0: the first tail chunk, taken now (its latency hides behind the stream)
    if (dyn && nch && threadIdx.x == 0) tail_grab = atomicAdd((unsigned long long*)(t.counters + CNT_TAIL), 1ULL);
    // Software pipeline: the next round's FAST_UNROLL loads are issued before this round is
    // filtered and queued, so a wave busy with its ballots and LDS queue writes still has
    // 64 B/lane in flight (without it the per-round processing sits on the load critical path).
    v4u y[FAST_UNROLL];
#pragma unroll
    for (int u = 0; u < FAST_UNROLL; ++u) {
        u64 idx = k + u * gstride;
        y[u] = __builtin_nontemporal_load(vp + (idx < nstat ? idx : lastv));
    }
    while (__ballot(k < nstat) != 0) {
        const u64 kn = k + step;
        v4u yn[FAST_UNROLL];
#pragma unroll
        for (int u = 0; u < FAST_UNROLL; ++u) {
            u64 idx = kn + u * gstride;
            yn[u] = __builtin_nontemporal_load(vp + (idx < nstat ? idx : lastv));
        }
        u64 bases[FAST_UNROLL];
        u32 actm = 0;
#pragma unroll
        for (int u = 0; u < FAST_UNROLL; ++u) {
            u64 idx = k + u * gstride;
            actm |= (idx < nstat ? 1u : 0u) << u;
            bases[u] = idx * V;
        }
        handle_group(y, bases, FAST_UNROLL, actm);
#pragma unroll
        for (int u = 0; u < FAST_UNROLL; ++u) y[u] = yn[u];
        k = kn;
    }
    if (dyn && nch) {
        // chunk ids pass through LDS behind a bare s_barrier (no fence: the loads in flight are
        // not drained); the next chunk's loads are issued, and the chunk after it taken, before
        // the current chunk is filtered
        __shared__ u32 tail_id[2];
        auto load_chunk = [&](u32 c, v4u* yy) {
#pragma unroll
            for (int u = 0; u < FAST_UNROLL; ++u) {
                const u64 idx = nstat + (u64)c * TAIL_CH + (u64)u * NT + threadIdx.x;
                yy[u] = __builtin_nontemporal_load(vp + (idx < nvec ? idx : lastv));
            }
        };
        auto publish = [&](u32 slot, u64 v) -> u32 {
            if (threadIdx.x == 0) tail_id[slot] = (u32)min<u64>(v, nch);
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            __builtin_amdgcn_s_barrier();
            return tail_id[slot];
        };
        u32 par = 0;
        u32 cur = publish(par, tail_grab);
        par ^= 1;
        v4u yc[FAST_UNROLL];
        if (cur < nch) {
            load_chunk(cur, yc);
            if (threadIdx.x == 0) tail_grab = atomicAdd((unsigned long long*)(t.counters + CNT_TAIL), 1ULL);
        }
        while (cur < nch) {
            const u32 nxt = publish(par, tail_grab);
            par ^= 1;
            v4u yn[FAST_UNROLL];
            if (nxt < nch) {
                load_chunk(nxt, yn);
                if (threadIdx.x == 0) tail_grab = atomicAdd((unsigned long long*)(t.counters + CNT_TAIL), 1ULL);
            }
            u64 bases[FAST_UNROLL];
            u32 actm = 0;
#pragma unroll
            for (int u = 0; u < FAST_UNROLL; ++u) {
                const u64 idx = nstat + (u64)cur * TAIL_CH + (u64)u * NT + threadIdx.x;
                actm |= (idx < nvec ? 1u : 0u) << u;
                bases[u] = idx * V;
            }
            handle_group(yc, bases, FAST_UNROLL, actm);
#pragma unroll
            for (int u = 0; u < FAST_UNROLL; ++u) yc[u] = yn[u];
            cur = nxt;
        }
    }
    if (PRED && vqn) {
        __builtin_amdgcn_wave_barrier();
        drain_vec(vqn);
    }
    // drain the queue's rest (< 64 entries): lanes below qn take one each
    if (PRED && qn) {
        __builtin_amdgcn_wave_barrier();
        if (lane < (int)qn) process(((vwptr<AS_LDS>)qkey)[lane], ((vwptr<AS_LDS>)qrow)[lane]);
        qn = 0;
    }
    for (u64 i = nvec * V + (u64)blockIdx.x * NT + threadIdx.x; i < rows; i += gstride) {
        T v = gld<T>(col + i);
        if (!PRED || pass(v)) process((u64)(typename std::make_unsigned<T>::type)v, i);
    }
    __syncthreads();
    if (kPhaseTrace && ff.trace && threadIdx.x == 0) {
        const u64 tm = __builtin_amdgcn_s_memrealtime();
        atomicMin((unsigned long long*)ff.trace + 1, (unsigned long long)tm);
        atomicMax((unsigned long long*)ff.trace + 2, (unsigned long long)tm);
    }
    if constexpr (CO && sizeof(T) <= 2) {
        if (ff.on && ff.dense && t.scratch != nullptr && gridDim.x > 1 && gridDim.x < 65536) {
            fused_dense<T>(S, batches, B, lds, lds_slots, sw, lcount, NT, t, my_claims, my_ovf, ff);
            return;
        }
    }
    if (ff.on && t.scratch != nullptr && gridDim.x > 1 && gridDim.x <= t.scr_blocks) {
        if constexpr (CO && sizeof(T) <= 2) {
            if (kChainTagged && lds_slots <= 4 * NT) {
                fused_chain_tagged<T>(S, batches, B, lds, lds_slots, sw, lcount, NT, t, my_claims, my_ovf, ff);
                return;
            }
        }
        fused_chain<T, CO>(S, batches, B, lds, lds_slots, sw, lcount, NT, t, my_claims, my_ovf, ff);
        return;
    }
    block_flush<true, false>(S, batches, B, lds, lds_slots, sw, lcount, NT, t, my_claims);
    if (kPhaseTrace && ff.trace && threadIdx.x == 0) atomicMax((unsigned long long*)ff.trace + 3, (unsigned long long)__builtin_amdgcn_s_memrealtime());
    if (ff.on) fused_finalize(S, batches, t, lds, ff);
}


bool prof_ext_events(hipEvent_t* a, hipEvent_t* b);  // abi.hip

static size_t fast_shmem(size_t table_bytes) { return table_bytes + (size_t)(1024 / 64) * WQW * 8; }
static size_t fast_table_bytes(const Spec& S) { return (size_t)lds_slots_for(S, 16 * 1024) * S.stride_words * 8 + 16; }

template <typename T>
static void launch_fast_t(hipStream_t s, const Spec* dspec, const BatchDesc* batches, u32 bid, u64 rows, const TableDesc& t,
                          u32 lslots, size_t table_bytes, bool pred, int op, i64 c, int count_only, const FusedFin* fused) {
    constexpr u64 V = 16 / sizeof(T);
    // `v <op> c` as `(lo <= v <= hi) ^ negate`, exact over T's range (constants outside it fold)
    typedef __int128 W;
    const W tmin = (W)std::numeric_limits<T>::min(), tmax = (W)std::numeric_limits<T>::max();
    const W C = std::is_signed<T>::value ? (W)c : (W)(u64)c;
    W lo = 1, hi = 0;  // empty range
    int neg = 0;
    auto all = [&]() { lo = tmin; hi = tmax; };
    switch (op) {
        case DBG_CMP_EQ: if (C >= tmin && C <= tmax) lo = hi = C; break;
        case DBG_CMP_NE: neg = 1; if (C >= tmin && C <= tmax) lo = hi = C; break;
        case DBG_CMP_LT: if (C > tmax) all(); else if (C > tmin) { lo = tmin; hi = C - 1; } break;
        case DBG_CMP_LE: if (C >= tmax) all(); else if (C >= tmin) { lo = tmin; hi = C; } break;
        case DBG_CMP_GT: if (C < tmin) all(); else if (C < tmax) { lo = C + 1; hi = tmax; } break;
        default: if (C <= tmin) all(); else if (C <= tmax) { lo = C; hi = tmax; } break;  // GE
    }
    if (lo > hi) { lo = 1; hi = 0; }  // stays empty in T (1 > 0 for every T)
    const int nt = 1024;
    static_assert(FIN_NT == 1024, "the fused finalize runs on the insert's workgroup");
    // one 1024-lane workgroup per CU (parked-row chain: 512 / 768 / 1024 / 2048 measured 52 / 55 / 63
    // / 90 us a C2 step); EXPERIMENT DBG_X_FAST_GRID for the dense hand-off, whose merge does not
    // grow with the grid
    static const u64 x_grid = X_ENV("DBG_X_FAST_GRID") ? (u64)atoll(X_ENV("DBG_X_FAST_GRID")) : 0;
    const u64 max_blocks = (x_grid && fused && fused->dense) ? x_grid : 256;
    size_t shmem = fast_shmem(table_bytes);
    FusedFin ff;
    if (fused) ff = *fused;
    else memset(&ff, 0, sizeof(ff));
    u64 quantum = V * (u64)nt * FAST_UNROLL;
    u64 blocks = (rows + quantum - 1) / quantum;
    if (blocks > max_blocks) blocks = max_blocks;
    if (blocks > DBG_INSERT_MAX_BLOCKS) blocks = DBG_INSERT_MAX_BLOCKS;
    if (blocks < 1) blocks = 1;
    // profiling on: the kernel stamps the enclosing scope's events itself (abi.hip, prof_ext_events)
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    const bool ext = prof_ext_events(&ev0, &ev1);
#define FAST_LAUNCH(P, N, F)                                                                                                     \
    do {                                                                                                                         \
        if (ext)                                                                                                                 \
            hipExtLaunchKernelGGL((agg_insert_fast_kernel<T, P, N, F>), dim3((u32)blocks), dim3(N), shmem, s, ev0, ev1, 0, dspec, \
                                  batches, bid, rows, t, lslots, (T)lo, (T)hi, neg, ff);                                        \
        else                                                                                                                     \
            hipLaunchKernelGGL((agg_insert_fast_kernel<T, P, N, F>), dim3((u32)blocks), dim3(N), shmem, s, dspec, batches, bid, \
                               rows, t, lslots, (T)lo, (T)hi, neg, ff);                                                          \
    } while (0)
    // CO: COUNT(*) is the only aggregate (ClickBench Q8/Q16 shape) — the kernel then carries no
    // apply_row code at all (smaller hot loop, fewer registers)
    if (count_only) {
        if (pred) FAST_LAUNCH(true, 1024, true); else FAST_LAUNCH(false, 1024, true);
    } else {
        if (pred) FAST_LAUNCH(true, 1024, false); else FAST_LAUNCH(false, 1024, false);
    }
#undef FAST_LAUNCH
}

// Host-side eligibility for the fast path (hb = host copy of the batch descriptor).
static bool fast_eligible(const Spec& S, const BatchDesc& hb, bool records) {
    if (records || !S.inline_keys || S.n_keys != 1 || S.key_types[0].nullable) return false;
    const DCol& k = hb.keys[0];
    int ty = k.type;
    bool intlike = (ty >= DBG_INT8 && ty <= DBG_UINT64) || ty == DBG_DATE || ty == DBG_TIMESTAMP;
    if (!intlike || k.layout != LAYOUT_ARROW || ((uintptr_t)k.data & 15)) return false;
    if (hb.n_nodes == 0) return true;
    if (hb.n_nodes != 1) return false;
    const DNode& n = hb.nodes[0];
    const DCol& f = hb.fcols[n.col];
    return n.op == DBG_PRED_CMP_CONST && f.data == k.data && f.type == ty && !f.nullable;
}

bool insert_can_fuse(const Spec& S, const BatchDesc& hb, u64 cap) {
    return hb.rows > 0 && fast_eligible(S, hb, false) && cap + 1 <= FUSED_FIN_SLOTS &&
           (cap + 1) * S.stride_words * 8 <= fast_shmem(fast_table_bytes(S));
}

void launch_insert(hipStream_t s, const Spec* dspec, const Spec& S, const BatchDesc* batches, u32 bid, u64 rows, bool records,
                   const TableDesc& t, bool use_lds, const BatchDesc* hb, const FusedFin* fused) {
    if (rows == 0) return;
    if (hb && use_lds && fast_eligible(S, *hb, records)) {
        u32 lslots = lds_slots_for(S, 16 * 1024);
        size_t shmem = fast_table_bytes(S);
        bool pred = hb->n_nodes == 1;
        int op = pred ? hb->nodes[0].cmp : 0;
        i64 c = pred ? hb->nodes[0].i64v : 0;
        int count_only = S.n_aggs == 1 && S.aggs[0].kind == DBG_AGG_COUNT && S.aggs[0].arg_type < 0 && S.aggs[0].w0 == 1;
        switch (hb->keys[0].type) {
            case DBG_INT8: launch_fast_t<int8_t>(s, dspec, batches, bid, rows, t, lslots, shmem, pred, op, c, count_only, fused); return;
            case DBG_UINT8: launch_fast_t<uint8_t>(s, dspec, batches, bid, rows, t, lslots, shmem, pred, op, c, count_only, fused); return;
            case DBG_INT16: launch_fast_t<int16_t>(s, dspec, batches, bid, rows, t, lslots, shmem, pred, op, c, count_only, fused); return;
            case DBG_UINT16: launch_fast_t<uint16_t>(s, dspec, batches, bid, rows, t, lslots, shmem, pred, op, c, count_only, fused); return;
            case DBG_INT32: case DBG_DATE: launch_fast_t<int32_t>(s, dspec, batches, bid, rows, t, lslots, shmem, pred, op, c, count_only, fused); return;
            case DBG_UINT32: launch_fast_t<uint32_t>(s, dspec, batches, bid, rows, t, lslots, shmem, pred, op, c, count_only, fused); return;
            case DBG_INT64: case DBG_TIMESTAMP: launch_fast_t<int64_t>(s, dspec, batches, bid, rows, t, lslots, shmem, pred, op, c, count_only, fused); return;
            case DBG_UINT64: launch_fast_t<uint64_t>(s, dspec, batches, bid, rows, t, lslots, shmem, pred, op, c, count_only, fused); return;
        }
    }
    // one non-null String key into a large key-caching table, filtered by `key <op> ''` or not
    if (!records && use_lds && hb && S.kc_word && t.cap + 1 > SHORT_MAX_SLOTS && str1_eligible(S, *hb, rows)) {
        const u32 lsw = (u32)S.kc_word + 1 + KC_KEY_WORDS;
        static const u32 x_mode = X_ENV("DBG_X_STR1") ? (u32)atoi(X_ENV("DBG_X_STR1")) : 0;
        static const u32 x_lds = X_ENV("DBG_X_STR1_LDS") ? (u32)atoi(X_ENV("DBG_X_STR1_LDS")) * 1024 : STR1_LDS_BUDGET;
        static const u32 fper = X_ENV("DBG_X_STR1_FLUSH") ? (u32)atoi(X_ENV("DBG_X_STR1_FLUSH")) : 4;
        u32 ls = 1;
        while ((ls * 2) * lsw * 8 <= x_lds) ls *= 2;
        const size_t shmem = (size_t)ls * lsw * 8 + 32 + (size_t)STR1_QCAP * 8;
        u64 blocks = (rows + (u64)STR1_NT * 16 - 1) / ((u64)STR1_NT * 16);
        if (blocks > DBG_INSERT_MAX_BLOCKS) blocks = DBG_INSERT_MAX_BLOCKS;
        if (blocks < 1) blocks = 1;
        u64 rpb = ((rows + blocks - 1) / blocks + 1) & ~1ULL;  // even: 16-B offset loads
        blocks = (rows + rpb - 1) / rpb;
        if (hb->n_nodes) hipLaunchKernelGGL(agg_insert_str1_kernel<true>, dim3((u32)blocks), dim3(STR1_NT), shmem, s, dspec, batches, bid, rows, rpb, t, ls, fper, x_mode);
        else hipLaunchKernelGGL(agg_insert_str1_kernel<false>, dim3((u32)blocks), dim3(STR1_NT), shmem, s, dspec, batches, bid, rows, rpb, t, ls, fper, x_mode);
        return;
    }
    u32 lslots = use_lds ? lds_slots_for(S, LDS_BUDGET_BYTES) : 1;
    static const int x_short = X_ENV("DBG_X_SHORT") ? atoi(X_ENV("DBG_X_SHORT")) : 1;
    static const u32 x_rep = X_ENV("DBG_X_SHORT_REP") ? (u32)atoi(X_ENV("DBG_X_SHORT_REP")) : 0;
    const bool x_noshort = x_short == 0;
    // low cardinality only: with a table already sized for many groups (the cardinality probe, or
    // earlier batches) most rows miss the workgroup's LDS table, and the generic kernel's queued
    // HBM path serves those far better than this kernel's per-row fallback (C5: 31 vs 95 ms)
    if (!records && use_lds && hb && !x_noshort && t.cap + 1 <= SHORT_MAX_SLOTS && short_eligible(S, *hb)) {
        u64 blocks = (rows + (u64)BLOCK * 16 - 1) / ((u64)BLOCK * 16);
        static const u64 x_blocks = X_ENV("DBG_X_SHORT_BLOCKS") ? (u64)atoll(X_ENV("DBG_X_SHORT_BLOCKS")) : 0;
        if (x_blocks) blocks = x_blocks;  // EXPERIMENT: grid size
        if (blocks > DBG_INSERT_MAX_BLOCKS) blocks = DBG_INSERT_MAX_BLOCKS;
        if (blocks < 1) blocks = 1;
        u64 rpb = (rows + blocks - 1) / blocks;
        blocks = (rows + rpb - 1) / rpb;
        const size_t shmem = (size_t)lslots * S.stride_words * 8 + 32 + (size_t)lslots * 16;
        // narrow Decimal sums: rows_per_block * 10^p < 2^63 (a workgroup's partial fits in i64)
        u32 narrow = 0;
        for (int a = 0; a < S.n_aggs; ++a) {
            const DAgg& A = S.aggs[a];
            if (A.sumk != SUMK_I128 || A.kind == DBG_AGG_COUNT || A.arg_type != DBG_DECIMAL128) continue;
            const int p = hb->args[a].precision;
            double lim = 1.0;
            for (int k = 0; k < p; ++k) lim *= 10.0;
            if (p > 0 && p <= 18 && lim * (double)rpb < 9.0e18) narrow |= 1u << a;
        }
        static const bool x_wide = X_ENV("DBG_X_NARROW") && X_ENV("DBG_X_NARROW")[0] == '0';
        if (x_wide) narrow = 0;
        static const bool x_tree = X_ENV("DBG_X_TREE") && X_ENV("DBG_X_TREE")[0] == '1';
        u64* x_tr = nullptr;
        if (kPhaseTrace && X_ENV("DBG_X_TRACE_SHORT")) {  // EXPERIMENT: 8 words per launch, 4096 launches
            static u64* buf = nullptr;
            static u32 launch = 0;
            static const u64 init[8] = {~0ULL, ~0ULL, 0, 0, 0, 0, 0, 0};
            if (!buf) {
                if (hipMalloc((void**)&buf, 4096 * 64) != hipSuccess) buf = nullptr;
                if (buf) hipMemset(buf, 0, 4096 * 64);
                atexit([] {
                    std::vector<u64> hb(4096 * 8);
                    (void)hipDeviceSynchronize();
                    (void)hipMemcpy(hb.data(), buf, hb.size() * 8, hipMemcpyDeviceToHost);
                    std::vector<std::vector<double>> d(4);
                    for (int k = 0; k < 4096; ++k) {
                        const u64* r = &hb[k * 8];
                        if (r[0] == 0 || r[0] == ~0ULL || r[4] == 0) continue;
                        for (int p = 1; p <= 4; ++p) d[p - 1].push_back((double)(r[p] - r[0]) * 0.01);
                    }
                    const char* nm[] = {"first row loop end", "last row loop end", "last flush start", "last workgroup end"};
                    for (int p = 0; p < 4; ++p) {
                        if (d[p].empty()) continue;
                        std::sort(d[p].begin(), d[p].end());
                        fprintf(stderr, "short trace %-20s median %7.2f us  (n=%zu)\n", nm[p], d[p][d[p].size() / 2], d[p].size());
                    }
                });
            }
            if (buf) {
                x_tr = buf + (u64)(launch++ & 4095) * 8;
                (void)hipMemcpyAsync(x_tr, init, sizeof(init), hipMemcpyHostToDevice, s);
            }
        }
        hipLaunchKernelGGL(agg_insert_short_kernel, dim3((u32)blocks), dim3(BLOCK), shmem, s, dspec, batches, bid, rows, rpb, t, lslots,
                           x_rep ? x_rep - 1 : 0u, x_short, narrow, x_tree && S.stride_words >= S.n_words + 3 ? 1 : 0, x_tr);
        return;
    }
    // enough workgroups to fill 256 CUs several times over, each a contiguous row range
    u64 min_rows_per_block = (u64)BLOCK * 16;
    u64 blocks = (rows + min_rows_per_block - 1) / min_rows_per_block;
    if (blocks > DBG_INSERT_MAX_BLOCKS) blocks = DBG_INSERT_MAX_BLOCKS;
    if (blocks < 1) blocks = 1;
    u64 rpb = (rows + blocks - 1) / blocks;
    blocks = (rows + rpb - 1) / rpb;
    size_t shmem = (size_t)lslots * S.stride_words * 8 + 16;
    // `string <op> ''` filter (one node on a non-null arrow String column): the kernel's
    // multi-round queue (5 rounds of BLOCK row indices) after the table
    u32 lenq = 0;
    if (hb && !records && hb->n_nodes == 1 && hb->nodes[0].op == DBG_PRED_CMP_CONST && hb->nodes[0].str_len == 0) {
        const DCol& c = hb->fcols[hb->nodes[0].col];
        if (c.type == DBG_STRING && !c.nullable && c.layout == LAYOUT_ARROW) lenq = 5 * BLOCK;
    }
    shmem += (size_t)lenq * 4;
    if (S.inline_keys) {
        if (records) hipLaunchKernelGGL((agg_insert_kernel<true, true>), dim3((u32)blocks), dim3(BLOCK), shmem, s, dspec, batches, bid, rows, rpb, t, lslots, lenq);
        else hipLaunchKernelGGL((agg_insert_kernel<true, false>), dim3((u32)blocks), dim3(BLOCK), shmem, s, dspec, batches, bid, rows, rpb, t, lslots, lenq);
    } else {
        if (records) hipLaunchKernelGGL((agg_insert_kernel<false, true>), dim3((u32)blocks), dim3(BLOCK), shmem, s, dspec, batches, bid, rows, rpb, t, lslots, lenq);
        else hipLaunchKernelGGL((agg_insert_kernel<false, false>), dim3((u32)blocks), dim3(BLOCK), shmem, s, dspec, batches, bid, rows, rpb, t, lslots, lenq);
    }
}

// Fused finalize tail: bit-pack every nullable output's validity and close the string offsets,
// with the group count read from device memory (totals[0]; totals[1 + c] string bytes).
// 8 flag bytes (any nonzero = set) -> 8 bits, LSB first
__device__ __forceinline__ u32 pack8(u64 x) {
    const u64 hi = 0x8080808080808080ULL, lo7 = 0x7F7F7F7F7F7F7F7FULL;
    const u64 nz = (((x & lo7) + lo7) | x) & hi;  // bit 7 of every nonzero byte
    return (u32)(((nz >> 7) * 0x0102040810204080ULL) >> 56);
}

// bytes [8k, 8k + 8) -> bits byte k: one 8-byte load per lane (consecutive lanes, consecutive
// words) where whole and aligned
__device__ __forceinline__ void pack_bits_at(const u8* __restrict__ bytes, u64 n, u8* __restrict__ bits, u64 k) {
    const u64 i0 = k * 8;
    if (i0 >= n) return;
    u32 b = 0;
    if (i0 + 8 <= n && !((uintptr_t)(bytes + i0) & 7)) {
        b = pack8(*(const u64*)(bytes + i0));
    } else {
        for (u64 i = i0; i < n && i < i0 + 8; ++i)
            if (bytes[i]) b |= 1u << (i - i0);
    }
    bits[k] = (u8)b;
}

// Validity bitmaps of the result columns: flag bytes packed 64 at a time into one u64 of bits
// (eight 8-byte loads, one 8-byte store), all-valid columns filled a word at a time; the bytes
// past the last whole word, and bitmaps not 8-byte aligned, byte by byte.  (One byte per thread
// and column was 0.87 ms for C4's 1e9 groups: instruction-bound, SQ_INSTS_VALU.)
__global__ void finish_outputs_kernel(OutDesc out, const u64* totals, int n_keys, int n_aggs) {
    u64 n = totals[0];
    if (n > out.cap_groups) n = out.cap_groups;
    const u64 nb = (n + 7) / 8, nw = (n / 8) / 8;  // bitmap bytes; whole u64 words of whole bytes
    const u64 tid = blockIdx.x * (u64)blockDim.x + threadIdx.x, stride = (u64)gridDim.x * blockDim.x;
    for (int c = 0; c < n_keys + n_aggs; ++c) {
        const u8* bytes = c < n_keys ? out.key_valid[c] : out.agg_valid[c - n_keys];
        u8* bits = c < n_keys ? out.key_bits[c] : out.agg_bits[c - n_keys];
        const bool fill = !bytes && bits && c >= n_keys && ((out.all_valid >> (c - n_keys)) & 1);
        if (!bits || (!bytes && !fill)) continue;
        const bool wide = !((uintptr_t)bits & 7) && (fill || !((uintptr_t)bytes & 7));
        const u64 w_end = wide ? nw : 0;
        for (u64 w = tid; w < w_end; w += stride) {
            u64 v = ~0ULL;
            if (!fill) {
                const u64* src = (const u64*)(bytes + w * 64);
                v = 0;
#pragma unroll
                for (int j = 0; j < 8; ++j) v |= (u64)pack8(src[j]) << (8 * j);
            }
            ((u64*)bits)[w] = v;
        }
        for (u64 k = w_end * 8 + tid; k < nb; k += stride) {
            if (fill) bits[k] = all_valid_byte(n, k);
            else pack_bits_at(bytes, n, bits, k);
        }
    }
    if (blockIdx.x == 0 && threadIdx.x == 0)
        for (int c = 0; c < n_keys; ++c)
            if (out.key_offsets[c] && totals[0] <= out.cap_groups) out.key_offsets[c][n] = totals[1 + c];
}

void launch_finish_outputs(hipStream_t s, const OutDesc& out, const u64* totals, int n_keys, int n_aggs) {
    u64 nb = (out.cap_groups + 7) / 8;
    u64 blocks = (nb + 255) / 256;
    if (blocks > 2048) blocks = 2048;
    if (blocks < 1) blocks = 1;
    hipLaunchKernelGGL(finish_outputs_kernel, dim3((u32)blocks), dim3(256), 0, s, out, totals, n_keys, n_aggs);
}

void launch_write_results(hipStream_t s, const Spec* dspec, const Spec& S, const BatchDesc* batches, const TableDesc& t,
                          const u64* pos, const u64* str_pos, const OutDesc& out) {
    u64 nb = finalize_blocks(t.cap);
    hipLaunchKernelGGL(write_results_kernel, dim3((u32)nb), dim3(BLOCK), 0, s, dspec, batches, t, pos, str_pos, nb, out);
}

__global__ void pack_bits_kernel(const u8* bytes, u64 n, u8* bits) {
    const u64 nb = (n + 7) / 8;
    for (u64 k = blockIdx.x * (u64)blockDim.x + threadIdx.x; k < nb; k += (u64)gridDim.x * blockDim.x) pack_bits_at(bytes, n, bits, k);
}

__global__ void fill_valid_kernel(u64 n, u8* bits) {
    const u64 nb = (n + 7) / 8;
    for (u64 k = blockIdx.x * (u64)blockDim.x + threadIdx.x; k < nb; k += (u64)gridDim.x * blockDim.x) bits[k] = all_valid_byte(n, k);
}

void launch_fill_valid(hipStream_t s, u64 n, u8* bits) {
    const u64 nb = (n + 7) / 8;
    u64 blocks = (nb + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    if (!blocks) return;
    hipLaunchKernelGGL(fill_valid_kernel, dim3((u32)blocks), dim3(256), 0, s, n, bits);
}

void launch_pack_bits(hipStream_t s, const u8* bytes, u64 n, u8* bits) {
    u64 nb = (n + 7) / 8;
    u64 blocks = (nb + 255) / 256;
    if (blocks > 4096) blocks = 4096;
    if (!blocks) return;
    hipLaunchKernelGGL(pack_bits_kernel, dim3((u32)blocks), dim3(256), 0, s, bytes, n, bits);
}

// ------------------------------------------------------------------------------------------
// Export partial-state records: [hash][key part][state words], partition-major.
// ------------------------------------------------------------------------------------------
// Key part of a record from an inline (packed) entry.
__device__ __forceinline__ void write_inline_key_part(const Spec& S, u64 key, u8* rec) {
    for (int c = 0; c < S.n_keys; ++c) {
        const dbg_datatype& ty = S.key_types[c];
        u32 w = type_width(ty.type);
        u64 b = (key >> (8 * S.koff[c])) & width_mask(w);
        if (ty.nullable) rec[S.rec_val_off[c]] = ((key >> (8 * S.voff[c])) & 0xff) != 0;
        for (u32 j = 0; j < w; ++j) rec[S.rec_key_off[c] + j] = (u8)(b >> (8 * j));
    }
}

__global__ void __launch_bounds__(BLOCK) export_kernel(const Spec* __restrict__ spec, const BatchDesc* __restrict__ batches,
                                                      TableDesc t, u32 n_parts, int scheme, const u32* __restrict__ lpart,
                                                      const u64* pos, const u64* str_pos, u64 nblocks, u8* rec_out, u8* str_out,
                                                      const u64* part_str_base) {
    const Spec& S = *spec;
    __shared__ unsigned long long cur[MAX_PARTS_LDS];
    __shared__ unsigned long long scur[DBG_MAX_KEYS][MAX_PARTS_LDS];
    for (u32 p = threadIdx.x; p < n_parts; p += BLOCK) cur[p] = pos[(u64)p * nblocks + blockIdx.x];
    bool ref_strings = S.has_strings && !S.inline_keys;
    if (ref_strings)
        for (u32 p = threadIdx.x; p < n_parts; p += BLOCK)
            for (int c = 0; c < S.n_keys; ++c)
                if (S.key_types[c].type == DBG_STRING) scur[c][p] = str_pos[((u64)p * S.n_keys + c) * nblocks + blockIdx.x];
    __syncthreads();
    u64 base = (u64)blockIdx.x * SLOTS_PER_BLOCK;
    for (u32 k = threadIdx.x; k < SLOTS_PER_BLOCK; k += BLOCK) {
        u64 s = base + k;
        if (s > t.cap) break;
        const u64* st = t.slots + s * t.stride_words;
        u64 e = st[0];
        if (e == SLOT_EMPTY) continue;
        u64 h = entry_hash(S, batches, e, s == t.cap);
        u32 p = part_of(h, n_parts, scheme, lpart, s);
        u64 r = atomicAdd(&cur[p], 1ULL);
        u8* rec = rec_out + r * S.rec_width;
        *(u64*)rec = h;
        if (S.inline_keys) {
            write_inline_key_part(S, s == t.cap ? SLOT_EMPTY : e, rec);
        } else {
            const BatchDesc& RB = batches[ref_bid(e)];
            u64 row = ref_row(e);
            for (int c = 0; c < S.n_keys; ++c) {
                const DCol& kc = RB.keys[c];
                bool v = dcol_valid(kc, row);
                if (S.key_types[c].nullable) rec[S.rec_val_off[c]] = v ? 1 : 0;
                u8* kd = rec + S.rec_key_off[c];
                if (kc.type == DBG_STRING) {
                    StrRef sr = dcol_str(kc, row);
                    u64 o = atomicAdd(&scur[c][p], (unsigned long long)sr.len);
                    for (u64 j = 0; j < sr.len; ++j) str_out[o + j] = sr.p[j];
                    ((u64*)kd)[0] = o - part_str_base[p];  // relative to the partition's blob
                    ((u64*)kd)[1] = sr.len;
                } else {
                    u32 w = type_width(kc.type);
                    u64 lo = dcol_bits(kc, row);
                    u64 hi = w == 16 ? dcol_hi(kc, row) : 0;
                    for (u32 j = 0; j < w && j < 8; ++j) kd[j] = (u8)(lo >> (8 * j));
                    for (u32 j = 8; j < w; ++j) kd[j] = (u8)(hi >> (8 * (j - 8)));
                }
            }
        }
        u64* sw = (u64*)(rec + S.rec_state_off);
        for (int w = 1; w <= S.n_words; ++w) sw[w - 1] = st[w];
    }
}

void launch_export(hipStream_t s, const Spec* dspec, const Spec& S, const BatchDesc* batches, const TableDesc& t, u32 n_parts,
                   int scheme, const u32* lpart, const u64* pos, const u64* str_pos, u8* rec_out, u8* str_out,
                   const u64* part_str_base) {
    u64 nb = finalize_blocks(t.cap);
    hipLaunchKernelGGL(export_kernel, dim3((u32)nb), dim3(BLOCK), 0, s, dspec, batches, t, n_parts, scheme, lpart, pos, str_pos, nb,
                       rec_out, str_out, part_str_base);
}


// ------------------------------------------------------------------------------------------
// export_fixed: the groups of a small inline-key table as records in a fixed-capacity buffer
// whose record 0 is the header [count][flags] — replicas + gather for low cardinality
// (SURVEY.md §8e): the count never leaves the device, so the exchange that follows (an RCCL
// all-gather of equal-size buffers) and the merge need no host round trip.  One workgroup, the
// same owned-slot scan as finalize_small.  flags = 1: incomplete (more groups than capacity, or
// inserts still deferred in the overflow lists); the merge turns that into a finalize error.
// ------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(FIN_NT) export_fixed_kernel(const Spec* __restrict__ spec, const BatchDesc* __restrict__ batches,
                                                              TableDesc t, u8* buf, u64 cap_records, int recycle) {
    const Spec& S = *spec;
    __shared__ u64 wsum[FIN_NT / 64];
    const u64 n_slots = t.cap + 1;
    const u32 per = (u32)((n_slots + FIN_NT - 1) / FIN_NT);
    const u64 base = (u64)threadIdx.x * per;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    u64 ent[FIN_MAXPER];
    u32 occ = 0, cnt = 0;
#pragma unroll
    for (u32 k = 0; k < FIN_MAXPER; ++k) {
        u64 s = base + k;
        ent[k] = (k < per && s < n_slots) ? gld<u64>(t.slots + s * t.stride_words) : SLOT_EMPTY;
    }
#pragma unroll
    for (u32 k = 0; k < FIN_MAXPER; ++k)
        if (ent[k] != SLOT_EMPTY) {
            occ |= 1u << k;
            cnt++;
        }
    u64 ic = cnt;
    for (int off = 1; off < 64; off <<= 1) {
        u64 o = __shfl_up(ic, off, 64);
        if (lane >= off) ic += o;
    }
    if (lane == 63) wsum[wave] = ic;
    __syncthreads();
    u64 p = ic - cnt, total = 0;
    for (int w = 0; w < FIN_NT / 64; ++w) {
        if (w < wave) p += wsum[w];
        total += wsum[w];
    }
    const u32 rw = S.rec_width;
    while (occ && p < cap_records) {
        const u32 k = __builtin_ctz(occ);
        occ &= occ - 1;
        const u64 s = base + k;
        const u64* st = t.slots + s * t.stride_words;
        const u64 e = gld<u64>(st);
        u8* rec = buf + (1 + p) * rw;
        const u64 key = s == t.cap ? SLOT_EMPTY : e;
        *(u64*)rec = hash_packed(S, key);
        write_inline_key_part(S, key, rec);
        u64* sw = (u64*)(rec + S.rec_state_off);
        for (int w = 1; w <= S.n_words; ++w) sw[w - 1] = gld<u64>(st + w);
        p++;
    }
    if (threadIdx.x == 0) {
        const bool pending = ld_sc1(t.counters + CNT_OVF_ROWS) != 0 || ld_sc1(t.counters + CNT_OVF_RECS) != 0;
        ((u64*)buf)[0] = total < cap_records ? total : cap_records;
        ((u64*)buf)[1] = (total > cap_records || pending) ? 1 : 0;
    }
    if (recycle) {  // dbg_agg_set_recycle: table_init of the owned slots + counter reset (an
                    // incomplete export is flagged above, so nothing is lost silently)
        __syncthreads();  // every state word has been read
        if (threadIdx.x < CNT_WORDS) t.counters[threadIdx.x] = 0;
        const u32 sw = (u32)t.stride_words;
        for (u32 k = 0; k < per; ++k) {
            u64 s = base + k;
            if (s >= n_slots) break;
            u64* d = t.slots + s * sw;
            for (u32 w = 0; w < sw; ++w) d[w] = S.slot_init[w];
        }
    }
}

void launch_export_fixed(hipStream_t s, const Spec* dspec, const BatchDesc* batches, const TableDesc& t, u8* buf, u64 cap_records,
                         int recycle) {
    hipLaunchKernelGGL(export_fixed_kernel, dim3(1), dim3(FIN_NT), 0, s, dspec, batches, t, buf, cap_records, recycle);
}

// ------------------------------------------------------------------------------------------
// Serialized states (dbg_agg_result_serialized): rows written at a fixed stride with their
// lengths -> a Binary column (offsets from an exclusive scan of the lengths, then the bytes).
// ------------------------------------------------------------------------------------------
__global__ void ser_lengths_kernel(const u8* __restrict__ lens, u64 n, u64* __restrict__ offs) {
    for (u64 i = blockIdx.x * (u64)blockDim.x + threadIdx.x; i <= n; i += (u64)gridDim.x * blockDim.x)
        offs[i] = i < n ? lens[i] : 0;
}
__global__ void ser_copy_kernel(const u8* __restrict__ src, u32 stride, u64 n, const u64* __restrict__ offs,
                                u8* __restrict__ dst) {
    for (u64 i = blockIdx.x * (u64)blockDim.x + threadIdx.x; i < n; i += (u64)gridDim.x * blockDim.x) {
        const u64 o = offs[i], len = offs[i + 1] - o;
        for (u64 b = 0; b < len; ++b) dst[o + b] = src[i * stride + b];
    }
}
void launch_ser_compact(hipStream_t s, const u8* lens, const u8* src, u32 stride, u64 n, u64* offs, u8* dst, u64* total) {
    u64 blocks = (n + 256) / 256;
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL(ser_lengths_kernel, dim3((u32)blocks), dim3(256), 0, s, lens, n, offs);
    launch_exclusive_scan(s, offs, n + 1, total);
    if (n) hipLaunchKernelGGL(ser_copy_kernel, dim3((u32)blocks), dim3(256), 0, s, src, stride, n, offs, dst);
}
