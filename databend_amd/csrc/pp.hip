// pp.hip — the radix-partitioned payload: high-cardinality GROUP BY without an HBM hash table.
//
// The reference's own design at high cardinality: TransformPartialAggregate's table keeps being
// cleared (clear_ht, EAGG/aggregate_hashtable.rs:225-239) so partial aggregation degenerates into
// appending rows to a radix-PartitionedPayload (EAGG/partitioned_payload.rs:100-143), and the final
// stage aggregates bucket by bucket on cache-sized tables (AGG/transform_aggregate_final.rs:71-156).
// On MI355X the same shape is one streaming pass per level plus one LDS pass:
//
//   level 1 (add_groups):   predicate -> group hash -> raw record [key part][args] scattered into
//                           256 partitions by the top bits of mix(hash)       (count, scan, scatter)
//   level 2..3 (finalize):  every partition re-scattered by the next hash bits until a partition's
//                           groups fit one workgroup's LDS table                (count, scan, scatter)
//   aggregate (finalize):   one workgroup per final partition: LDS hash table, LDS atomics,
//                           groups written straight to the result columns (or as state records)
//
// Every scatter is a stable-by-tile counting sort: a count pass writes per-(work unit, bucket)
// histograms, one workgroup scans them in (source partition, bucket, unit) order, and the scatter
// pass stages records in LDS, sorts each tile by bucket and writes whole runs.  No device-scope
// atomics touch the data: HBM traffic is record streams only.
#include <cstring>
#include "legacy.hpp"
#include "agg.hpp"
#include "agg_dev.hpp"

#define PP_AGG_NT 512
#define PP_AGG_LDS (72 * 1024)  // two workgroups per CU
#define PP_AU 4                  // raw records per thread in flight (aggregation)
#define PP_MAXK 1024
#define PP_WINDOW 96
// the literal pp_agg instances: PP_LIT_PER_CU workgroups of PP_LIT_NT lanes per CU, PP_LIT_RPT
// records per lane.  C4 pp_agg: 512 x 16 (8 waves per CU) 36.4 ms, 1024 x 8 (16 waves: the inserts'
// LDS round trips hidden by twice the waves) 32.1 ms; two 512 x 8 workgroups per CU cap a partition
// at 4096 records, below what 18 partition bits leave C4 (3815 on average): the generic path, 58 ms
#ifndef PP_LIT_NT
#define PP_LIT_NT 1024
#endif
#ifndef PP_LIT_RPT
#define PP_LIT_RPT 8
#endif
#ifndef PP_LIT_PER_CU
#define PP_LIT_PER_CU 1  // workgroups per CU (each with 1 / PP_LIT_PER_CU of the LDS)
#endif

typedef __attribute__((address_space(3))) u8 l8;
typedef __attribute__((address_space(3))) u16 l16;
typedef __attribute__((address_space(3))) u32 l32;
typedef __attribute__((address_space(3))) u64 l64;

// Partition bits are the top bits of the reference group hash itself (its murmur finalizer mixes
// every input bit into them; only a Boolean-only key, <= 3 groups, never partitioned, hashes to
// 0/1): level-local bucket = (h >> shift) & (K - 1); the LDS slot uses the low 32 bits.
__device__ __forceinline__ u64 pp_mix(u64 h) { return h; }

// little-endian value of w (1..8) bytes at p (global memory, any alignment)
__device__ __forceinline__ u64 ld_le(const u8* p, u32 w) { return load_partial(p, w) & width_mask(w); }

// group_hash_columns of a packed fixed-width key (row format, Spec koff/voff).
__device__ __forceinline__ u64 pp_fixed_hash(const Spec& S, const u8* k) {
    u64 h = 0;
    for (int c = 0; c < S.n_keys; ++c) {
        const dbg_datatype& t = S.key_types[c];
        u64 x;
        const bool v = !t.nullable || gld<u8>(k + S.voff[c]) != 0;
        if (!v) x = NULL_HASH_VAL;
        else if (t.type == DBG_DECIMAL128) x = hash_i128(ld_le(k + S.koff[c], 8), ld_le(k + S.koff[c] + 8, 8));
        else x = hash_bits(t.type, ld_le(k + S.koff[c], type_width(t.type)));
        h = c == 0 ? x : (h * NULL_HASH_VAL) ^ x;
    }
    return h;
}
__device__ __forceinline__ u64 pp_rec_hash(const Spec& S, const u8* rec) { return S.pp_str ? gld<u64>(rec) : pp_fixed_hash(S, rec); }

// hash of input row i of a batch (raw rows or exchange records, which carry it)
__device__ __forceinline__ u64 pp_row_hash(const Spec& S, const BatchDesc& B, u64 i) {
    if (B.is_records) return gld<u64>(B.rec_base + i * (u64)B.rec_width);
    return group_hash(B.keys, S.n_keys, i);
}

// ---- LDS byte helpers ----
__device__ __forceinline__ void lput(l8* d, u32 off, u64 v, u32 w) {
    if (w == 8 && !(off & 7)) { *(l64*)(d + off) = v; return; }
    if (w == 4 && !(off & 3)) { *(l32*)(d + off) = (u32)v; return; }
    if (w == 2 && !(off & 1)) { *(l16*)(d + off) = (u16)v; return; }
    for (u32 j = 0; j < w; ++j) d[off + j] = (u8)(v >> (8 * j));
}
__device__ __forceinline__ u64 lget(const l8* d, u32 off, u32 w) {
    if (w == 8 && !(off & 7)) return *(const l64*)(d + off);
    if (w == 4 && !(off & 3)) return *(const l32*)(d + off);
    if (w == 2 && !(off & 1)) return *(const l16*)(d + off);
    u64 v = 0;
    for (u32 j = 0; j < w; ++j) v |= (u64)d[off + j] << (8 * j);
    return v;
}

// Key part of row i into d (LDS, zeroed): packed row format or [hash][klen][blob].
__device__ __forceinline__ void pp_put_key(const Spec& S, const DCol* keys, u32 bid, u64 i, u64 h, l8* d) {
    if (!S.pp_str) {
        for (int c = 0; c < S.n_keys; ++c) {
            const DCol& col = keys[c];
            const bool v = dcol_valid(col, i);
            if (S.key_types[c].nullable) d[S.voff[c]] = v ? 1 : 0;
            if (!v) continue;
            const u32 w = type_width(col.type);
            if (col.type == DBG_DECIMAL128) {
                lput(d, S.koff[c], dcol_bits(col, i), 8);
                lput(d, S.koff[c] + 8, dcol_hi(col, i), 8);
            } else {
                u64 b = dcol_bits(col, i);
                if (col.type == DBG_FLOAT32 || col.type == DBG_FLOAT64) b = canon_float_bits(col.type, b);
                lput(d, S.koff[c], b, w);
            }
        }
        return;
    }
    *(l64*)d = h;
    u32 len = 0;
    for (int c = 0; c < S.n_keys; ++c) {
        const DCol& col = keys[c];
        const bool v = dcol_valid(col, i);
        len += S.key_types[c].nullable ? 1 : 0;
        if (col.type == DBG_STRING) len += 1 + (v ? (u32)min<u64>(dcol_str(col, i).len, 256) : 0);
        else len += type_width(col.type);
    }
    if (len > PP_BLOB) {
        d[8] = PP_KLEN_LONG;
        *(l64*)(d + 16) = ((u64)bid << 32) | (u64)(u32)i;
        return;
    }
    d[8] = (u8)len;
    u32 o = 9;
    for (int c = 0; c < S.n_keys; ++c) {
        const DCol& col = keys[c];
        const bool v = dcol_valid(col, i);
        if (S.key_types[c].nullable) d[o++] = v ? 1 : 0;
        if (col.type == DBG_STRING) {
            StrRef s = v ? dcol_str(col, i) : StrRef{nullptr, 0};
            d[o++] = (u8)s.len;
            for (u64 j = 0; j < s.len; ++j) d[o + j] = gld<u8>(s.p + j);
            o += (u32)s.len;
        } else {
            const u32 w = type_width(col.type);
            if (v) {
                if (col.type == DBG_DECIMAL128) {
                    lput(d, o, dcol_bits(col, i), 8);
                    lput(d, o + 8, dcol_hi(col, i), 8);
                } else {
                    u64 b = dcol_bits(col, i);
                    if (col.type == DBG_FLOAT32 || col.type == DBG_FLOAT64) b = canon_float_bits(col.type, b);
                    lput(d, o, b, w);
                }
            }
            o += w;
        }
    }
}

// Raw record of row i: key part + argument values + argument validity bits (d zeroed).
__device__ __forceinline__ void pp_put_raw(const Spec& S, const BatchDesc& B, u32 bid, u64 i, u64 h, l8* d) {
    pp_put_key(S, B.keys, bid, i, h, d);
    u64 vm = 0;
    for (int a = 0; a < S.n_aggs; ++a) {
        const DAgg& A = S.aggs[a];
        if (A.arg_type < 0) continue;
        const DCol& c = B.args[a];
        const bool v = dcol_valid(c, i);
        if (S.pp_avbit[a] >= 0 && v) vm |= 1ULL << S.pp_avbit[a];
        if (!v) continue;
        const u32 w = A.arg_type == DBG_BOOLEAN ? 1 : type_width(A.arg_type);
        if (A.arg_type == DBG_DECIMAL128) {
            lput(d, S.pp_aoff[a], dcol_bits(c, i), 8);
            lput(d, S.pp_aoff[a] + 8, dcol_hi(c, i), 8);
        } else {
            lput(d, S.pp_aoff[a], dcol_bits(c, i), w);
        }
    }
    if (vm) {
        const u32 nb = (S.pp_rw_raw - S.pp_avoff) < 8 ? (S.pp_rw_raw - S.pp_avoff) : 8;
        lput(d, S.pp_avoff, vm, nb);
    }
}

// State record of exchange record i (LAYOUT_RECORD batch): key part + the record's state words.
__device__ __forceinline__ void pp_put_state(const Spec& S, const BatchDesc& B, u32 bid, u64 i, u64 h, l8* d) {
    pp_put_key(S, B.keys, bid, i, h, d);
    const u8* src = B.rec_base + i * (u64)B.rec_width + S.rec_state_off;
    for (int w = 0; w < S.n_words; ++w) *(l64*)(d + S.pp_kw + 8 * w) = load_u64_unaligned(src + 8 * w);
}

// ---- argument values of a raw record (global) ----
__device__ __forceinline__ i64 pp_sext(int t, u64 b) {
    switch (t) {
        case DBG_INT8: return (i64)(int8_t)b;
        case DBG_INT16: return (i64)(int16_t)b;
        case DBG_INT32: case DBG_DATE: return (i64)(int32_t)b;
        case DBG_BOOLEAN: return (i64)(b & 1);
        default: return (i64)b;
    }
}

// accumulate_keys of one raw record into the slot states st (st[A.w0] = first word).
template <int AS>
__device__ __forceinline__ void pp_apply_raw(const Spec& S, wptr<AS> st, const u8* rec) {
    u64 vm = ~0ULL;
    if (S.pp_avoff < S.pp_rw_raw) vm = ld_le(rec + S.pp_avoff, min(8u, S.pp_rw_raw - S.pp_avoff));
    for (int a = 0; a < S.n_aggs; ++a) {
        const DAgg& A = S.aggs[a];
        if (A.arg_type >= 0 && S.pp_avbit[a] >= 0 && !((vm >> S.pp_avbit[a]) & 1)) continue;
        wptr<AS> w = st + A.w0;
        const u8* p = rec + S.pp_aoff[a];
        const u32 aw = A.arg_type == DBG_BOOLEAN ? 1 : (A.arg_type >= 0 ? type_width(A.arg_type) : 0);
        switch (A.kind) {
            case DBG_AGG_COUNT: at_add<AS>(w, 1ULL); break;
            case DBG_AGG_SUM: case DBG_AGG_AVG: {
                if (A.sumk == SUMK_I64) at_add<AS>(w, (u64)pp_sext(A.arg_type, ld_le(p, aw)));
                else if (A.sumk == SUMK_F64) {
                    const u64 b = ld_le(p, aw);
                    at_addf<AS>(w, A.arg_type == DBG_FLOAT32 ? (double)__uint_as_float((u32)b) : __longlong_as_double((long long)b));
                } else {
                    add128<AS>(w, ld_le(p, 8), ld_le(p + 8, 8));
                }
                if (A.kind == DBG_AGG_AVG) at_add<AS>(w + (A.sumk == SUMK_I128 ? 2 : 1), 1ULL);
                break;
            }
            case DBG_AGG_MIN: case DBG_AGG_MAX: {
                const bool mn = A.kind == DBG_AGG_MIN;
                const u64 b = ld_le(p, aw < 8 ? aw : 8);  // Decimal128 (p <= 18): the low word
                if (A.mmk == MMK_I128) at_minmax128<AS>(w, b, ld_le(p + 8, 8), mn, S.err);
                else if (A.mmk == MMK_I64) at_minmax<AS>(w, (u64)pp_sext(A.arg_type, b), mn, true);
                else if (A.mmk == MMK_U64) at_minmax<AS>(w, b, mn, false);
                else
                    at_minmax<AS>(w, f64_order_key(A.arg_type == DBG_FLOAT32 ? (double)__uint_as_float((u32)b)
                                                                          : __longlong_as_double((long long)b)),
                                  mn, false);
                break;
            }
        }
        if (A.flag_bit >= 0) set_flag<AS>(st, S.flags_word, A.flag_bit);
    }
}

// ------------------------------------------------------------------------------------------
// Cardinality probe: distinct group hashes among n_sample evenly spaced (selected) rows.
// set: 2 * set_cap words [hash | count]; out: [0] selected, [1] distinct, [2] f1, [3] f2.
// (Per-sample counts come out right even when the LDS set spills: one hash's count may then sit in
// the global set from two adds, never in two slots.)
// ------------------------------------------------------------------------------------------
// Each workgroup counts its contiguous share of the samples in an LDS set first (a handful of
// distinct keys — TPC-H Q1's four groups — would otherwise put every sample's atomics on the same
// few HBM words) and adds each distinct hash to the global set once.
#define PP_PROBE_SLOTS 2048
__device__ __forceinline__ void pp_probe_global(u64* set, u64 set_cap, u64* out, u64 h, u64 c) {
    u64 s = slot_mix(h) & (set_cap - 1);
    for (u64 p = 0; p < set_cap; ++p) {
        u64 old = atomicCAS((unsigned long long*)(set + 2 * s), 0ULL, (unsigned long long)h);
        if (old == 0) atomicAdd((unsigned long long*)(out + 1), 1ULL);
        if (old == 0 || old == h) {
            atomicAdd((unsigned long long*)(set + 2 * s + 1), (unsigned long long)c);
            return;
        }
        s = (s + 1) & (set_cap - 1);
    }
}
__global__ void __launch_bounds__(256) pp_sample_kernel(const Spec* __restrict__ spec, const BatchDesc* __restrict__ batches,
                                                       u32 bid, u64 rows, u64 n_sample, u64* set, u64 set_cap, u64* out) {
    const Spec& S = *spec;
    const BatchDesc& B = batches[bid];
    __shared__ u64 lkey[PP_PROBE_SLOTS];
    __shared__ u32 lcnt[PP_PROBE_SLOTS];
    __shared__ u32 nsel;
    for (u32 t = threadIdx.x; t < PP_PROBE_SLOTS; t += 256) {
        lkey[t] = 0;
        lcnt[t] = 0;
    }
    if (threadIdx.x == 0) nsel = 0;
    __syncthreads();
    const u64 per = (n_sample + gridDim.x - 1) / gridDim.x;
    const u64 k0 = (u64)blockIdx.x * per, k1 = min(n_sample, k0 + per);
    u32 mysel = 0;
    for (u64 k = k0 + threadIdx.x; k < k1; k += 256) {
        const u64 i = (k * rows) / n_sample;
        if (!B.is_records && B.n_nodes && !eval_pred(B.nodes, B.n_nodes, B.fcols, i)) continue;
        mysel++;
        u64 h = pp_row_hash(S, B, i);
        h = h ? h : 1;
        u32 s = (u32)slot_mix(h) & (PP_PROBE_SLOTS - 1);
        bool done = false;
        for (u32 p = 0; p < 64 && !done; ++p) {  // short probes: a full LDS set spills to the global one
            u64 old = atomicCAS((unsigned long long*)&lkey[s], 0ULL, (unsigned long long)h);
            if (old == 0 || old == h) {
                atomicAdd(&lcnt[s], 1u);
                done = true;
            }
            s = (s + 1) & (PP_PROBE_SLOTS - 1);
        }
        if (!done) pp_probe_global(set, set_cap, out, h, 1);
    }
    if (mysel) atomicAdd(&nsel, mysel);
    __syncthreads();
    for (u32 t = threadIdx.x; t < PP_PROBE_SLOTS; t += 256)
        if (lcnt[t]) pp_probe_global(set, set_cap, out, lkey[t], lcnt[t]);
    if (threadIdx.x == 0 && nsel) atomicAdd((unsigned long long*)out, (unsigned long long)nsel);
}
__global__ void __launch_bounds__(256) pp_sample_stats_kernel(const u64* set, u64 set_cap, u64* out) {
    u32 f1 = 0, f2 = 0;
    for (u64 s = blockIdx.x * 256ULL + threadIdx.x; s < set_cap; s += (u64)gridDim.x * 256) {
        const u64 c = set[2 * s + 1];
        f1 += c == 1;
        f2 += c == 2;
    }
    if (f1) atomicAdd((unsigned long long*)(out + 2), (unsigned long long)f1);
    if (f2) atomicAdd((unsigned long long*)(out + 3), (unsigned long long)f2);
}

void launch_pp_sample(hipStream_t s, const Spec* dspec, const BatchDesc* batches, u32 bid, u64 rows, u64 n_sample, u64* set,
                      u64 set_cap, u64* out) {
    hipMemsetAsync(set, 0, set_cap * 16, s);
    hipMemsetAsync(out, 0, 32, s);
    hipLaunchKernelGGL(pp_sample_kernel, dim3(1024), dim3(256), 0, s, dspec, batches, bid, rows, n_sample, set, set_cap, out);
    hipLaunchKernelGGL(pp_sample_stats_kernel, dim3(1024), dim3(256), 0, s, set, set_cap, out);
}

// A record as the aggregation reads it: W words held in registers (raw records of up to 64 bytes,
// loaded PP_AU per thread before any LDS work so the loads overlap), or read from global memory
// (wide raw records, state records).  word(w) / le(off, bytes) give little-endian fields.
template <int W>
struct RegRec {
    u64 r[W];
    __device__ __forceinline__ u64 word(u32 w) const {
        // a select chain over register values: the opaque copy keeps the optimizer from folding it
        // into one load at a dynamic index, which puts the whole record array in scratch (W >= 3)
        u64 v = r[0];
#pragma unroll
        for (int k = 1; k < W; ++k) {
            u64 c = r[k];
            asm volatile("" : "+v"(c));
            v = w == (u32)k ? c : v;
        }
        return v;
    }
    __device__ __forceinline__ u64 le(u32 off, u32 nb) const {
        const u32 wi = off >> 3, sh = (off & 7) * 8;
        u64 v = word(wi) >> sh;
        if (sh && (off & 7) + nb > 8) v |= word(wi + 1) << (64 - sh);
        return v & width_mask(nb);
    }
};
struct GlbRec {
    const u8* p;
    __device__ __forceinline__ u64 word(u32 w) const { return gld<u64>(p + 8 * w); }
    __device__ __forceinline__ u64 le(u32 off, u32 nb) const { return ld_le(p + off, nb); }
};

template <typename R>
__device__ __forceinline__ u64 pp_hash_of(const Spec& S, const R& rk) {
    if (S.pp_str) return rk.word(0);
    u64 h = 0;
    for (int c = 0; c < S.n_keys; ++c) {
        const dbg_datatype& t = S.key_types[c];
        u64 x;
        const bool v = !t.nullable || rk.le(S.voff[c], 1) != 0;
        if (!v) x = NULL_HASH_VAL;
        else if (t.type == DBG_DECIMAL128) x = hash_i128(rk.le(S.koff[c], 8), rk.le(S.koff[c] + 8, 8));
        else x = hash_bits(t.type, rk.le(S.koff[c], type_width(t.type)));
        h = c == 0 ? x : (h * NULL_HASH_VAL) ^ x;
    }
    return h;
}

// ------------------------------------------------------------------------------------------
// count: per work unit, a histogram of the level's local bucket over its (selected) rows/records
// ------------------------------------------------------------------------------------------
#define PP_CU 8  // rows / records per thread in flight (count)
template <int SRC, int W = 0>
__global__ void __launch_bounds__(PP_NT) pp_count_kernel(const Spec* __restrict__ spec, const BatchDesc* __restrict__ batches,
                                                        int kind, const u8* __restrict__ recs, const PPChunk* __restrict__ chunks,
                                                        u32 shift, u32 kbits, u32* __restrict__ cnt) {
    const Spec& S = *spec;
    __shared__ u32 hist[PP_MAXK];
    const u32 K = 1u << kbits;
    for (u32 b = threadIdx.x; b < K; b += PP_NT) hist[b] = 0;
    __syncthreads();
    const PPChunk ch = chunks[blockIdx.x];
    const u64 end = ch.start + ch.n;
    const BatchDesc& B = batches[ch.bid];
    const u32 rw = kind ? S.pp_rw_state : S.pp_rw_raw;
    for (u64 i0 = ch.start + threadIdx.x; i0 < end; i0 += (u64)PP_NT * PP_CU) {
        u32 bk[PP_CU];
#pragma unroll
        for (int u = 0; u < PP_CU; ++u) {  // hashes of PP_CU rows, loads independent of each other
            const u64 i = i0 + (u64)u * PP_NT;
            bk[u] = ~0u;
            if (i >= end) continue;
            if (SRC == 0) {
                if (!B.is_records && B.n_nodes && !eval_pred(B.nodes, B.n_nodes, B.fcols, i)) continue;
                bk[u] = (u32)(pp_mix(pp_row_hash(S, B, i)) >> shift) & (K - 1);
            } else if constexpr (W > 0) {  // records of W words: whole-word loads, key fields from registers
                RegRec<(W > 0 ? W : 1)> rr;
#pragma unroll
                for (int w = 0; w < W; ++w) rr.r[w] = gld<u64>(recs + i * rw + 8 * w);
                bk[u] = (u32)(pp_mix(pp_hash_of(S, rr)) >> shift) & (K - 1);
            } else {
                bk[u] = (u32)(pp_mix(pp_rec_hash(S, recs + i * rw)) >> shift) & (K - 1);
            }
        }
#pragma unroll
        for (int u = 0; u < PP_CU; ++u)
            if (bk[u] != ~0u) atomicAdd(&hist[bk[u]], 1u);
    }
    __syncthreads();
    for (u32 b = threadIdx.x; b < K; b += PP_NT) cnt[(u64)blockIdx.x * K + b] = hist[b];
}

void launch_pp_count(hipStream_t s, const Spec* dspec, const BatchDesc* batches, int src, int kind, const u8* src_recs,
                     const PPChunk* chunks, u32 n_chunks, u32 shift, u32 kbits, u32* cnt, u32 wpr) {
    if (!n_chunks) return;
    if (src == 0) {
        hipLaunchKernelGGL(pp_count_kernel<0>, dim3(n_chunks), dim3(PP_NT), 0, s, dspec, batches, kind, src_recs, chunks, shift, kbits, cnt);
        return;
    }
    // raw records of 1 or 2 words (the fixed-key shapes): key fields from whole-word loads
    if (wpr == 1)
        hipLaunchKernelGGL((pp_count_kernel<1, 1>), dim3(n_chunks), dim3(PP_NT), 0, s, dspec, batches, kind, src_recs, chunks, shift, kbits, cnt);
    else if (wpr == 2)
        hipLaunchKernelGGL((pp_count_kernel<1, 2>), dim3(n_chunks), dim3(PP_NT), 0, s, dspec, batches, kind, src_recs, chunks, shift, kbits, cnt);
    else
        hipLaunchKernelGGL((pp_count_kernel<1>), dim3(n_chunks), dim3(PP_NT), 0, s, dspec, batches, kind, src_recs, chunks, shift, kbits, cnt);
}

// Level-2 histograms from the digit array the level-1 scatter wrote (2 bytes per record instead
// of the record): bucket = dig >> (16 - kbits)
__global__ void __launch_bounds__(PP_NT) pp_count_dig_kernel(const PPChunk* __restrict__ chunks, const uint16_t* __restrict__ dig,
                                                            u32 kbits, u32* __restrict__ cnt) {
    __shared__ u32 hist[PP_MAXK];
    const u32 K = 1u << kbits, dsh = 16 - kbits;
    for (u32 b = threadIdx.x; b < K; b += PP_NT) hist[b] = 0;
    __syncthreads();
    const PPChunk ch = chunks[blockIdx.x];
    const u64 end = ch.start + ch.n;
    for (u64 i0 = ch.start + threadIdx.x; i0 < end; i0 += (u64)PP_NT * PP_CU) {
        u32 d[PP_CU];
#pragma unroll
        for (int u = 0; u < PP_CU; ++u) {
            const u64 i = i0 + (u64)u * PP_NT;
            d[u] = i < end ? (u32)gld<uint16_t>(dig + i) : ~0u;
        }
#pragma unroll
        for (int u = 0; u < PP_CU; ++u)
            if (d[u] != ~0u) atomicAdd(&hist[d[u] >> dsh], 1u);
    }
    __syncthreads();
    for (u32 b = threadIdx.x; b < K; b += PP_NT) cnt[(u64)blockIdx.x * K + b] = hist[b];
}

void launch_pp_count_dig(hipStream_t s, const PPChunk* chunks, u32 n_chunks, const uint16_t* dig, u32 kbits, u32* cnt) {
    if (!n_chunks) return;
    hipLaunchKernelGGL(pp_count_dig_kernel, dim3(n_chunks), dim3(PP_NT), 0, s, chunks, dig, kbits, cnt);
}

// ------------------------------------------------------------------------------------------
// scan: destinations of every (unit, bucket) run, all parallel.
//   within:  one thread per (group g, bucket b): exclusive prefix over the group's units
//            -> off[unit][b] (relative to the partition start), tot[g * K + b]
//   blocks:  tot scanned in blocks of SCAN_ITEMS -> part_off (block-relative) + block sums
//   sums:    one workgroup scans the block sums; fixup adds them -> part_off[g * K + b] = start
//            of destination partition (g, b), part_off[G * K] = total.
// A scatter unit starts its bucket-b run at part_off[group * K + b] + off[unit][b].
// ------------------------------------------------------------------------------------------
#define SCAN_NT 256
#define SCAN_PER 16
#define SCAN_ITEMS (SCAN_NT * SCAN_PER)

__global__ void __launch_bounds__(SCAN_NT) pp_scan_within_kernel(const u32* __restrict__ cnt, u32 kbits, const u32* __restrict__ c0,
                                                                u32 G, u64* __restrict__ off, u64* __restrict__ tot) {
    const u32 K = 1u << kbits;
    const u64 j = blockIdx.x * (u64)SCAN_NT + threadIdx.x;
    if (j >= (u64)G * K) return;
    const u32 g = (u32)(j >> kbits), b = (u32)(j & (K - 1));
    u64 run = 0;
    for (u32 c = c0[g]; c < c0[g + 1]; ++c) {
        const u64 idx = (u64)c * K + b;
        off[idx] = run;
        run += cnt[idx];
    }
    tot[j] = run;
}

// the same for groups of many units (level 1: one group): one workgroup per (group, bucket)
__global__ void __launch_bounds__(SCAN_NT) pp_scan_within_wg_kernel(const u32* __restrict__ cnt, u32 kbits, const u32* __restrict__ c0,
                                                                   u32 G, u64* __restrict__ off, u64* __restrict__ tot) {
    __shared__ u64 ws[SCAN_NT / 64];
    const u32 K = 1u << kbits;
    const u64 j = blockIdx.x;
    const u32 g = (u32)(j >> kbits), b = (u32)(j & (K - 1));
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    u64 run = 0;
    for (u32 cb = c0[g]; cb < c0[g + 1]; cb += SCAN_NT) {
        const u32 c = cb + threadIdx.x;
        const u64 v = c < c0[g + 1] ? cnt[(u64)c * K + b] : 0;
        u64 x = v;
        for (int o = 1; o < 64; o <<= 1) {
            const u64 y = __shfl_up(x, o, 64);
            if (lane >= o) x += y;
        }
        if (lane == 63) ws[wave] = x;
        __syncthreads();
        u64 pre = x - v, all = 0;
        for (int w = 0; w < SCAN_NT / 64; ++w) {
            if (w < wave) pre += ws[w];
            all += ws[w];
        }
        if (c < c0[g + 1]) off[(u64)c * K + b] = run + pre;
        run += all;
        __syncthreads();
    }
    if (threadIdx.x == 0) tot[j] = run;
}

__global__ void __launch_bounds__(SCAN_NT) pp_scan_blocks_kernel(const u64* __restrict__ tot, u64 E, u64* __restrict__ part_off,
                                                                u64* __restrict__ bsum) {
    __shared__ u64 ws[SCAN_NT / 64];
    const u64 base = (u64)blockIdx.x * SCAN_ITEMS + (u64)threadIdx.x * SCAN_PER;
    u64 v[SCAN_PER], s = 0;
#pragma unroll
    for (int k = 0; k < SCAN_PER; ++k) {
        v[k] = base + k < E ? tot[base + k] : 0;
        s += v[k];
    }
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    u64 x = s;
    for (int o = 1; o < 64; o <<= 1) {
        const u64 y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) ws[wave] = x;
    __syncthreads();
    u64 pre = x - s, all = 0;
    for (int w = 0; w < SCAN_NT / 64; ++w) {
        if (w < wave) pre += ws[w];
        all += ws[w];
    }
#pragma unroll
    for (int k = 0; k < SCAN_PER; ++k) {
        if (base + k < E) part_off[base + k] = pre;
        pre += v[k];
    }
    if (threadIdx.x == 0) bsum[blockIdx.x] = all;
}

__global__ void __launch_bounds__(SCAN_NT) pp_scan_fixup_kernel(u64* __restrict__ part_off, u64 E, const u64* __restrict__ bsum,
                                                               u64 nb) {
    const u64 i = blockIdx.x * (u64)SCAN_NT + threadIdx.x;
    if (i < E) part_off[i] += bsum[i / SCAN_ITEMS];
    if (i == 0) part_off[E] = bsum[nb];  // the total (exclusive scan of nb sums writes it at [nb])
}

void launch_exclusive_scan(hipStream_t s, u64* data, u64 n, u64* total);

u64 pp_scan_scratch_words(u32 n_groups, u32 kbits) {
    const u64 E = (u64)n_groups << kbits;
    return E + (E + SCAN_ITEMS - 1) / SCAN_ITEMS + 2;
}

void launch_pp_scan(hipStream_t s, const u32* cnt, u32 n_chunks, u32 kbits, const u32* group_c0, u32 n_groups, u64* off,
                    u64* part_off, u64* scratch) {
    const u64 E = (u64)n_groups << kbits;
    const u64 nb = (E + SCAN_ITEMS - 1) / SCAN_ITEMS;
    u64* tot = scratch;
    u64* bsum = scratch + E;
    if (n_chunks >= 64 * (u64)n_groups)  // many units per group: a workgroup per (group, bucket)
        hipLaunchKernelGGL(pp_scan_within_wg_kernel, dim3((u32)E), dim3(SCAN_NT), 0, s, cnt, kbits, group_c0, n_groups, off, tot);
    else
        hipLaunchKernelGGL(pp_scan_within_kernel, dim3((u32)((E + SCAN_NT - 1) / SCAN_NT)), dim3(SCAN_NT), 0, s, cnt, kbits,
                           group_c0, n_groups, off, tot);
    hipLaunchKernelGGL(pp_scan_blocks_kernel, dim3((u32)nb), dim3(SCAN_NT), 0, s, tot, E, part_off, bsum);
    launch_exclusive_scan(s, bsum, nb, bsum + nb);
    hipLaunchKernelGGL(pp_scan_fixup_kernel, dim3((u32)((E + SCAN_NT - 1) / SCAN_NT)), dim3(SCAN_NT), 0, s, part_off, E, bsum, nb);
}

// ------------------------------------------------------------------------------------------
// scatter
// ------------------------------------------------------------------------------------------
// block-wide exclusive scan of one u32 per thread (PP_NT threads); returns the total
__device__ __forceinline__ u32 block_excl_scan(u32 v, u32* wtot, u32& total) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    u32 x = v;
    for (int o = 1; o < 64; o <<= 1) {
        const u32 y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) wtot[wave] = x;
    __syncthreads();
    u32 pre = 0, tot = 0;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) {
        if (w < wave) pre += wtot[w];
        tot += wtot[w];
    }
    __syncthreads();
    total = tot;
    return pre + x - v;
}

// Direct scatter (the form every level runs): per tile of T x U rows, each selected row's bucket
// and its rank in the bucket (one LDS atomic) give its destination run[bucket] + rank, and the
// record is stored straight there — from registers (records of W words, W > 0) or from a
// per-thread LDS scratch slot where a raw row's record is built (W == 0).  Three barriers per tile;
// the records of one bucket land contiguously within the tile, so the XCD's L2 merges them into
// whole lines.  LDS: hist u32 [K] | run u64 [K] | scratch [T * U * rw] (W == 0).
#ifndef PP_DIRECT_U2
#define PP_DIRECT_U2 4  // records per thread per tile at W <= 2 (8: longer runs, half the occupancy — C4 level 2 14.8 -> 17.2 ms)
#endif
__host__ __device__ __forceinline__ u32 pp_direct_u(int W, u32 rw) {  // rows per thread per step
    if (W > 0) return W <= 2 ? PP_DIRECT_U2 : (W <= 4 ? 2 : 1);
    const u32 u = PP_SCRATCH_BYTES / (PP_NT * rw);
    return u >= 4 ? 4 : (u >= 1 ? u : 1);
}

// Exclusive scan of a tile histogram (K <= 1024 buckets) by wave 0 into toff; *total = sum.
__device__ __forceinline__ void pp_tile_scan(const l32* hist, u32 K, l32* toff, l32* total) {
    if (threadIdx.x >= 64) return;
    const u32 per = (K + 63) / 64, b0 = threadIdx.x * per;
    u32 t = 0;
    for (u32 j = 0; j < per; ++j)
        if (b0 + j < K) t += hist[b0 + j];
    u32 incl = t;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
        const u32 y = __shfl_up(incl, d);
        if ((int)threadIdx.x >= d) incl += y;
    }
    u32 e = incl - t;
    for (u32 j = 0; j < per; ++j)
        if (b0 + j < K) {
            const u32 c = hist[b0 + j];
            toff[b0 + j] = e;
            e += c;
        }
    if (threadIdx.x == 63) *total = incl;
}

template <int SRC, int W, int SORTED>
__global__ void __launch_bounds__(PP_NT) pp_scatter_direct_kernel(const Spec* __restrict__ spec, const BatchDesc* __restrict__ batches,
                                                                 int kind, const u8* __restrict__ recs,
                                                                 const PPChunk* __restrict__ chunks, u32 shift, u32 kbits,
                                                                 const u64* __restrict__ off, const u64* __restrict__ part_off,
                                                                 u8* __restrict__ dst, u32* __restrict__ cnt_next, u32 sh_next,
                                                                 u32 kb_next) {
    extern __shared__ __attribute__((aligned(16))) u64 lds_raw[];
    __shared__ u32 tile_total;
    const Spec& S = *spec;
    const u32 K = 1u << kbits;
    const u32 rw = kind ? S.pp_rw_state : S.pp_rw_raw;
    const u32 wpr = rw / 8;
    l32* hist = (l32*)lds_raw;
    l64* run = (l64*)(hist + K + (K & 1));
    l8* scratch = (l8*)(run + K);
    constexpr u32 UMAX = (W > 0 && W <= 2) ? PP_DIRECT_U2 : 4;
    const u32 U = pp_direct_u(W, rw);
    const u32 T = W > 0 ? PP_NT : pp_direct_t(rw);
    const PPChunk ch = chunks[blockIdx.x];
    for (u32 b = threadIdx.x; b < K; b += PP_NT) {
        hist[b] = 0;
        run[b] = part_off[(u64)ch.group * K + b] + off[(u64)blockIdx.x * K + b];
    }
    // next level's histogram per destination partition (records only): [b][digit] after the scratch
    const u32 KN = cnt_next ? K << kb_next : 0;
    l32* hn = (l32*)(scratch + (W == 0 ? (size_t)T * U * rw : 0));
    for (u32 i = threadIdx.x; i < KN; i += PP_NT) hn[i] = 0;
    // tile-sorted stores (records in registers, `sorted`): as pp_l1_fixed_kernel — staged words
    // [T * U * W] u64 | bucket per staged record [T * U] u16 | tile offsets [K] u32
    l64* stage = (l64*)(hn + KN + (KN & 1));
    l16* sbk = (l16*)(stage + (size_t)T * U * (W > 0 ? W : 1));
    l32* toff = (l32*)(sbk + (size_t)T * U + ((T * U) & 1));
    __syncthreads();
    const u64 end = ch.start + ch.n;
    const BatchDesc& B = batches[ch.bid];
    const u64 step = (u64)T * U;
    // records in registers (W > 0): the next tile's loads are issued before this tile is ranked and
    // stored, so the tile's three barriers do not each wait out a memory latency
    RegRec<(W > 0 ? W : 1)> nx[UMAX];
    auto load_tile = [&](u64 base) {
        if constexpr (SRC == 1 && W > 0) {
#pragma unroll
            for (u32 u = 0; u < UMAX; ++u) {
                const u64 i = base + (u64)u * T + threadIdx.x;
                if (u >= U || i >= end) continue;
                const u8* r = recs + i * rw;
#pragma unroll
                for (int w = 0; w < W; ++w) nx[u].r[w] = gld<u64>(r + 8 * w);
            }
        }
    };
    load_tile(ch.start);
    for (u64 base = ch.start; base < end; base += step) {
        u32 bk[UMAX], rk[UMAX];
        RegRec<(W > 0 ? W : 1)> rr[UMAX];
        u32 m = 0;
#pragma unroll
        for (u32 u = 0; u < UMAX; ++u) {
            const u64 i = base + (u64)u * T + threadIdx.x;
            if (u >= U || threadIdx.x >= T || i >= end) continue;
            if constexpr (SRC == 1 && W > 0) rr[u] = nx[u];
            m |= 1u << u;
        }
        if (base + step < end) load_tile(base + step);
#pragma unroll
        for (u32 u = 0; u < UMAX; ++u) {
            if (!((m >> u) & 1)) continue;
            const u64 i = base + (u64)u * T + threadIdx.x;
            u64 h;
            if constexpr (SRC == 1 && W > 0) {
                h = pp_hash_of(S, rr[u]);
            } else {
                l8* d = scratch + ((size_t)threadIdx.x * U + u) * rw;
                if (SRC == 0) {
                    if (!B.is_records && B.n_nodes && !eval_pred(B.nodes, B.n_nodes, B.fcols, i)) {
                        m &= ~(1u << u);
                        continue;
                    }
                    for (u32 w = 0; w < wpr; ++w) ((l64*)d)[w] = 0;
                    h = pp_row_hash(S, B, i);
                    if (kind) pp_put_state(S, B, ch.bid, i, h, d);
                    else pp_put_raw(S, B, ch.bid, i, h, d);
                } else {
                    const u8* r = recs + i * rw;
                    for (u32 w = 0; w < wpr; ++w) ((l64*)d)[w] = gld<u64>(r + 8 * w);
                    h = pp_rec_hash(S, r);
                }
            }
            bk[u] = (u32)(pp_mix(h) >> shift) & (K - 1);
            rk[u] = __hip_atomic_fetch_add(&hist[bk[u]], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            if (KN) {
                const u32 dn = (u32)(pp_mix(h) >> sh_next) & ((1u << kb_next) - 1);
                __hip_atomic_fetch_add(&hn[(bk[u] << kb_next) | dn], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            }
        }
        __syncthreads();
        if constexpr (SRC == 1 && W > 0 && SORTED) {  // wpr == W here
            pp_tile_scan(hist, K, toff, (l32*)&tile_total);
            __syncthreads();
#pragma unroll
            for (u32 u = 0; u < UMAX; ++u) {
                if (!((m >> u) & 1)) continue;
                const u32 pos = toff[bk[u]] + rk[u];
#pragma unroll
                for (int w = 0; w < (W > 0 ? W : 1); ++w) stage[(size_t)pos * (W > 0 ? W : 1) + w] = rr[u].r[w];
                sbk[pos] = (u16)bk[u];
            }
            __syncthreads();
            constexpr u32 WW = W > 0 ? W : 1;
            const u32 nw = tile_total * WW;
            for (u32 q = threadIdx.x; q < nw; q += PP_NT) {
                const u32 j = q / WW, w = q - j * WW;
                const u32 b = sbk[j];
                u64 __attribute__((address_space(1)))* o = (u64 __attribute__((address_space(1)))*)(dst + (run[b] + (j - toff[b])) * rw);
                o[w] = stage[q];
            }
        } else {
#pragma unroll
            for (u32 u = 0; u < UMAX; ++u) {
                if (!((m >> u) & 1)) continue;
                const u64 di = run[bk[u]] + rk[u];
                u64 __attribute__((address_space(1)))* o = (u64 __attribute__((address_space(1)))*)(dst + di * rw);
                if constexpr (SRC == 1 && W > 0) {
#pragma unroll
                    for (int w = 0; w < W; ++w)
                        if ((u32)w < wpr) o[w] = rr[u].r[w];
                } else {
                    const l64* s = (const l64*)(scratch + ((size_t)threadIdx.x * U + u) * rw);
                    for (u32 w = 0; w < wpr; ++w) o[w] = s[w];
                }
            }
        }
        __syncthreads();
        for (u32 b = threadIdx.x; b < K; b += PP_NT) {
            run[b] += hist[b];
            hist[b] = 0;
        }
        __syncthreads();
    }
    // every unit of the next level is a whole destination partition: add this chunk's share
    for (u32 i = threadIdx.x; i < KN; i += PP_NT) {
        const u32 v = hn[i];
        if (v) atomicAdd(cnt_next + (u64)ch.group * KN + i, v);
    }
}

void launch_pp_scatter(hipStream_t s, const Spec* dspec, const Spec& hspec, const BatchDesc* batches, int src, int kind,
                       const u8* src_recs, const PPChunk* chunks, u32 n_chunks, u32 shift, u32 kbits, const u64* off,
                       const u64* part_off, u8* dst, u32* cnt_next, u32 sh_next, u32 kb_next) {
    if (!n_chunks) return;
    const u32 rw = kind ? hspec.pp_rw_state : hspec.pp_rw_raw;
    const u32 K = 1u << kbits;
    const u32 wpr = rw / 8;
    const int W = src == 0 ? 0 : (wpr == 1 ? 1 : wpr == 2 ? 2 : wpr == 4 ? 4 : wpr == 6 ? 6 : wpr == 8 ? 8 : 0);
    if (src == 0 || (K << kb_next) > PP_NEXT_HIST_MAX) cnt_next = nullptr;  // host checks: never taken
    // only wide fanouts: with few buckets a tile's runs are long already and the staging LDS costs
    // occupancy (level 3 at 32 buckets: 9.3 -> 10.3 ms sorted, C4)
    const int sorted = (src == 1 && W > 0 && K >= 128) ? 1 : 0;
    const size_t KN = cnt_next ? ((size_t)K << kb_next) : 0;
    const size_t TU = (size_t)PP_NT * pp_direct_u(W, rw);
    const size_t lds = 4 * (size_t)(K + (K & 1)) + 8 * (size_t)K +
                       (W == 0 ? (size_t)pp_direct_t(rw) * pp_direct_u(0, rw) * rw : 0) + 4 * (KN + (KN & 1)) +
                       (sorted ? TU * W * 8 + 2 * (TU + (TU & 1)) + 4 * (size_t)K : 0);
#define PP_SC(SR, WW, SO)                                                                                                     \
    hipLaunchKernelGGL((pp_scatter_direct_kernel<SR, WW, SO>), dim3(n_chunks), dim3(PP_NT), lds, s, dspec, batches, kind, src_recs, \
                       chunks, shift, kbits, off, part_off, dst, cnt_next, sh_next, kb_next)
#define PP_SC2(WW)                   \
    do {                             \
        if (sorted) PP_SC(1, WW, 1); \
        else PP_SC(1, WW, 0);        \
    } while (0)
    if (src == 0) {
        PP_SC(0, 0, 0);
    } else {
        switch (W) {
            case 1: PP_SC2(1); break;
            case 2: PP_SC2(2); break;
            case 4: PP_SC2(4); break;
            case 6: PP_SC2(6); break;
            case 8: PP_SC2(8); break;
            default: PP_SC(1, 0, 0); break;
        }
    }
#undef PP_SC2
#undef PP_SC
}

// ------------------------------------------------------------------------------------------
// Level 1 from raw columns, specialised (count and scatter in one template): the shapes of the
// high-cardinality benchmarks — fixed-width non-null keys and arguments with an optional
// `column <cmp> constant` predicate (ClickBench Q16/Q33), or one non-null String key with an
// optional string-constant predicate and COUNT(*) (Q13).  Every column value of U rows per thread
// is loaded before any LDS work (the loads overlap), the record is assembled in registers and
// stored straight to its run.  Same records, buckets and offsets as the generic kernels.
// ------------------------------------------------------------------------------------------
template <typename T>
__device__ __forceinline__ u64 pp_ldw(const u8* base, u64 i) { return (u64)gld<T>(base + i * sizeof(T)); }
__device__ __forceinline__ u64 pp_ld_width(const u8* base, u32 w, u64 i) {
    switch (w) {
        case 1: return pp_ldw<uint8_t>(base, i);
        case 2: return pp_ldw<uint16_t>(base, i);
        case 4: return pp_ldw<uint32_t>(base, i);
        default: return pp_ldw<u64>(base, i);
    }
}
__device__ __forceinline__ bool pp_fast_pred(const PPFast& F, u64 v) {
    const int t = F.ptype;
    int o;
    if (is_unsigned_t(t)) o = cmp3_u64(v, (u64)F.pconst);
    else o = cmp3_i64(pp_sext(t, v), F.pconst);
    return apply_cmp(F.pcmp, o);
}

// Tile-sorted stores (scatter, `sorted`): the tile's records are placed in LDS in bucket order
// (exclusive scan of the tile histogram + each record's rank) and written back by consecutive
// threads, so consecutive lanes store consecutive 8-byte words of one bucket's run — whole lines
// per wave instead of 64 scattered records per store instruction.  LDS (dynamic): staged words
// [NT * U * W] u64 | bucket of each staged record [NT * U] u16 | tile offsets [K] u32.
// rows per thread of a level-1 tile: C4 (W = 2) scatter at 1 / 2 / 4 -> 19.7-20.2 / 17.2-18.3 /
// 18.6-19.9 ms, step 64.0-65.2 at 2 against 65.0-66.6 at 4 (alternating runs on one box,
// scripts/gpu_cfg_variants.sh); the count 4.4 / 3.6 / 3.6 ms
__host__ __device__ constexpr int pp_l1_u(int W) { return W <= 4 ? 2 : 1; }
__host__ __device__ constexpr size_t pp_l1_sorted_lds(int W) {  // + the staged level-2 digits (u16 each)
    return (size_t)PP_NT * pp_l1_u(W) * W * 8 + (size_t)PP_NT * pp_l1_u(W) * 2 + 4 * (1u << PP_L1_BITS) +
           (size_t)PP_NT * pp_l1_u(W) * 2;
}

template <int COUNT, int W, int NC>
__global__ void __launch_bounds__(PP_NT) pp_l1_fixed_kernel(const PPFast F, const PPChunk* __restrict__ chunks, u32 shift,
                                                           u32* __restrict__ cnt, const u64* __restrict__ off,
                                                           const u64* __restrict__ part_off, u8* __restrict__ dst, int sorted) {
    constexpr u32 K = 1u << PP_L1_BITS;
    constexpr int U = pp_l1_u(W);  // rows per thread and tile
    __shared__ u32 hist[K];
    __shared__ u64 run[K];
    __shared__ u32 hist_total_;
    extern __shared__ __attribute__((aligned(16))) u64 l1_dyn[];
    l64* stage = (l64*)l1_dyn;
    l16* sbk = (l16*)(stage + (size_t)PP_NT * U * W);
    l32* toff = (l32*)(sbk + (size_t)PP_NT * U);
    l16* sdg = (l16*)(toff + K);
    const PPChunk ch = chunks[blockIdx.x];
    for (u32 b = threadIdx.x; b < K; b += PP_NT) {
        hist[b] = 0;
        if (!COUNT) run[b] = part_off[(u64)ch.group * K + b] + off[(u64)blockIdx.x * K + b];
    }
    uint16_t __attribute__((address_space(1)))* dig = (uint16_t __attribute__((address_space(1)))*)F.dig;
    __syncthreads();
    const u64 end = ch.start + ch.n;
    const u64 step = (u64)PP_NT * U;
    const u32 nload = COUNT ? F.nk : F.ncol;  // the count needs the key columns only
    u64 v[U][NC], pv[U];
    auto load = [&](u64 base) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const u64 i = base + (u64)u * PP_NT + threadIdx.x;
            const u64 ii = i < end ? i : ch.start;
#pragma unroll
            for (int c = 0; c < NC; ++c)
                if ((u32)c < nload) v[u][c] = pp_ld_width(F.ptr[c], F.width[c], ii);
            pv[u] = F.has_pred ? pp_ld_width(F.pptr, F.pwidth, ii) : 0;
        }
    };
    u32 bk[U], rk[U], dg[U], m = 0;
    RegRec<W> rec[U];
    // selection mask, bucket and (scatter) record of the tile at base from v / pv
    auto assemble = [&](u64 base) {
        m = 0;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const u64 i = base + (u64)u * PP_NT + threadIdx.x;
            if (i >= end || (F.has_pred && !pp_fast_pred(F, pv[u]))) continue;
            m |= 1u << u;
            u64 h = 0;
#pragma unroll
            for (int k = 0; k < W; ++k) rec[u].r[k] = 0;
#pragma unroll
            for (int c = 0; c < NC; ++c) {
                if ((u32)c >= nload) continue;
                u64 x = v[u][c];
                if (F.type[c] == DBG_FLOAT32 || F.type[c] == DBG_FLOAT64) x = canon_float_bits(F.type[c], x);
                if ((u32)c < F.nk) {
                    const u64 hx = hash_bits(F.type[c], x);
                    h = c == 0 ? hx : (h * NULL_HASH_VAL) ^ hx;
                }
                if (!COUNT) {  // place the value at its record offset (may straddle two words)
                    const u32 o = F.off[c], wi = o >> 3, sh = (o & 7) * 8;
#pragma unroll
                    for (int k = 0; k < W; ++k) {
                        if ((u32)k == wi) rec[u].r[k] |= x << sh;
                        if (sh && (u32)k == wi + 1 && sh + 8 * F.width[c] > 64) rec[u].r[k] |= x >> (64 - sh);
                    }
                }
            }
            const u64 mh = pp_mix(h);
            bk[u] = (u32)(mh >> shift) & (K - 1);
            dg[u] = (u32)(mh >> (shift - 16)) & 0xFFFF;
        }
    };
    if (COUNT) {
        for (u64 base = ch.start; base < end; base += step) {
            load(base);
            assemble(base);
#pragma unroll
            for (int u = 0; u < U; ++u)
                if ((m >> u) & 1) atomicAdd(&hist[bk[u]], 1u);
        }
    } else {
        // software pipeline: tile k + 1's column loads are in flight while tile k is ranked and
        // stored (three barriers per tile would otherwise each sit behind a memory latency)
        u64 base = ch.start;
        if (base < end) {
            load(base);
            assemble(base);
        }
        while (base < end) {
            const u64 nb = base + step;
            if (nb < end) load(nb);
#pragma unroll
            for (int u = 0; u < U; ++u)
                if ((m >> u) & 1) rk[u] = atomicAdd(&hist[bk[u]], 1u);
            __syncthreads();
            if (sorted) {
                if (threadIdx.x < 64) {  // wave 0: exclusive scan of the K-bucket tile histogram
                    constexpr u32 PER = K / 64;
                    u32 c[PER], t = 0;
#pragma unroll
                    for (u32 j = 0; j < PER; ++j) {
                        c[j] = hist[threadIdx.x * PER + j];
                        t += c[j];
                    }
                    u32 incl = t;
#pragma unroll
                    for (int d = 1; d < 64; d <<= 1) {
                        const u32 y = __shfl_up(incl, d);
                        if ((int)threadIdx.x >= d) incl += y;
                    }
                    u32 e = incl - t;
#pragma unroll
                    for (u32 j = 0; j < PER; ++j) {
                        toff[threadIdx.x * PER + j] = e;
                        e += c[j];
                    }
                    if (threadIdx.x == 63) hist_total_ = incl;
                }
                __syncthreads();
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    if (!((m >> u) & 1)) continue;
                    const u32 pos = toff[bk[u]] + rk[u];
#pragma unroll
                    for (int k = 0; k < W; ++k) stage[(size_t)pos * W + k] = rec[u].r[k];
                    sbk[pos] = (u16)bk[u];
                    sdg[pos] = (u16)dg[u];
                }
                __syncthreads();
                // word q of the tile's staged records -> consecutive threads, consecutive words
                const u32 nw = hist_total_ * F.wpr;
                for (u32 q = threadIdx.x; q < nw; q += PP_NT) {
                    const u32 j = q / F.wpr, k = q - j * F.wpr;
                    const u32 b = sbk[j];
                    const u64 di = run[b] + (j - toff[b]);
                    u64 __attribute__((address_space(1)))* o = (u64 __attribute__((address_space(1)))*)(dst + di * (8 * F.wpr));
                    o[k] = stage[(size_t)j * W + k];
                    if (dig && k == 0) dig[di] = sdg[j];  // the digit beside its record
                }
            } else {
#pragma unroll
                for (int u = 0; u < U; ++u) {
                    if (!((m >> u) & 1)) continue;
                    u64 __attribute__((address_space(1)))* o = (u64 __attribute__((address_space(1)))*)(dst + (run[bk[u]] + rk[u]) * (8 * F.wpr));
#pragma unroll
                    for (int k = 0; k < W; ++k)
                        if ((u32)k < F.wpr) o[k] = rec[u].r[k];
                    if (dig) dig[run[bk[u]] + rk[u]] = (uint16_t)dg[u];
                }
            }
            __syncthreads();
            for (u32 b = threadIdx.x; b < K; b += PP_NT) {
                run[b] += hist[b];
                hist[b] = 0;
            }
            __syncthreads();
            if (nb < end) assemble(nb);
            base = nb;
        }
    }
    if (COUNT) {
        __syncthreads();
        for (u32 b = threadIdx.x; b < K; b += PP_NT) cnt[(u64)blockIdx.x * K + b] = hist[b];
    }
}

// One non-null String key, COUNT-only records: [hash][klen = 1 + len][len][bytes] (6 words).
template <int COUNT>
__global__ void __launch_bounds__(PP_NT) pp_l1_str1_kernel(const PPFast F, const PPChunk* __restrict__ chunks, u32 shift,
                                                          u32* __restrict__ cnt, const u64* __restrict__ off,
                                                          const u64* __restrict__ part_off, u8* __restrict__ dst) {
    constexpr u32 K = 1u << PP_L1_BITS;
    constexpr int U = 4;
    __shared__ u32 hist[K];
    __shared__ u64 run[K];
    const PPChunk ch = chunks[blockIdx.x];
    for (u32 b = threadIdx.x; b < K; b += PP_NT) {
        hist[b] = 0;
        if (!COUNT) run[b] = part_off[(u64)ch.group * K + b] + off[(u64)blockIdx.x * K + b];
    }
    __syncthreads();
    const u64 end = ch.start + ch.n;
    for (u64 base = ch.start; base < end; base += (u64)PP_NT * U) {
        u64 a[U], e[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const u64 i = base + (u64)u * PP_NT + threadIdx.x;
            const u64 ii = i < end ? i : ch.start;
            a[u] = gld<u64>(F.soffs + ii);
            e[u] = gld<u64>(F.soffs + ii + 1);
        }
        u32 m = 0;
#pragma unroll
        for (int u = 0; u < U; ++u) {
            const u64 i = base + (u64)u * PP_NT + threadIdx.x;
            if (i >= end) continue;
            if (F.has_pred && !apply_cmp(F.pcmp, cmp3_bytes(F.sdata + a[u], e[u] - a[u], F.pstr, F.pstr_len))) continue;
            m |= 1u << u;
        }
        u32 bk[U], rk[U];
        u64 h[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (!((m >> u) & 1)) continue;
            h[u] = hash_bytes(F.sdata + a[u], e[u] - a[u]);
            bk[u] = (u32)(pp_mix(h[u]) >> shift) & (K - 1);
        }
        if (COUNT) {
#pragma unroll
            for (int u = 0; u < U; ++u)
                if ((m >> u) & 1) atomicAdd(&hist[bk[u]], 1u);
            continue;
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
            if ((m >> u) & 1) rk[u] = atomicAdd(&hist[bk[u]], 1u);
        __syncthreads();
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (!((m >> u) & 1)) continue;
            const u64 i = base + (u64)u * PP_NT + threadIdx.x;
            const u8* s = F.sdata + a[u];
            const u64 len = e[u] - a[u];
            u64 w[6] = {h[u], 0, 0, 0, 0, 0};
            if (1 + len > PP_BLOB) {
                w[1] = PP_KLEN_LONG;
                w[2] = ((u64)F.bid << 32) | (u64)(u32)i;
            } else {
                const u32 r1 = len < 6 ? (u32)len : 6;
                w[1] = (1 + len) | (len << 8) | (r1 ? (load_partial(s, r1) & width_mask(r1)) << 16 : 0);
#pragma unroll
                for (int j = 2; j < 6; ++j) {
                    const u64 q = 8 * j - 10;
                    if (len > q) {
                        const u32 r = len - q < 8 ? (u32)(len - q) : 8;
                        w[j] = load_partial(s + q, r) & width_mask(r);
                    }
                }
            }
            u64 __attribute__((address_space(1)))* o = (u64 __attribute__((address_space(1)))*)(dst + (run[bk[u]] + rk[u]) * 48);
#pragma unroll
            for (int j = 0; j < 6; ++j) o[j] = w[j];
        }
        __syncthreads();
        for (u32 b = threadIdx.x; b < K; b += PP_NT) {
            run[b] += hist[b];
            hist[b] = 0;
        }
        __syncthreads();
    }
    if (COUNT) {
        __syncthreads();
        for (u32 b = threadIdx.x; b < K; b += PP_NT) cnt[(u64)blockIdx.x * K + b] = hist[b];
    }
}

int launch_pp_l1_fast(hipStream_t s, const PPFast& F, int count, const PPChunk* chunks, u32 n_chunks, u32* cnt, const u64* off,
                      const u64* part_off, u8* dst) {
    if (!n_chunks) return 0;
    const u32 shift = 64 - PP_L1_BITS;
    if (F.kind == 2) {
        if (count) hipLaunchKernelGGL(pp_l1_str1_kernel<1>, dim3(n_chunks), dim3(PP_NT), 0, s, F, chunks, shift, cnt, off, part_off, dst);
        else hipLaunchKernelGGL(pp_l1_str1_kernel<0>, dim3(n_chunks), dim3(PP_NT), 0, s, F, chunks, shift, cnt, off, part_off, dst);
        return 0;
    }
    const int W = F.wpr <= 1 ? 1 : F.wpr <= 2 ? 2 : F.wpr <= 4 ? 4 : F.wpr <= 6 ? 6 : 8;
    // columns held per row: 4 (the benchmark shapes) or all 8 — fewer VGPRs, more waves
    const int sorted = 1;  // tile-sorted stores (C4 level 1: 26.5 -> 16.0 ms)
    const size_t dyn = count ? 0 : pp_l1_sorted_lds(W);
#define PP_L1F(C, WW)                                                                                                        \
    do {                                                                                                                      \
        if (F.ncol <= 4)                                                                                                      \
            hipLaunchKernelGGL((pp_l1_fixed_kernel<C, WW, 4>), dim3(n_chunks), dim3(PP_NT), dyn, s, F, chunks, shift, cnt, off, \
                               part_off, dst, sorted);                                                                        \
        else                                                                                                                  \
            hipLaunchKernelGGL((pp_l1_fixed_kernel<C, WW, 8>), dim3(n_chunks), dim3(PP_NT), dyn, s, F, chunks, shift, cnt, off, \
                               part_off, dst, sorted);                                                                        \
    } while (0)
#define PP_L1F_W(C)                      \
    switch (W) {                         \
        case 1: PP_L1F(C, 1); break;     \
        case 2: PP_L1F(C, 2); break;     \
        case 4: PP_L1F(C, 4); break;     \
        case 6: PP_L1F(C, 6); break;     \
        default: PP_L1F(C, 8); break;    \
    }
    if (count) {
        PP_L1F_W(1)
    } else {
        PP_L1F_W(0)
    }
#undef PP_L1F_W
#undef PP_L1F
    return 0;
}

// ------------------------------------------------------------------------------------------
// aggregate: one workgroup per final partition, an LDS table of `cap` slots
// [tag][key part][state words].  tag 0 = empty, 1 = being claimed, else (mix | 2).  A key whose
// probe window is full in this round overflows — consistently for all its records, since slots
// only ever fill — into the partition's region of the alternate buffer, aggregated in a further
// round once this round's groups are written.
// ------------------------------------------------------------------------------------------
u32 pp_agg_slots(const Spec& S) { return (u32)((PP_AGG_LDS - 256) / (8 * S.pp_sw + 2)); }

__device__ __forceinline__ u64 lds_ld_acq(l64* p) { return __hip_atomic_load(p, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP); }

__device__ __forceinline__ bool pp_long_equal(const Spec& S, const BatchDesc* batches, u64 ra, u64 rb) {
    const DCol* ka = batches[ref_bid(ra)].keys;
    const DCol* kb = batches[ref_bid(rb)].keys;
    for (int c = 0; c < S.n_keys; ++c)
        if (!cell_equal(ka[c], ref_row(ra), kb[c], ref_row(rb))) return false;
    return true;
}

// key part of a record == key part of a slot (LDS)
template <typename R>
__device__ __forceinline__ bool pp_key_eq(const Spec& S, const BatchDesc* batches, const l64* sk, const R& rk) {
    const u32 kw8 = S.pp_kw / 8;
    if (!S.pp_str) {
        for (u32 w = 0; w + 1 < kw8; ++w)
            if (sk[w] != rk.word(w)) return false;
        return sk[kw8 - 1] == (rk.word(kw8 - 1) & S.pp_klast_mask);
    }
    if (sk[0] != rk.word(0)) return false;  // group hash
    const u64 w1 = rk.word(1);
    const bool rl = (w1 & 0xff) == PP_KLEN_LONG, sl = (sk[1] & 0xff) == PP_KLEN_LONG;
    if (rl || sl) return rl && sl && pp_long_equal(S, batches, sk[2], rk.word(2));
    if (sk[1] != w1) return false;
    for (u32 w = 2; w < kw8; ++w)
        if (sk[w] != rk.word(w)) return false;
    return true;
}

// find or claim the slot of a record; -1 = no room in its probe window (overflow).  A claimed
// slot is appended to the partition's group list.
template <typename R>
__device__ __forceinline__ int pp_find(const Spec& S, const BatchDesc* batches, l64* slots, u32 cap, u32 sw, const R& rk, u64 pm,
                                       l16* list, u32* nlist) {
    const u32 kw8 = S.pp_kw / 8;
    const u64 tag = pm | 2;
    u32 pos = (u32)(((u64)(u32)pm * cap) >> 32);
    const u32 win = cap < PP_WINDOW ? cap : PP_WINDOW;
    for (u32 n = 0; n < win; ++n) {
        l64* e = slots + (size_t)pos * sw;
        u64 t = lds_ld_acq(e);
        if (t == 0) {
            u64 old = 0;
            __hip_atomic_compare_exchange_strong(e, &old, 1ULL, __ATOMIC_ACQUIRE, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
            if (old == 0) {  // claimed: key, initial states, then publish the tag
                for (u32 w = 0; w < kw8; ++w) e[1 + w] = rk.word(w) & (w + 1 == kw8 ? S.pp_klast_mask : ~0ULL);
                for (int w = 1; w <= S.n_words; ++w) e[kw8 + w] = S.slot_init[w];
                __hip_atomic_store(e, tag, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
                list[atomicAdd(nlist, 1u)] = (u16)pos;
                return (int)pos;
            }
            t = old;
        }
        while (t == 1) t = lds_ld_acq(e);  // the claimer publishes in straight-line code
        if (t == tag && pp_key_eq(S, batches, e + 1, rk)) return (int)pos;
        pos = pos + 1 == cap ? 0 : pos + 1;
    }
    return -1;
}

// accumulate_keys of one raw record into the slot states st (st[A.w0] = first word)
template <typename R>
__device__ __forceinline__ void pp_apply_rec(const Spec& S, wptr<AS_LDS> st, const R& rk) {
    u64 vm = ~0ULL;
    if (S.pp_avoff < S.pp_rw_raw) vm = rk.le(S.pp_avoff, min(8u, S.pp_rw_raw - S.pp_avoff));
    for (int a = 0; a < S.n_aggs; ++a) {
        const DAgg& A = S.aggs[a];
        if (A.arg_type >= 0 && S.pp_avbit[a] >= 0 && !((vm >> S.pp_avbit[a]) & 1)) continue;
        wptr<AS_LDS> w = st + A.w0;
        const u32 off = S.pp_aoff[a];
        const u32 aw = A.arg_type == DBG_BOOLEAN ? 1 : (A.arg_type >= 0 ? type_width(A.arg_type) : 0);
        switch (A.kind) {
            case DBG_AGG_COUNT: at_add<AS_LDS>(w, 1ULL); break;
            case DBG_AGG_SUM: case DBG_AGG_AVG: {
                if (A.sumk == SUMK_I64) at_add<AS_LDS>(w, (u64)pp_sext(A.arg_type, rk.le(off, aw)));
                else if (A.sumk == SUMK_F64) {
                    const u64 b = rk.le(off, aw);
                    at_addf<AS_LDS>(w, A.arg_type == DBG_FLOAT32 ? (double)__uint_as_float((u32)b) : __longlong_as_double((long long)b));
                } else {
                    add128<AS_LDS>(w, rk.le(off, 8), rk.le(off + 8, 8));
                }
                if (A.kind == DBG_AGG_AVG) at_add<AS_LDS>(w + (A.sumk == SUMK_I128 ? 2 : 1), 1ULL);
                break;
            }
            case DBG_AGG_MIN: case DBG_AGG_MAX: {
                const bool mn = A.kind == DBG_AGG_MIN;
                const u64 b = rk.le(off, aw < 8 ? aw : 8);  // Decimal128 (p <= 18): the low word
                if (A.mmk == MMK_I128) at_minmax128<AS_LDS>(w, b, rk.le(off + 8, 8), mn, S.err);
                else if (A.mmk == MMK_I64) at_minmax<AS_LDS>(w, (u64)pp_sext(A.arg_type, b), mn, true);
                else if (A.mmk == MMK_U64) at_minmax<AS_LDS>(w, b, mn, false);
                else
                    at_minmax<AS_LDS>(w, f64_order_key(A.arg_type == DBG_FLOAT32 ? (double)__uint_as_float((u32)b)
                                                                              : __longlong_as_double((long long)b)),
                                      mn, false);
                break;
            }
        }
        if (A.flag_bit >= 0) set_flag<AS_LDS>(st, S.flags_word, A.flag_bit);
    }
}

// write one group (slot key part + states) as output row `row` (fixed-width keys only)
__device__ __forceinline__ void pp_write_fixed_row(const Spec& S, const l64* e, u64 row, const OutDesc& out, u64* err) {
    const u32 kw8 = S.pp_kw / 8;
    const l8* k = (const l8*)(e + 1);
    for (int c = 0; c < S.n_keys; ++c) {
        const dbg_datatype& t = S.key_types[c];
        const u32 w = type_width(t.type);
        const bool v = !t.nullable || k[S.voff[c]] != 0;
        u64 lo = 0, hi = 0;
        if (t.type == DBG_DECIMAL128) {
            lo = lget(k, S.koff[c], 8);
            hi = lget(k, S.koff[c] + 8, 8);
        } else {
            lo = lget(k, S.koff[c], w);
        }
        write_bytes(out.key_data[c], row, w, lo, hi);
        if (out.key_valid[c]) out.key_valid[c][row] = v ? 1 : 0;
    }
    const u64* st = (const u64*)(e + kw8);
    for (int a = 0; a < S.n_aggs; ++a) write_agg(S, a, st, row, out, err);
}

template <typename R>
__device__ __forceinline__ void pp_store_rec(u8* dst, const R& rk, u32 rw) {
    for (u32 w = 0; w < rw / 8; ++w) ((u64*)dst)[w] = rk.word(w);
}

// One workgroup per final partition (grid-strided), an LDS table of `cap` slots
// [tag][key part][state words] plus the list of claimed slots.  tag 0 = empty, 1 = being claimed,
// else (mix | 2).  A key whose probe window is full in this round overflows — consistently for all
// its records, since slots only fill within a round — into the partition's region of the alternate
// buffer and is aggregated in a further round, after this round's groups are written.  W > 0: raw
// records of W words are held in registers, PP_AU per thread loaded together.
template <int MODE, int W>
__global__ void __launch_bounds__(PP_AGG_NT) pp_agg_kernel(const Spec* __restrict__ spec, const BatchDesc* __restrict__ batches,
                                                          u32 n_parts, const u64* __restrict__ raw_off, const u64* __restrict__ st_off,
                                                          u8* raw, u8* raw_alt, u8* st, u8* st_alt, u32 cap, PPAggOut out,
                                                          const u32* __restrict__ plist, u32 plist_cap) {
    extern __shared__ __attribute__((aligned(16))) u64 lds_raw[];
    const Spec& S = *spec;
    // plist: aggregate only the partitions plist[1 .. plist[0]] (those the record-centric kernel
    // spilled), numbered 0 .. plist[0] - 1 here
    if (plist) n_parts = min(n_parts, min(plist[0], plist_cap));  // (a count past the cap flagged ERR_OVF_LOST)
    auto pid = [&](u32 q) -> u32 { return plist ? plist[1 + q] : q; };
    const u32 sw = S.pp_sw, kw8 = S.pp_kw / 8, rwr = S.pp_rw_raw, rws = S.pp_rw_state;
    l64* slots = (l64*)lds_raw;
    l16* list = (l16*)(slots + (size_t)cap * sw);
    __shared__ u32 nlist, novf[2];
    __shared__ u64 gbase;
    for (u32 s = threadIdx.x; s < cap; s += PP_AGG_NT) slots[(size_t)s * sw] = 0;
    if (threadIdx.x == 0) nlist = novf[0] = novf[1] = 0;
    // Software pipeline over this workgroup's partitions p, p + G, p + 2G, ...: the first record tile
    // of a partition is loaded into registers two partitions ahead — buffer A serves p, p + 2G, ...,
    // buffer B p + G, p + 3G, ... — and reloaded as soon as it is consumed, so a partition's inserts
    // start on data that has had two partitions' worth of time to arrive (with one partition of
    // lead time the insert phase still waited on its own records).  Tiles of AU x NT records: the
    // final partitions hold ~0.45 x cap groups, fewer than 2 x NT for the usual record widths.
    constexpr int AU = W > 0 ? (W <= 2 ? 2 : 1) : 1;
    typedef RegRec<(W > 0 ? W : 1)> Tile[AU];
    auto part_range = [&](u32 q, u64& o0, u64& n) {
        o0 = (raw_off && q < n_parts) ? raw_off[pid(q)] : 0;
        n = (raw_off && q < n_parts) ? raw_off[pid(q) + 1] - o0 : 0;
    };
    auto load_tile = [&](RegRec<(W > 0 ? W : 1)>* rr, const u8* src, u64 o0, u64 n, u64 base) {
        if constexpr (W > 0) {
#pragma unroll
            for (int u = 0; u < AU; ++u) {
                const u64 i = base + (u64)u * PP_AGG_NT + threadIdx.x;
                if (i < n) {
                    const u8* rk = src + (o0 + i) * rwr;
#pragma unroll
                    for (int w = 0; w < W; ++w) rr[u].r[w] = gld<u64>(rk + 8 * w);
                }
            }
        }
    };
    Tile bufA, bufB;
    u64 a_r0, a_nr, b_r0, b_nr;
    part_range(blockIdx.x, a_r0, a_nr);
    load_tile(bufA, raw, a_r0, a_nr, 0);
    part_range(blockIdx.x + gridDim.x, b_r0, b_nr);
    load_tile(bufB, raw, b_r0, b_nr, 0);
    __syncthreads();
    const bool tr = kPhaseTrace && out.trace && (blockIdx.x & 63) == 0 && threadIdx.x == 0;
    u64 tm0 = tr ? __builtin_amdgcn_s_memrealtime() : 0;
    auto run_part = [&](u32 q, Tile& buf, u64& br0, u64& bnr) {
        const u32 p = pid(q);
        const u64 r0 = br0, s0 = st_off ? st_off[p] : 0;
        u64 nr = bnr, ns = st_off ? st_off[p + 1] - s0 : 0;
        u8 *rin = raw, *rout = raw_alt, *sin = st, *sout = st_alt;
        Tile cur;
#pragma unroll
        for (int u = 0; u < AU; ++u) cur[u] = buf[u];
        part_range(q + 2 * gridDim.x, br0, bnr);  // the buffer's next partition, loaded now
        load_tile(buf, raw, br0, bnr, 0);
        for (int round = 0;; ++round) {
            auto raw_one = [&](const auto& rk) {
                const u64 pm = pp_mix(pp_hash_of(S, rk));
                const int ls = pp_find(S, batches, slots, cap, sw, rk, pm, list, &nlist);
                if (ls >= 0) pp_apply_rec(S, (wptr<AS_LDS>)(slots + (size_t)ls * sw + kw8), rk);
                else pp_store_rec(rout + (r0 + atomicAdd(&novf[0], 1u)) * rwr, rk, rwr);
            };
            if constexpr (W > 0) {
                for (u64 base = 0; base < nr; base += (u64)PP_AGG_NT * AU) {
                    if (round || base) load_tile(cur, rin, r0, nr, base);  // round 0's first tile: prefetched
#pragma unroll
                    for (int u = 0; u < AU; ++u)
                        if (base + (u64)u * PP_AGG_NT + threadIdx.x < nr) raw_one(cur[u]);
                }
            } else {
                for (u64 i = threadIdx.x; i < nr; i += PP_AGG_NT) raw_one(GlbRec{rin + (r0 + i) * rwr});
            }
            for (u64 i = threadIdx.x; i < ns; i += PP_AGG_NT) {
                const GlbRec rk{sin + (s0 + i) * rws};
                const u64 pm = pp_mix(pp_hash_of(S, rk));
                const int ls = pp_find(S, batches, slots, cap, sw, rk, pm, list, &nlist);
                if (ls >= 0)
                    apply_state<AS_LDS, false, AS_GLB>(S, (wptr<AS_LDS>)(slots + (size_t)ls * sw + kw8),
                                                       (const u64*)(rk.p + S.pp_kw) - 1);
                else
                    pp_store_rec(sout + (s0 + atomicAdd(&novf[1], 1u)) * rws, rk, rws);
            }
            if (tr) { const u64 tm = __builtin_amdgcn_s_memrealtime(); atomicAdd((unsigned long long*)out.trace + 0, tm - tm0); tm0 = tm; }
            __syncthreads();
            if (tr) { const u64 tm = __builtin_amdgcn_s_memrealtime(); atomicAdd((unsigned long long*)out.trace + 1, tm - tm0); tm0 = tm; }
            if (threadIdx.x == 0) gbase = nlist ? atomicAdd((unsigned long long*)(out.tot + PPT_GROUPS), (unsigned long long)nlist) : 0;
            __syncthreads();
            if (tr) { const u64 tm = __builtin_amdgcn_s_memrealtime(); atomicAdd((unsigned long long*)out.trace + 2, tm - tm0); tm0 = tm; }
            // emit the claimed slots in claim order, clearing their tags for the next table
            const u32 ng = nlist;
            for (u32 k = threadIdx.x; k < ng; k += PP_AGG_NT) {
                l64* e = slots + (size_t)list[k] * sw;
                const u64 row = gbase + k;
                if (MODE == 0) {
                    if (row < out.cols.cap_groups) pp_write_fixed_row(S, e, row, out.cols, out.tot + PPT_ERR);
                } else if (row < out.grec_cap) {
                    u64* d = (u64*)(out.grec + row * rws);
                    for (u32 w = 0; w < kw8; ++w) d[w] = e[1 + w];
                    for (int w = 0; w < S.n_words; ++w) d[kw8 + w] = e[1 + kw8 + w];
                }
                e[0] = 0;
            }
            const u32 o0 = novf[0], o1 = novf[1];
            if (tr) { const u64 tm = __builtin_amdgcn_s_memrealtime(); atomicAdd((unsigned long long*)out.trace + 3, tm - tm0); tm0 = tm; }
            __syncthreads();
            if (threadIdx.x == 0) nlist = novf[0] = novf[1] = 0;
            __syncthreads();
            if (tr) {
                const u64 tm = __builtin_amdgcn_s_memrealtime();
                atomicAdd((unsigned long long*)out.trace + 4, tm - tm0);
                atomicAdd((unsigned long long*)out.trace + 5, 1ULL);
                atomicAdd((unsigned long long*)out.trace + 6, (unsigned long long)ng);
                tm0 = tm;
            }
            if (o0 == 0 && o1 == 0) break;
            if (threadIdx.x == 0) atomicAdd((unsigned long long*)(out.tot + PPT_ROUNDS), 1ULL);
            // the overflow, written to this partition's region of the alternate buffers, is the
            // next round's input; the consumed input region takes the round after's overflow
            u8* t0 = rin; rin = rout; rout = t0;
            u8* t1 = sin; sin = sout; sout = t1;
            nr = o0;
            ns = o1;
        }
    };
    for (u32 p = blockIdx.x; p < n_parts; p += 2 * gridDim.x) {
        run_part(p, bufA, a_r0, a_nr);
        if (p + gridDim.x < n_parts) run_part(p + gridDim.x, bufB, b_r0, b_nr);  // uniform
    }
}

// ------------------------------------------------------------------------------------------
// Record-centric aggregation of raw records (mostly-unique keys, ClickBench Q33).  The slot
// table above claims a slot per group — CAS, key copy, state init, publish, list append, and
// readers spinning on the publish — which for ~one record per group is all overhead.  Here a
// round's records sit in LDS first; a table of record indices (u32, 0 = empty) groups them: a
// record whose CAS wins leads its group, one that finds an equal key (compared in LDS, already
// there: no publish to wait for) joins that group; every record adds its contribution into the
// leader's state words, kept beside the records.  Leaders are then written out in LDS order.
// One workgroup per partition holds the partition's records in registers (PP_RC_RPT per thread)
// and aggregates it in 2^sub_bits rounds by the next hash bits, so partitions are 2^sub_bits
// times larger than one LDS table and the level-3 scatter disappears.
// ------------------------------------------------------------------------------------------
#define PP_RC_LDS (72 * 1024)  // two workgroups per CU
static u32 rc_tcap(u32 n) {
    u32 t = 64;
    while (t < 2 * n) t <<= 1;
    return t;
}
#define PP_RC_MAXN 8192  // records of one partition (its round bytes)
u32 pp_rc_records(const Spec& S) {
    const u32 per = 8 * (S.pp_rw_raw / 8) + 8 * (u32)S.n_words + 1 + 8;  // record + states + leader flag + 2 tags
    const u32 budget = PP_RC_LDS - 256 - PP_RC_MAXN;
    u32 n = budget / per;
    while (n > 64 && n * (8 * (S.pp_rw_raw / 8) + 8 * (u32)S.n_words + 1) + 4 * rc_tcap(n) > budget) --n;
    return n;
}
bool pp_rc_ok(const Spec& S) { return !S.pp_str && S.pp_rw_raw / 8 <= PP_RC_W && S.pp_rw_raw % 8 == 0; }

template <int W>
__device__ __forceinline__ bool rc_key_eq(const Spec& S, const RegRec<W>& a, const l64* b, u32 kw8) {
    bool eq = true;
#pragma unroll
    for (int w = 0; w < W; ++w) {
        if ((u32)w + 1 < kw8) eq &= a.r[w] == b[w];
        else if ((u32)w + 1 == kw8) eq &= ((a.r[w] ^ b[w]) & S.pp_klast_mask) == 0;
    }
    return eq;
}

template <int MODE, int W>
__global__ void __launch_bounds__(PP_AGG_NT) pp_agg_rc_kernel(const Spec* __restrict__ spec, const BatchDesc* __restrict__ batches,
                                                             u32 n_parts, const u64* __restrict__ raw_off, const u8* __restrict__ raw,
                                                             u32 sub_shift, u32 sub_bits, u32 rcap, u32 tcap, PPAggOut out,
                                                             u32* __restrict__ spill, u32 spill_cap) {
    extern __shared__ __attribute__((aligned(16))) u64 lds_raw[];
    const Spec& S = *spec;
    const u32 kw8 = S.pp_kw / 8, nw = (u32)S.n_words;
    l64* recs = (l64*)lds_raw;                       // [rcap][W]
    l64* acc = recs + (size_t)rcap * W;              // [rcap][nw]
    l32* tags = (l32*)(acc + (size_t)rcap * nw);     // [tcap]
    l8* lead = (l8*)(tags + tcap);                   // [rcap]
    l8* subid = lead + rcap;                         // [PP_RC_MAXN] round of every record of the partition
    __shared__ u32 cnt, nlead, rcnt[32];
    __shared__ u32 wsum[PP_AGG_NT / 64];
    __shared__ u64 gbase;
    const u32 tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    const u32 smask = (1u << sub_bits) - 1;
    auto spill_part = [&](u32 p) {
        const u32 k = atomicAdd(spill, 1u);
        if (k < spill_cap) spill[1 + k] = p;
        else atomicOr((unsigned long long*)(out.tot + PPT_ERR), (unsigned long long)ERR_OVF_LOST);
    };
    for (u32 p = blockIdx.x; p < n_parts; p += gridDim.x) {
        const u64 o0 = raw_off[p], n = raw_off[p + 1] - o0;
        const u8* base = raw + o0 * (8 * W);
        if (n > PP_RC_MAXN) {  // larger than the round table can index: the slot-table kernel
            if (tid == 0) spill_part(p);
            continue;
        }
        // every record's round (hash bits below the partition's), counted per round
        if (tid < 32) rcnt[tid] = 0;
        __syncthreads();
        for (u32 i = tid; i < (u32)n; i += PP_AGG_NT) {
            RegRec<W> rk;
#pragma unroll
            for (int w = 0; w < W; ++w) rk.r[w] = gld<u64>(base + (u64)i * (8 * W) + 8 * w);
            const u32 sb = (u32)(pp_mix(pp_hash_of(S, rk)) >> sub_shift) & smask;
            subid[i] = (u8)sb;
            atomicAdd(&rcnt[sb], 1u);
        }
        __syncthreads();
        u32 mx = 0;
        for (u32 x = 0; x <= smask; ++x) mx = max(mx, rcnt[x]);
        if (mx > rcap) {  // a round does not fit one LDS table: decided before any group is written
            if (tid == 0) spill_part(p);
            __syncthreads();
            continue;
        }
        for (u32 sb = 0; sb <= smask; ++sb) {
            if (tid == 0) cnt = nlead = 0;
            for (u32 j = tid; j < tcap; j += PP_AGG_NT) tags[j] = 0;
            __syncthreads();
            // this round's records -> LDS (re-read: the partition was just streamed, L2 / MALL)
            for (u32 i = tid; i < (u32)n; i += PP_AGG_NT) {
                if (subid[i] != sb) continue;
                const u32 k = atomicAdd(&cnt, 1u);
#pragma unroll
                for (int w = 0; w < W; ++w) recs[(size_t)k * W + w] = gld<u64>(base + (u64)i * (8 * W) + 8 * w);
                for (u32 w = 0; w < nw; ++w) acc[(size_t)k * nw + w] = S.slot_init[1 + w];
                lead[k] = 0;
            }
            __syncthreads();
            const u32 m = cnt;  // <= rcap (checked above)
            // group: the table holds record indices + 1; placement mixes the key words only
            for (u32 me = tid; me < m; me += PP_AGG_NT) {
                RegRec<W> rk;
#pragma unroll
                for (int w = 0; w < W; ++w) rk.r[w] = recs[(size_t)me * W + w];
                u64 hm = 0;
#pragma unroll
                for (int w = 0; w < W; ++w)
                    if ((u32)w < kw8) hm = slot_mix(hm ^ ((u32)w + 1 == kw8 ? rk.r[w] & S.pp_klast_mask : rk.r[w]));
                u32 pos = (u32)hm & (tcap - 1);
                u32 leader = me;
                for (u32 probe = 0; probe < tcap; ++probe) {
                    u32 old = 0;
                    __hip_atomic_compare_exchange_strong(tags + pos, &old, me + 1, __ATOMIC_RELAXED, __ATOMIC_RELAXED,
                                                         __HIP_MEMORY_SCOPE_WORKGROUP);
                    if (old == 0) {
                        lead[me] = 1;
                        break;
                    }
                    if (rc_key_eq<W>(S, rk, recs + (size_t)(old - 1) * W, kw8)) {
                        leader = old - 1;
                        break;
                    }
                    pos = (pos + 1) & (tcap - 1);
                }
                pp_apply_rec(S, (wptr<AS_LDS>)(acc + (size_t)leader * nw) - 1, rk);
            }
            __syncthreads();
            u32 mine = 0;
            for (u32 j = tid; j < m; j += PP_AGG_NT) mine += lead[j];
            if (mine) atomicAdd(&nlead, mine);
            __syncthreads();
            if (tid == 0) gbase = nlead ? atomicAdd((unsigned long long*)(out.tot + PPT_GROUPS), (unsigned long long)nlead) : 0;
            __syncthreads();
            // leaders out in slot order: row = gbase + leaders among smaller slots
            u32 carry = 0;
            for (u32 j0 = 0; j0 < m; j0 += PP_AGG_NT) {
                const u32 j = j0 + tid;
                const bool isl = j < m && lead[j];
                const u64 bl = __ballot(isl);
                if (lane == 0) wsum[wv] = (u32)__popcll(bl);
                __syncthreads();
                u32 before = carry, all = 0;
                for (u32 x = 0; x < PP_AGG_NT / 64; ++x) {
                    if (x < wv) before += wsum[x];
                    all += wsum[x];
                }
                before += (u32)__popcll(bl & ((1ULL << lane) - 1));
                if (isl) {
                    const u64 row = gbase + before;
                    const l64* kp = recs + (size_t)j * W;
                    const u64* st = (const u64*)(acc + (size_t)j * nw) - 1;  // st[w0] = first state word
                    if (MODE == 0) {
                        if (row < out.cols.cap_groups) {
                            const l8* k = (const l8*)kp;
                            for (int c = 0; c < S.n_keys; ++c) {
                                const dbg_datatype& t = S.key_types[c];
                                const u32 wd = type_width(t.type);
                                const bool v = !t.nullable || k[S.voff[c]] != 0;
                                u64 lo = 0, hi = 0;
                                if (t.type == DBG_DECIMAL128) {
                                    lo = lget(k, S.koff[c], 8);
                                    hi = lget(k, S.koff[c] + 8, 8);
                                } else {
                                    lo = lget(k, S.koff[c], wd);
                                }
                                write_bytes(out.cols.key_data[c], row, wd, lo, hi);
                                if (out.cols.key_valid[c]) out.cols.key_valid[c][row] = v ? 1 : 0;
                            }
                            for (int a = 0; a < S.n_aggs; ++a) write_agg(S, a, st, row, out.cols, out.tot + PPT_ERR);
                        }
                    } else if (row < out.grec_cap) {
                        u64* d = (u64*)(out.grec + row * S.pp_rw_state);
                        for (u32 w = 0; w < kw8; ++w) d[w] = (w + 1 == kw8) ? (kp[w] & S.pp_klast_mask) : kp[w];
                        for (u32 w = 0; w < nw; ++w) d[kw8 + w] = acc[(size_t)j * nw + w];
                    }
                }
                carry += all;
                __syncthreads();
            }
        }
    }
}

void launch_pp_agg_rc(hipStream_t s, const Spec* dspec, const Spec& hspec, const BatchDesc* batches, int mode, u32 n_parts,
                      const u64* raw_off, const u8* raw, u32 sub_shift, u32 sub_bits, const PPAggOut& out, u32* spill,
                      u32 spill_cap) {
    if (!n_parts) return;
    const u32 rcap = pp_rc_records(hspec), tcap = rc_tcap(rcap);
    const u32 W = hspec.pp_rw_raw / 8;
    const size_t lds = (size_t)rcap * (8 * W + 8 * (u32)hspec.n_words + 1) + 4 * (size_t)tcap + PP_RC_MAXN + 16;
    const u32 grid = n_parts < 16384 ? n_parts : 16384;
#define PP_RC_LAUNCH(M, WW)                                                                                                  \
    hipLaunchKernelGGL((pp_agg_rc_kernel<M, WW>), dim3(grid), dim3(PP_AGG_NT), lds, s, dspec, batches, n_parts, raw_off, raw, \
                       sub_shift, sub_bits, rcap, tcap, out, spill, spill_cap)
#define PP_RC_W_(M)                          \
    switch (W) {                            \
        case 1: PP_RC_LAUNCH(M, 1); break;  \
        case 2: PP_RC_LAUNCH(M, 2); break;  \
        case 3: PP_RC_LAUNCH(M, 3); break;  \
        default: PP_RC_LAUNCH(M, 4); break; \
    }
    if (mode == 0) {
        PP_RC_W_(0)
    } else {
        PP_RC_W_(1)
    }
#undef PP_RC_W_
#undef PP_RC_LAUNCH
}

void launch_pp_agg(hipStream_t s, const Spec* dspec, const Spec& hspec, const BatchDesc* batches, int mode, u32 n_parts,
                   const u64* raw_off, const u64* st_off, u8* raw, u8* raw_alt, u8* st, u8* st_alt, const PPAggOut& out,
                   const u32* plist, u32 plist_cap) {
    if (!n_parts) return;
    const u32 cap = pp_agg_slots(hspec);
    const size_t lds = (size_t)cap * (hspec.pp_sw * 8 + 2);
    u32 grid = n_parts < 8192 ? n_parts : 8192;
    if (plist) grid = std::min<u32>(grid, std::max<u32>(plist_cap, 1));
    const u32 wpr = hspec.pp_rw_raw / 8;  // record buffers carry >= 64 bytes of slack: W may round up
    const int W = wpr <= 1 ? 1 : wpr <= 2 ? 2 : wpr <= 4 ? 4 : wpr <= 6 ? 6 : wpr <= 8 ? 8 : 0;
#define PP_AGG_LAUNCH(M, WW)                                                                                        \
    hipLaunchKernelGGL((pp_agg_kernel<M, WW>), dim3(grid), dim3(PP_AGG_NT), lds, s, dspec, batches, n_parts, raw_off, \
                       st_off, raw, raw_alt, st, st_alt, cap, out, plist, plist_cap)
#define PP_AGG_W(M)                                  \
    switch (W) {                                     \
        case 1: PP_AGG_LAUNCH(M, 1); break;          \
        case 2: PP_AGG_LAUNCH(M, 2); break;          \
        case 4: PP_AGG_LAUNCH(M, 4); break;          \
        case 6: PP_AGG_LAUNCH(M, 6); break;          \
        case 8: PP_AGG_LAUNCH(M, 8); break;          \
        default: PP_AGG_LAUNCH(M, 0); break;         \
    }
    if (mode == 0) {
        PP_AGG_W(0)
    } else {
        PP_AGG_W(1)
    }
#undef PP_AGG_W
#undef PP_AGG_LAUNCH
}

// ------------------------------------------------------------------------------------------
// Specialised aggregation of raw records (pp_agg_spec_kernel).
//
// The generic kernel above interprets the Spec per record: a loop over the aggregates with a
// switch on kind, argument width and type, a generic row writer, and a slot-table claim that
// initialises states and then applies the record with LDS atomics.  This kernel covers the class
// of mostly-unique GROUP BYs the partitioned payload exists for — one or two fixed-width
// non-nullable integer keys (<= 16 key bytes), up to PS_MAXA COUNT / SUM / AVG / MIN / MAX over
// non-nullable integer arguments — with the record's word count W a template parameter (the
// registers that hold a partition) and the rest a uniform descriptor (PsDesc: key types and
// widths, per aggregate its kind, argument type, offset and slot word), built on the host from the
// Spec and checked against the raw-record packing of build_spec:
//   * a slot is [key words][row count][one value word per SUM / AVG / MIN / MAX]: AVG's count and
//     COUNT are the same row count (arguments are non-nullable), so an AVG costs one word;
//   * a claimer initialises the slot from its own record (count 1, values = its arguments) before
//     publishing the tag: a new group costs no LDS atomics, a repeat one add / min / max per word;
//   * probes read a dense u32 tag array (one LDS word per probe step), the key words only on a
//     tag match;
//   * claimed slots join the output list with one LDS add per wave (ballot), not one per lane;
//   * a partition (up to PP_SPEC_NT x RPT records) is loaded into registers once and aggregated in
//     2^sub_bits rounds selected by the hash bits below the partition's, so a partition holds
//     2^sub_bits LDS tables' worth of groups and the level-3 scatter is gone (AGG/
//     transform_aggregate_final.rs:71-156 aggregates one bucket per task the same way).
// A record whose probe window is full stays pending and is inserted into the emptied table in
// a further mini-round (consistent per key: slots only fill within a mini-round).  Partitions
// larger than the register budget are listed in `spill` for the generic kernel.
// ------------------------------------------------------------------------------------------
enum { PS_COUNT = 1, PS_SUM = 2, PS_AVG = 3, PS_MIN = 4, PS_MAX = 5 };
#define PS_MAXA 4
struct PsDesc {
    u32 nk;                 // keys (1 or 2), packed at bytes [0, kb0) and [kb0, kb0 + kb1)
    int32_t kt[2];          // their types (the group hash's per-type mixer)
    u32 kb0, kb1;           // their widths
    u32 k1w, k1s;           // key 1 as a shift pair: record word and bit offset (it may straddle into the next word)
    u64 km0, km1;           // value masks of key 0 and key 1
    u32 hc;                 // hash mixer classes of the keys (ps_hclass): hc0 * 5 + hc1, hc1 = 4 for one key
    u32 kw;                 // key words (1 or 2)
    u64 klast;              // key bytes of the last key word
    u32 na;                 // aggregates
    u32 bw;                 // slot body words: key words, row count, one word per valued aggregate
    u32 rec_bytes;          // state record bytes (MODE 1): key words + the Spec's state words
    int32_t kind[PS_MAXA];  // PS_COUNT .. PS_MAX
    int32_t at[PS_MAXA];    // argument type (valued aggregates)
    u32 aoff[PS_MAXA];      // argument byte offset in the raw record
    u32 aw[PS_MAXA];        // argument width
    u32 xw[PS_MAXA];        // the argument as a shift pair: record word, bit offset in it (arguments
    u32 xs[PS_MAXA];        // are aligned to their width, so never straddle a word), and the
    u32 xe[PS_MAXA];        // shift that extends it (64 - 8 x width) — sign- or zero- per xsg
    u32 xsg[PS_MAXA];
    u32 vw[PS_MAXA];        // slot word of the aggregate's value
    u32 rw[PS_MAXA];        // result column width
};
__host__ __device__ constexpr u32 ps_tw(int t) {
    return (t == DBG_INT8 || t == DBG_UINT8) ? 1u
           : (t == DBG_INT16 || t == DBG_UINT16) ? 2u
           : (t == DBG_INT32 || t == DBG_UINT32 || t == DBG_DATE) ? 4u : 8u;
}
__host__ __device__ constexpr bool ps_signed(int t) { return !(t == DBG_UINT8 || t == DBG_UINT16 || t == DBG_UINT32 || t == DBG_UINT64); }

__device__ __forceinline__ u64 ps_ext(u64 v, int t) {  // argument bits -> the 64-bit addend / min-max operand
    const u32 w = ps_tw(t);
    if (w == 8) return v;
    v &= (1ULL << (8 * w)) - 1;
    if (ps_signed(t) && ((v >> (8 * w - 1)) & 1)) v |= ~((1ULL << (8 * w)) - 1);
    return v;
}

// LDS of one workgroup: [tags u32 cap][body u64 cap x BW][list u16 cap][stage: words u64 PS_STAGE x W,
// slot hash u32 PS_STAGE, origin u16 PS_STAGE][pending u32 PP_AGG_NT]
#define PS_STAGE 1024
__host__ __device__ constexpr size_t ps_lds_bytes(u32 cap, u32 bw, u32 w, u32 nt) {
    return 8 * (size_t)((cap + 1) / 2) + (size_t)cap * 8 * bw + 2 * (size_t)((cap + 3) & ~3u) + (size_t)PS_STAGE * (8 * w + 4 + 2) +
           4 * (size_t)nt;
}

// one result cell: stores through an address-space-1 view (a generic pointer compiles to flat
// stores, which count against lgkmcnt: every LDS wait of the emit loop would then drain them)
__device__ __forceinline__ void ps_store(void* dst, u64 row, u32 w, u64 v) {
    typedef __attribute__((address_space(1))) u8 g8;
    g8* p = (g8*)dst + row * w;
    if (w == 8) *(__attribute__((address_space(1))) u64*)p = v;
    else if (w == 4) *(__attribute__((address_space(1))) u32*)p = (u32)v;
    else if (w == 2) *(__attribute__((address_space(1))) uint16_t*)p = (uint16_t)v;
    else *p = (u8)v;
}

// The group hash's per-type mixer (hash_bits) in four classes: sign-extended 8 / 16 / 32-bit
// values, and the raw 64-bit pattern (64-bit and unsigned types).  The slot hashes of a
// partition's records are computed under ONE uniform dispatch on the key classes (a per-record
// switch on the runtime key type made the hash phase a chain of branches: 2.6 -> 8.7 us a partition).
__host__ __device__ constexpr int ps_hclass(int t) {
    return t == DBG_INT8 ? 0 : (t == DBG_INT16 ? 1 : ((t == DBG_INT32 || t == DBG_DATE) ? 2 : 3));
}
template <int C>
__device__ __forceinline__ u64 ps_hmix(u64 b) {
    if (C == 0) return hash_prim((u64)(i64)(int8_t)b);
    if (C == 1) return hash_prim((u64)(i64)(int16_t)b);
    if (C == 2) return hash_prim((u64)(i64)(int32_t)b);
    return hash_prim(b);
}
template <int W, int RPT, int C0, int C1>
__device__ __forceinline__ void ps_hash_all(const PsDesc& D, const RegRec<W>* rr, u32* lo) {
#pragma unroll
    for (int u = 0; u < RPT; ++u) {
        u64 h = ps_hmix<C0>(rr[u].r[0] & D.km0);
        if (C1 < 4) {
            u64 k1 = rr[u].word(D.k1w) >> D.k1s;
            if (D.k1s && W > 1) k1 |= rr[u].word(D.k1w + 1) << (64 - D.k1s);
            h = (h * NULL_HASH_VAL) ^ ps_hmix<C1 < 4 ? C1 : 3>(k1 & D.km1);
        }
        lo[u] = (u32)pp_mix(h);
    }
}
template <int W, int RPT, int C0>
__device__ __forceinline__ void ps_hash_c1(const PsDesc& D, const RegRec<W>* rr, u32* lo) {
    switch (D.hc % 5) {
        case 0: ps_hash_all<W, RPT, C0, 0>(D, rr, lo); break;
        case 1: ps_hash_all<W, RPT, C0, 1>(D, rr, lo); break;
        case 2: ps_hash_all<W, RPT, C0, 2>(D, rr, lo); break;
        case 3: ps_hash_all<W, RPT, C0, 3>(D, rr, lo); break;
        default: ps_hash_all<W, RPT, C0, 4>(D, rr, lo); break;
    }
}
template <int W, int RPT>
__device__ __forceinline__ void ps_hash(const PsDesc& D, const RegRec<W>* rr, u32* lo) {
    switch (D.hc / 5) {
        case 0: ps_hash_c1<W, RPT, 0>(D, rr, lo); break;
        case 1: ps_hash_c1<W, RPT, 1>(D, rr, lo); break;
        case 2: ps_hash_c1<W, RPT, 2>(D, rr, lo); break;
        default: ps_hash_c1<W, RPT, 3>(D, rr, lo); break;
    }
}

// argument a of a register record, extended to 64 bits (the sum addend / min-max operand)
template <int W>
__device__ __forceinline__ u64 ps_arg(const PsDesc& D, const RegRec<W>& r, u32 a) {
    const u64 x = r.word(D.xw[a]) >> D.xs[a];
    return D.xsg[a] ? (u64)((i64)(x << D.xe[a]) >> D.xe[a]) : ((x << D.xe[a]) >> D.xe[a]);
}

template <int MODE, int W, int RPT, int SNT>
__global__ void __launch_bounds__(SNT, SNT / 256) pp_agg_desc_kernel(const PsDesc D, u32 n_parts, const u64* __restrict__ raw_off,
                                                               const u8* __restrict__ raw, u32 sub_bits, u32 cap, PPAggOut out,
                                                               u32* __restrict__ spill, u32 spill_cap) {
    static_assert(RPT < 32, "per-lane record mask");
    extern __shared__ __attribute__((aligned(16))) u64 lds_raw[];
    const u32 KW = D.kw, BW = D.bw;
    l32* tags = (l32*)lds_raw;                                     // [cap] 0 empty, 1 being claimed, else tag
    l64* body = (l64*)lds_raw + (cap + 1) / 2;                     // [cap][BW]
    l16* list = (l16*)(body + (size_t)cap * BW);                   // claimed slots of the round
    l64* sw_ = (l64*)(list + ((cap + 3) & ~3u));                   // staged records [PS_STAGE][W]
    l32* slo = (l32*)(sw_ + (size_t)PS_STAGE * W);                 // their slot hash bits
    l16* sorg = (l16*)(slo + PS_STAGE);                            // their origin (thread << 4 | register index)
    l32* pend = (l32*)(((uintptr_t)(sorg + PS_STAGE) + 3) & ~(uintptr_t)3);  // [SNT] probe-window misses
    __shared__ u32 nlist, scount, anyw[3];
    __shared__ u64 gbase;
    const u32 tid = threadIdx.x, lane = tid & 63;
    // Barriers order LDS only: the output stores and the next partition's prefetched loads stay in
    // flight across them (__syncthreads' workgroup fence would wait for every outstanding global
    // access — the prefetch included).
    auto lds_barrier = [] { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); };
    // block-wide OR over three rotating LDS words: call c clears the word call c + 1 votes into
    // before its barrier (that word was last read in call c - 2, before call c - 1's barrier)
    u32 anyc = 0;
    auto block_any = [&](bool v) -> bool {
        const u32 q = anyc % 3;
        if (tid == 0) anyw[(q + 1) % 3] = 0;
        if (__ballot(v) && lane == 0) atomicOr(&anyw[q], 1u);
        lds_barrier();
        ++anyc;
        return anyw[q] != 0;
    };
    // key word w of a record, masked to the key bytes
    auto kword = [&](const RegRec<W>& r, u32 w) -> u64 { return w + 1 == KW ? (r.r[w] & D.klast) : r.r[w]; };
    const u32 smask = (1u << sub_bits) - 1;
    const u32 win = cap < PP_WINDOW ? cap : PP_WINDOW;
    // EXPERIMENT (TRACE=1 build, DBG_X_PPTRACE): phase times of sampled workgroups, thread 0
    const bool tr = kPhaseTrace && out.trace && (blockIdx.x & 15) == 0 && tid == 0;
    u64 tm0 = tr ? __builtin_amdgcn_s_memrealtime() : 0;
    auto tick = [&](int slot) {
        if (tr) {
            const u64 tm = __builtin_amdgcn_s_memrealtime();
            atomicAdd((unsigned long long*)out.trace + slot, tm - tm0);
            tm0 = tm;
        }
    };
    for (u32 j = tid; j < cap; j += SNT) tags[j] = 0;
    pend[tid] = 0;
    if (tid == 0) {
        nlist = scount = 0;
        anyw[0] = anyw[1] = anyw[2] = 0;
    }
    lds_barrier();
    // one staged record into the table; false = no room in its probe window
    auto insert = [&](u32 k) -> bool {
        RegRec<W> rk;
#pragma unroll
        for (int w = 0; w < W; ++w) rk.r[w] = sw_[(size_t)k * W + w];
        const u32 lo = slo[k];
        const u32 tag = (lo & ~3u) | 2u;
        u32 pos = (u32)(((u64)lo * cap) >> 32);
        bool claimed = false;
        int at = -1;
        for (u32 q = 0; q < win; ++q) {
            l32* tp = tags + pos;
            u32 t = __hip_atomic_load(tp, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
            if (t == 0) {
                u32 old = 0;
                __hip_atomic_compare_exchange_strong(tp, &old, 1u, __ATOMIC_ACQUIRE, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
                if (old == 0) {  // claimed: key words, the record's own contribution, then the tag
                    l64* e = body + (size_t)pos * BW;
#pragma unroll
                    for (u32 w = 0; w < 2; ++w)
                        if (w < KW) e[w] = kword(rk, w);
                    e[KW] = 1;
#pragma unroll
                    for (u32 a = 0; a < PS_MAXA; ++a)
                        if (a < D.na && D.kind[a] != PS_COUNT) e[D.vw[a]] = ps_arg<W>(D, rk, a);
                    __hip_atomic_store(tp, tag, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
                    claimed = true;
                    at = (int)pos;
                    break;
                }
                t = old;
            }
            while (t == 1) t = __hip_atomic_load(tp, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
            if (t == tag) {
                l64* e = body + (size_t)pos * BW;
                bool eq = true;
#pragma unroll
                for (u32 w = 0; w < 2; ++w)
                    if (w < KW) eq &= e[w] == kword(rk, w);
                if (eq) {
                    at_add<AS_LDS>((wptr<AS_LDS>)(e + KW), 1ULL);
#pragma unroll
                    for (u32 a = 0; a < PS_MAXA; ++a) {
                        if (a >= D.na || D.kind[a] == PS_COUNT) continue;
                        const u64 v = ps_arg<W>(D, rk, a);
                        wptr<AS_LDS> vp = (wptr<AS_LDS>)(e + D.vw[a]);
                        if (D.kind[a] == PS_SUM || D.kind[a] == PS_AVG) at_add<AS_LDS>(vp, v);
                        else at_minmax<AS_LDS>(vp, v, D.kind[a] == PS_MIN, ps_signed(D.at[a]));
                    }
                    at = (int)pos;
                    break;
                }
            }
            pos = pos + 1 == cap ? 0 : pos + 1;
        }
        // new groups join the round's list: one LDS add per wave (called with the wave converged)
        const u64 m = __ballot(claimed);
        if (m) {
            const u32 lead = (u32)__ffsll((long long)m) - 1;
            u32 b = 0;
            if (lane == lead) b = atomicAdd(&nlist, (u32)__popcll(m));
            b = __shfl(b, (int)lead);
            if (claimed) list[b + (u32)__popcll(m & ((1ULL << lane) - 1))] = (u16)at;
        }
        return at >= 0;
    };
    // A partition's records live in registers (RPT per lane, loaded with buffer loads: one 32-bit
    // lane offset, the range check returning zeros past the partition), and the next partition of
    // this workgroup is loaded into a second register set while the current one is aggregated.
    typedef u32 v2u32 __attribute__((ext_vector_type(2)));
    auto load_part = [&](u32 q, RegRec<W>* dst, u64& n_out) {
        n_out = 0;
        if (q >= n_parts) return;
        const u64 o0 = raw_off[q], n = raw_off[q + 1] - o0;
        n_out = n;
        if (n == 0 || n > (u64)SNT * RPT) return;
        const u8* base = raw + o0 * (8 * W);
        const auto rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, (int)(n * (8 * W)), 0x00020000);
#pragma unroll
        for (int u = 0; u < RPT; ++u)
#pragma unroll
            for (int w = 0; w < W; ++w) {
                const v2u32 v = __builtin_amdgcn_raw_buffer_load_b64(rsrc, tid * (8 * W) + 8 * w, u * (SNT * 8 * W), 0);
                dst[u].r[w] = (u64)v.x | ((u64)v.y << 32);
            }
    };
    RegRec<W> nxt[RPT];
    u64 n_nxt;
    load_part(blockIdx.x, nxt, n_nxt);
    for (u32 p = blockIdx.x; p < n_parts; p += gridDim.x) {
        RegRec<W> rr[RPT];
#pragma unroll
        for (int u = 0; u < RPT; ++u) rr[u] = nxt[u];
        const u64 n = n_nxt;
        load_part(p + gridDim.x, nxt, n_nxt);  // in flight during this partition's rounds
        if (n == 0) continue;
        if (n > (u64)SNT * RPT) {  // uniform: the generic kernel takes it
            if (tid == 0) {
                const u32 k = atomicAdd(spill, 1u);
                if (k < spill_cap) spill[1 + k] = p;
                else atomicOr((unsigned long long*)(out.tot + PPT_ERR), (unsigned long long)ERR_OVF_LOST);
            }
            continue;
        }
        if (tr) atomicAdd((unsigned long long*)out.trace + 5, 1ULL);
        // slot hash bits; a record's round is the low sub_bits of its hash (the partition is the
        // top bits, the slot position the top bits of the low word)
        u32 lo[RPT];  // slot hash bits; the round is the low sub_bits
        ps_hash<W, RPT>(D, rr, lo);
        // records this lane holds: register u is row u * SNT + tid (32-bit: n <= SNT * RPT; a 64-bit
        // row test per register had the compiler keep RPT 64-bit row constants live, and spill them)
        const u32 valid = (1u << ((u32)n > tid ? ((u32)n - 1 - tid) / SNT + 1 : 0u)) - 1;
        tick(0);  // the partition's loads landed, hashed
        for (u32 round = 0; round <= smask; ++round) {
            u32 act = 0;
#pragma unroll
            for (int u = 0; u < RPT; ++u) act |= (lo[u] & smask) == round ? (1u << u) : 0u;
            act &= valid;
            while (true) {  // mini-rounds: the round's records, then its probe-window misses
                while (true) {  // stage <= PS_STAGE of them at a time (compacted: every lane busy)
                    // one LDS add per wave for all RPT slots: the ballots first (no memory ops),
                    // then the wave's base, then each slot's running offset (wave-uniform)
                    u64 mb[RPT];
                    u32 wtot = 0;
#pragma unroll
                    for (int u = 0; u < RPT; ++u) {
                        mb[u] = __ballot((act >> u) & 1);
                        wtot += (u32)__popcll(mb[u]);
                    }
                    u32 wbase = 0;
                    if (wtot) {
                        if (lane == 0) wbase = atomicAdd(&scount, wtot);
                        wbase = __builtin_amdgcn_readfirstlane(wbase);
                    }
                    u32 run = wbase;
#pragma unroll
                    for (int u = 0; u < RPT; ++u) {
                        const u64 m = mb[u];
                        const bool on = (act >> u) & 1;
                        const u32 k = run + (u32)__popcll(m & ((1ULL << lane) - 1));
                        run += (u32)__popcll(m);
                        if (on && k < PS_STAGE) {
#pragma unroll
                            for (int w = 0; w < W; ++w) sw_[(size_t)k * W + w] = rr[u].r[w];
                            slo[k] = lo[u];
                            sorg[k] = (u16)((tid << 4) | (u32)u);
                            act &= ~(1u << u);
                        }
                    }
                    tick(1);
                    lds_barrier();
                    tick(4);
                    const u32 ms = min(scount, (u32)PS_STAGE);
                    for (u32 k0 = 0; k0 < ms; k0 += SNT) {
                        const u32 k = k0 + tid;
                        if (k < ms && !insert(k))
                            __hip_atomic_fetch_or(pend + (sorg[k] >> 4), 1u << (sorg[k] & 15), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    }
                    tick(2);
                    lds_barrier();
                    if (tid == 0) scount = 0;
                    const bool more = block_any(act != 0);
                    tick(4);
                    if (!more) break;
                }
                // the round's groups out as result rows, their tags cleared for the next table
                if (tid == 0) gbase = nlist ? atomicAdd((unsigned long long*)(out.tot + PPT_GROUPS), (unsigned long long)nlist) : 0;
                lds_barrier();
                const u32 ng = nlist;
                if (MODE == 1) {
                    for (u32 k = tid; k < ng; k += SNT) {  // group records in the state-record format
                        const l64* e = body + (size_t)list[k] * BW;
                        const u64 row = gbase + k;
                        const u64 cnt = e[KW];
                        if (row >= out.grec_cap) continue;
                        __attribute__((address_space(1))) u64* d = (__attribute__((address_space(1))) u64*)(out.grec + row * D.rec_bytes);
                        u32 q = 0;
#pragma unroll
                        for (u32 w = 0; w < 2; ++w)
                            if (w < KW) d[q++] = e[w];
#pragma unroll
                        for (u32 a = 0; a < PS_MAXA; ++a) {
                            if (a >= D.na) continue;
                            const int kd = D.kind[a];
                            if (kd == PS_COUNT) {
                                d[q++] = cnt;
                            } else if (kd == PS_AVG) {  // the Spec's AVG state: sum, count
                                d[q++] = e[D.vw[a]];
                                d[q++] = cnt;
                            } else {
                                d[q++] = e[D.vw[a]];
                            }
                        }
                    }
                } else {
                    // result columns, one column at a time: the column's kind and width are
                    // decided once (uniform), so each loop is a plain LDS read -> global store
                    // (a per-group switch over kinds and widths tripled this phase)
                    const u64 cap_g = out.cols.cap_groups;
                    auto col_loop = [&](auto value_of, void* dst, u32 w) {
                        typedef __attribute__((address_space(1))) u8 g8;
                        g8* base = (g8*)dst;
                        for (u32 k = tid; k < ng; k += SNT) {
                            const u64 row = gbase + k;
                            if (row >= cap_g) continue;
                            const u64 v = value_of(body + (size_t)list[k] * BW);
                            if (w == 8) ((__attribute__((address_space(1))) u64*)base)[row] = v;
                            else if (w == 4) ((__attribute__((address_space(1))) u32*)base)[row] = (u32)v;
                            else if (w == 2) ((__attribute__((address_space(1))) uint16_t*)base)[row] = (uint16_t)v;
                            else base[row] = (u8)v;
                        }
                    };
                    auto ones = [&](u8* dst) {
                        if (dst) col_loop([](const l64*) -> u64 { return 1; }, dst, 1);
                    };
                    col_loop([&](const l64* e) -> u64 { return e[0] & D.km0; }, out.cols.key_data[0], D.kb0);
                    ones(out.cols.key_valid[0]);
                    if (D.nk == 2) {
                        if (D.k1w) col_loop([&](const l64* e) -> u64 { return (e[1] >> D.k1s) & D.km1; }, out.cols.key_data[1], D.kb1);
                        else col_loop([&](const l64* e) -> u64 { return ((e[0] >> D.k1s) | (KW > 1 ? e[1] << (64 - D.k1s) : 0)) & D.km1; },
                                      out.cols.key_data[1], D.kb1);
                        ones(out.cols.key_valid[1]);
                    }
                    for (u32 a = 0; a < D.na; ++a) {
                        const int kd = D.kind[a];
                        const u32 vw = D.vw[a];
                        if (kd == PS_COUNT) {
                            col_loop([&](const l64* e) -> u64 { return e[KW]; }, out.cols.agg_data[a], 8);
                        } else if (kd == PS_AVG) {  // the sum as i64 (u64 for unsigned arguments) / count, as f64
                            if (ps_signed(D.at[a]))
                                col_loop([&](const l64* e) -> u64 { return (u64)__double_as_longlong((double)(i64)e[vw] / (double)e[KW]); },
                                         out.cols.agg_data[a], 8);
                            else
                                col_loop([&](const l64* e) -> u64 { return (u64)__double_as_longlong((double)e[vw] / (double)e[KW]); },
                                         out.cols.agg_data[a], 8);
                        } else {
                            col_loop([&](const l64* e) -> u64 { return e[vw]; }, out.cols.agg_data[a], D.rw[a]);
                        }
                        ones(out.cols.agg_valid[a]);
                    }
                }
                for (u32 k = tid; k < ng; k += SNT) tags[list[k]] = 0;
                tick(3);
                lds_barrier();
                tick(4);
                if (tid == 0) nlist = 0;
                act = pend[tid];
                pend[tid] = 0;
                if (!block_any(act != 0)) break;
                if (tid == 0) atomicAdd((unsigned long long*)(out.tot + PPT_ROUNDS), 1ULL);
            }
        }
    }
}

#define PP_SPEC_NT 1024  // 16 waves per CU (C4 shape: 512 lanes x 16 records 36 ms, 1024 x 8 32 ms)
#define PS_MAXW 6  // raw record words: 16 key bytes + 4 x 8 argument bytes
// records per lane: the two register sets (the partition and the next one's prefetch) stay at
// <= 128 VGPRs
#ifndef PS_RPT2
#define PS_RPT2 8
#endif
// records per lane (x PP_SPEC_NT lanes: 8192 records at W <= 2, 4096 at W <= 4, 2048 beyond)
__host__ __device__ constexpr int ps_rpt(int w) { return w <= 1 ? 8 : (w <= 2 ? PS_RPT2 : (w <= 4 ? 4 : 2)); }

static bool ps_int_type(int t) {
    return t == DBG_INT8 || t == DBG_INT16 || t == DBG_INT32 || t == DBG_INT64 || t == DBG_UINT8 || t == DBG_UINT16 ||
           t == DBG_UINT32 || t == DBG_UINT64;
}

// The descriptor of a Spec the kernel covers, or false.  Checks the raw-record packing of
// build_spec (keys contiguous from byte 0, each argument aligned to its width after them) and
// the state record format against what the kernel reads and writes.
static bool ps_desc(const Spec& S, PsDesc& D, u32& W) {
    memset(&D, 0, sizeof(D));
    if (S.pp_str || S.n_keys < 1 || S.n_keys > 2 || S.n_aggs < 1 || S.n_aggs > PS_MAXA || S.flags_word >= 0) return false;
    D.nk = (u32)S.n_keys;
    u32 kb = 0;
    for (int c = 0; c < S.n_keys; ++c) {
        const int t = S.key_types[c].type;
        const bool ok = ps_int_type(t) || t == DBG_DATE || t == DBG_TIMESTAMP;
        if (!ok || S.key_types[c].nullable || S.koff[c] != kb) return false;
        D.kt[c] = t;
        const u32 w = t == DBG_TIMESTAMP ? 8u : ps_tw(t);
        const u64 m = w == 8 ? ~0ULL : ((1ULL << (8 * w)) - 1);
        if (c == 0) {
            D.kb0 = w;
            D.km0 = m;
        } else {
            D.kb1 = w;
            D.km1 = m;
            D.k1w = kb / 8;
            D.k1s = 8 * (kb % 8);
        }
        kb += w;
    }
    D.hc = (u32)(ps_hclass(D.kt[0]) * 5 + (D.nk == 2 ? ps_hclass(D.kt[1]) : 4));
    D.kw = (kb + 7) / 8;
    D.klast = (kb & 7) == 0 ? ~0ULL : ((1ULL << (8 * (kb & 7))) - 1);
    if (S.pp_kw != 8 * D.kw) return false;
    D.na = (u32)S.n_aggs;
    u32 po = kb, vw = D.kw + 1, rec_words = D.kw;
    for (int a = 0; a < S.n_aggs; ++a) {
        const DAgg& A = S.aggs[a];
        int kd;
        if (A.kind == DBG_AGG_COUNT) {
            if (A.arg_type >= 0 && A.arg_nullable) return false;
            kd = PS_COUNT;  // COUNT(*) or COUNT(non-nullable x): the row count
        } else {
            if (A.arg_type < 0 || A.arg_nullable || !ps_int_type(A.arg_type)) return false;
            if (A.kind == DBG_AGG_SUM && A.sumk == SUMK_I64 && A.res_width == 8) kd = PS_SUM;
            else if (A.kind == DBG_AGG_AVG && A.sumk == SUMK_I64 && !A.avg_round && A.res_type == DBG_FLOAT64) kd = PS_AVG;
            else if ((A.kind == DBG_AGG_MIN || A.kind == DBG_AGG_MAX) && (A.mmk == MMK_I64 || A.mmk == MMK_U64) &&
                     (u32)A.res_width == ps_tw(A.arg_type))
                kd = A.kind == DBG_AGG_MIN ? PS_MIN : PS_MAX;
            else
                return false;
        }
        D.kind[a] = kd;
        D.rw[a] = kd == PS_MIN || kd == PS_MAX ? ps_tw(A.arg_type) : 8u;
        const u32 nwords = kd == PS_AVG ? 2u : 1u;  // the Spec's state words
        if (A.nwords != (int)nwords || A.w0 != (int)(rec_words - D.kw + 1)) return false;
        rec_words += nwords;
        if (A.arg_type >= 0 && kd != PS_COUNT) {
            const u32 w = ps_tw(A.arg_type);
            po = (po + w - 1) & ~(w - 1);
            D.at[a] = A.arg_type;
            D.aoff[a] = po;
            D.aw[a] = w;
            D.xw[a] = po / 8;
            D.xs[a] = 8 * (po % 8);
            D.xe[a] = 64 - 8 * w;
            D.xsg[a] = ps_signed(A.arg_type) ? 1u : 0u;
            if (S.pp_aoff[a] != po) return false;
            po += w;
            D.vw[a] = vw++;
        } else if (A.arg_type >= 0) {
            // COUNT(x): build_spec still packs x into the raw record
            const u32 w = ps_tw(A.arg_type);
            po = (po + w - 1) & ~(w - 1);
            if (S.pp_aoff[a] != po) return false;
            po += w;
        }
    }
    D.bw = vw;
    D.rec_bytes = 8 * rec_words;
    W = (S.pp_rw_raw + 7) / 8;
    return S.pp_rw_raw == ((po + 7) & ~7u) && W >= 1 && W <= PS_MAXW && S.pp_rw_state == D.rec_bytes;
}

#define PS_LDS (152 * 1024)  // one workgroup per CU: the largest table, the fewest rounds
static u32 ps_cap(u32 bw, u32 w, u32 nt = PP_SPEC_NT, size_t budget = PS_LDS) {
    u32 cap = (u32)((budget - ps_lds_bytes(0, bw, w, nt) - 64) / (4 + 8 * bw + 2)) & ~3u;
    while (cap > 64 && ps_lds_bytes(cap, bw, w, nt) + 64 > budget) cap -= 4;
    return std::min<u32>(cap, 65532);
}

static int ps_desc_shape(const Spec& S, u32* cap, u32* max_records) {
    PsDesc D;
    u32 W = 0;
    if (!ps_desc(S, D, W)) return -1;
    *cap = ps_cap(D.bw, W);
    *max_records = PP_SPEC_NT * ps_rpt((int)W);
    return (int)W;
}

static void launch_ps_desc(hipStream_t s, const Spec& S, int shape, int mode, u32 n_parts, const u64* raw_off, const u8* raw,
                           u32 sub_bits, const PPAggOut& out, u32* spill, u32 spill_cap) {
    if (!n_parts) return;
    PsDesc D;
    u32 W = 0;
    if (!ps_desc(S, D, W) || (int)W != shape) return;  // the host planned with pp_spec_shape: never taken
    const u32 grid = n_parts < 256 ? n_parts : 256;  // one persistent workgroup per CU
    // test hook: a smaller LDS table than the plan assumed (probe-window misses, pending rounds)
    const u32 cap = std::min(ps_cap(D.bw, W), S.x_pp_cap);
    const size_t lds = ps_lds_bytes(cap, D.bw, W, PP_SPEC_NT) + 16;
#define PS_LAUNCH(WW)                                                                                                            \
    case WW:                                                                                                                     \
        if (mode == 0)                                                                                                           \
            hipLaunchKernelGGL((pp_agg_desc_kernel<0, WW, ps_rpt(WW), PP_SPEC_NT>), dim3(grid), dim3(PP_SPEC_NT), lds, s, D,     \
                               n_parts, raw_off, raw, sub_bits, cap, out, spill, spill_cap);                                     \
        else                                                                                                                     \
            hipLaunchKernelGGL((pp_agg_desc_kernel<1, WW, ps_rpt(WW), PP_SPEC_NT>), dim3(grid), dim3(PP_SPEC_NT), lds, s, D,     \
                               n_parts, raw_off, raw, sub_bits, cap, out, spill, spill_cap);                                     \
        break;
    switch (W) {
        PS_LAUNCH(1)
        PS_LAUNCH(2)
        PS_LAUNCH(3)
        PS_LAUNCH(4)
        PS_LAUNCH(5)
        PS_LAUNCH(6)
    }
#undef PS_LAUNCH
}

// ------------------------------------------------------------------------------------------
// Compile-time specialised aggregation of raw records (pp_agg_spec_kernel).
//
// The generic kernel above interprets the Spec per record: a loop over the aggregates with a
// switch on kind, argument width and type, a generic row writer, and a slot-table claim that
// initialises states and then applies the record with LDS atomics.  For the common shape —
// fixed-width non-nullable keys, COUNT(*) / SUM / AVG over non-nullable integer arguments, the
// final result written as columns — every one of those decisions is a template parameter here:
//   * key types and argument types / offsets are compile-time (offsets from the same packing rule
//     as build_spec, checked against the Spec on the host before launch);
//   * a slot is [key words][row count][one sum word per SUM / AVG]: AVG's count and COUNT(*) are the
//     same row count (arguments are non-nullable), so C4's state is 3 words instead of 4;
//   * a claimer initialises the slot from its own record (count 1, sums = its values) before
//     publishing the tag: a new group costs no LDS atomics, a repeat costs one add per word;
//   * probes read a dense u32 tag array (one LDS word per probe step), the key words only on a
//     tag match;
//   * claimed slots join the output list with one LDS add per wave (ballot), not one per lane;
//   * a partition (up to PP_AGG_NT x RPT records) is loaded into registers once and aggregated in
//     2^sub_bits rounds selected by the hash bits below the partition's, so a partition holds
//     2^sub_bits LDS tables' worth of groups and the level-3 scatter is gone (AGG/
//     transform_aggregate_final.rs:71-156 aggregates one bucket per task the same way).
// A record whose probe window is full stays pending and is inserted into the emptied table in
// a further mini-round (consistent per key: slots only fill within a mini-round).  Partitions
// larger than the register budget are listed in `spill` for the generic kernel.
// ------------------------------------------------------------------------------------------
#define PS_AGG(kind, t) (((kind) << 8) | ((t) & 0xff))
__host__ __device__ constexpr int ps_kind(int a) { return a >> 8; }
__host__ __device__ constexpr int ps_type(int a) { return a & 0xff; }
__host__ __device__ constexpr bool ps_has_arg(int a) { return ps_kind(a) == PS_SUM || ps_kind(a) == PS_AVG; }
// build_spec's raw record packing: key bytes, then each argument aligned to its width
__host__ __device__ constexpr u32 ps_align(u32 po, int a) { return ps_has_arg(a) ? ((po + ps_tw(ps_type(a)) - 1) & ~(ps_tw(ps_type(a)) - 1)) : po; }
__host__ __device__ constexpr u32 ps_next(u32 po, int a) { return ps_has_arg(a) ? ps_align(po, a) + ps_tw(ps_type(a)) : po; }

template <int K0, int K1, int A0, int A1, int A2>
struct PsShape {
    static constexpr int NK = K1 < 0 ? 1 : 2;
    static constexpr u32 KB = ps_tw(K0) + (K1 < 0 ? 0u : ps_tw(K1));  // packed key bytes
    static constexpr u32 KW = (KB + 7) / 8;
    static constexpr u64 KLAST = (KB & 7) == 0 ? ~0ULL : ((1ULL << (8 * (KB & 7))) - 1);
    static constexpr u32 OFF0 = ps_align(KB, A0);
    static constexpr u32 OFF1 = ps_align(ps_next(KB, A0), A1);
    static constexpr u32 OFF2 = ps_align(ps_next(ps_next(KB, A0), A1), A2);
    static constexpr u32 END = ps_next(ps_next(ps_next(KB, A0), A1), A2);
    static constexpr int NSUM = (ps_has_arg(A0) ? 1 : 0) + (ps_has_arg(A1) ? 1 : 0) + (ps_has_arg(A2) ? 1 : 0);
    static constexpr u32 BW = KW + 1 + NSUM;  // slot body words: key, row count, sums
    // Narrow slots: a partition holds at most PP_LIT_NT x PP_LIT_RPT (8192) records, so the row
    // count fits 32 bits, and so does a sum of arguments of at most 2 bytes (|sum| < 8192 x 2^16):
    // [key as u32 words][count u32][one i32 sum per SUM / AVG] — C4's slot 40 -> 24 bytes, so the
    // LDS table holds 1.7x the groups and a partition needs half the rounds.  Keys must fill
    // whole u32 words (their bytes are compared word by word).
    static constexpr bool small_arg(int a) { return !ps_has_arg(a) || ps_tw(ps_type(a)) <= 2; }
    static constexpr bool NARROW = (KB % 4 == 0) && small_arg(A0) && small_arg(A1) && small_arg(A2);
    static constexpr u32 KW32 = KB / 4;
    static constexpr u32 BW32 = KW32 + 1 + NSUM;
    static constexpr u32 BWL = NARROW ? (BW32 + 1) / 2 : BW;  // the slot's LDS size in u64 words
    static constexpr u32 sum32(int a) {
        return KW32 + 1 + (a > 0 && ps_has_arg(A0) ? 1 : 0) + (a > 1 && ps_has_arg(A1) ? 1 : 0);
    }
    // Spec state words (build_spec: COUNT 1, SUM 1, AVG 2 — sum, count) and the state record bytes
    static constexpr u32 swords(int a) { return a == 0 ? 0u : (ps_kind(a) == PS_AVG ? 2u : 1u); }
    static constexpr u32 REC_BYTES = 8 * (KW + swords(A0) + swords(A1) + swords(A2));
    static constexpr u32 off(int a) { return a == 0 ? OFF0 : (a == 1 ? OFF1 : OFF2); }
    static constexpr int agg(int a) { return a == 0 ? A0 : (a == 1 ? A1 : A2); }
    // sum word of aggregate a (after the row count)
    static constexpr u32 sumw(int a) {
        return KW + 1 + (a > 0 && ps_has_arg(A0) ? 1 : 0) + (a > 1 && ps_has_arg(A1) ? 1 : 0);
    }
};

template <int MODE, int W, int RPT, int SNT, int K0, int K1, int A0, int A1, int A2>
__global__ void __launch_bounds__(SNT, (SNT / 256) * PP_LIT_PER_CU) pp_agg_spec_kernel(u32 n_parts, const u64* __restrict__ raw_off, const u8* __restrict__ raw,
                                                               u32 sub_bits, u32 cap, PPAggOut out, u32* __restrict__ spill, u32 spill_cap) {
    typedef PsShape<K0, K1, A0, A1, A2> SH;
    constexpr u32 KW = SH::KW, BW = SH::BWL;
    constexpr bool NW = SH::NARROW;
    static_assert(KW <= (u32)W && SH::END <= 8u * W, "record words");
    static_assert(!NW || SNT * RPT <= 8192, "narrow slots: counts and 2-byte sums of <= 8192 records fit 32 bits");
    static_assert(RPT < 32, "per-lane record mask");
    extern __shared__ __attribute__((aligned(16))) u64 lds_raw[];
    l32* tags = (l32*)lds_raw;                                     // [cap] 0 empty, 1 being claimed, else tag
    l64* body = (l64*)lds_raw + (cap + 1) / 2;                     // [cap][BW]
    l16* list = (l16*)(body + (size_t)cap * BW);                   // claimed slots of the round
    l64* sw_ = (l64*)(list + ((cap + 3) & ~3u));                   // staged records [PS_STAGE][W]
    l32* slo = (l32*)(sw_ + (size_t)PS_STAGE * W);                 // their slot hash bits
    l16* sorg = (l16*)(slo + PS_STAGE);                            // their origin (thread << 4 | register index)
    l32* pend = (l32*)(((uintptr_t)(sorg + PS_STAGE) + 3) & ~(uintptr_t)3);  // [SNT] probe-window misses
    __shared__ u32 nlist, scount, anyw[3];
    __shared__ u64 gbase;
    const u32 tid = threadIdx.x, lane = tid & 63;
    // Barriers order LDS only: the output stores and the next partition's prefetched loads stay in
    // flight across them (__syncthreads' workgroup fence would wait for every outstanding global
    // access — the prefetch included).
    auto lds_barrier = [] { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); };
    // block-wide OR over three rotating LDS words: call c clears the word call c + 1 votes into
    // before its barrier (that word was last read in call c - 2, before call c - 1's barrier)
    u32 anyc = 0;
    auto block_any = [&](bool v) -> bool {
        const u32 q = anyc % 3;
        if (tid == 0) anyw[(q + 1) % 3] = 0;
        if (__ballot(v) && lane == 0) atomicOr(&anyw[q], 1u);
        lds_barrier();
        ++anyc;
        return anyw[q] != 0;
    };
    const u32 smask = (1u << sub_bits) - 1;
    const u32 win = cap < PP_WINDOW ? cap : PP_WINDOW;
    // EXPERIMENT (TRACE=1 build, DBG_X_PPTRACE): phase times of sampled workgroups, thread 0
    const bool tr = kPhaseTrace && out.trace && (blockIdx.x & 15) == 0 && tid == 0;
    u64 tm0 = tr ? __builtin_amdgcn_s_memrealtime() : 0;
    auto tick = [&](int slot) {
        if (tr) {
            const u64 tm = __builtin_amdgcn_s_memrealtime();
            atomicAdd((unsigned long long*)out.trace + slot, tm - tm0);
            tm0 = tm;
        }
    };
    for (u32 j = tid; j < cap; j += SNT) tags[j] = 0;
    pend[tid] = 0;
    if (tid == 0) {
        nlist = scount = 0;
        anyw[0] = anyw[1] = anyw[2] = 0;
    }
    lds_barrier();
    // one staged record into the table; false = no room in its probe window
    auto insert = [&](u32 k) -> bool {
        RegRec<W> rk;
#pragma unroll
        for (int w = 0; w < W; ++w) rk.r[w] = sw_[(size_t)k * W + w];
        const u32 lo = slo[k];
        const u32 tag = (lo & ~3u) | 2u;
        u32 pos = (u32)(((u64)lo * cap) >> 32);
        bool claimed = false;
        int at = -1;
        for (u32 q = 0; q < win; ++q) {
            l32* tp = tags + pos;
            u32 t = __hip_atomic_load(tp, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
            if (t == 0) {
                u32 old = 0;
                __hip_atomic_compare_exchange_strong(tp, &old, 1u, __ATOMIC_ACQUIRE, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
                if (old == 0) {  // claimed: key words, the record's own contribution, then the tag
                    l64* e = body + (size_t)pos * BW;
                    if constexpr (NW) {
                        l32* e32 = (l32*)e;
#pragma unroll
                        for (u32 w = 0; w < SH::KW32; ++w) e32[w] = (u32)(rk.r[w / 2] >> (32 * (w & 1)));
                        e32[SH::KW32] = 1;
#pragma unroll
                        for (int a = 0; a < 3; ++a)
                            if (ps_has_arg(SH::agg(a)))
                                e32[SH::sum32(a)] = (u32)ps_ext(rk.le(SH::off(a), ps_tw(ps_type(SH::agg(a)))), ps_type(SH::agg(a)));
                    } else {
#pragma unroll
                        for (u32 w = 0; w < KW; ++w) e[w] = w + 1 == KW ? (rk.r[w] & SH::KLAST) : rk.r[w];
                        e[KW] = 1;
#pragma unroll
                        for (int a = 0; a < 3; ++a)
                            if (ps_has_arg(SH::agg(a))) e[SH::sumw(a)] = ps_ext(rk.le(SH::off(a), ps_tw(ps_type(SH::agg(a)))), ps_type(SH::agg(a)));
                    }
                    __hip_atomic_store(tp, tag, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
                    claimed = true;
                    at = (int)pos;
                    break;
                }
                t = old;
            }
            while (t == 1) t = __hip_atomic_load(tp, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_WORKGROUP);
            if (t == tag) {
                l64* e = body + (size_t)pos * BW;
                bool eq = true;
                if constexpr (NW) {
                    l32* e32 = (l32*)e;
#pragma unroll
                    for (u32 w = 0; w < SH::KW32; ++w) eq &= e32[w] == (u32)(rk.r[w / 2] >> (32 * (w & 1)));
                    if (eq) {
                        auto add32 = [](l32* p, u32 v) {
                            __hip_atomic_fetch_add((__attribute__((address_space(3))) u32*)p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                        };
                        add32(e32 + SH::KW32, 1u);
#pragma unroll
                        for (int a = 0; a < 3; ++a)
                            if (ps_has_arg(SH::agg(a)))
                                add32(e32 + SH::sum32(a), (u32)ps_ext(rk.le(SH::off(a), ps_tw(ps_type(SH::agg(a)))), ps_type(SH::agg(a))));
                    }
                } else {
#pragma unroll
                    for (u32 w = 0; w < KW; ++w) eq &= e[w] == (w + 1 == KW ? (rk.r[w] & SH::KLAST) : rk.r[w]);
                    if (eq) {
                        at_add<AS_LDS>((wptr<AS_LDS>)(e + KW), 1ULL);
#pragma unroll
                        for (int a = 0; a < 3; ++a)
                            if (ps_has_arg(SH::agg(a)))
                                at_add<AS_LDS>((wptr<AS_LDS>)(e + SH::sumw(a)),
                                               ps_ext(rk.le(SH::off(a), ps_tw(ps_type(SH::agg(a)))), ps_type(SH::agg(a))));
                    }
                }
                if (eq) {
                    at = (int)pos;
                    break;
                }
            }
            pos = pos + 1 == cap ? 0 : pos + 1;
        }
        // new groups join the round's list: one LDS add per wave (called with the wave converged)
        const u64 m = __ballot(claimed);
        if (m) {
            const u32 lead = (u32)__ffsll((long long)m) - 1;
            u32 b = 0;
            if (lane == lead) b = atomicAdd(&nlist, (u32)__popcll(m));
            b = __shfl(b, (int)lead);
            if (claimed) list[b + (u32)__popcll(m & ((1ULL << lane) - 1))] = (u16)at;
        }
        return at >= 0;
    };
    // A partition's records live in registers (RPT per lane, loaded with buffer loads: one 32-bit
    // lane offset, the range check returning zeros past the partition), and the next partition of
    // this workgroup is loaded into a second register set while the current one is aggregated.
    typedef u32 v2u32 __attribute__((ext_vector_type(2)));
    auto load_part = [&](u32 q, RegRec<W>* dst, u64& n_out) {
        n_out = 0;
        if (q >= n_parts) return;
        const u64 o0 = raw_off[q], n = raw_off[q + 1] - o0;
        n_out = n;
        if (n == 0 || n > (u64)SNT * RPT) return;
        const u8* base = raw + o0 * (8 * W);
        const auto rsrc = __builtin_amdgcn_make_buffer_rsrc((void*)base, 0, (int)(n * (8 * W)), 0x00020000);
#pragma unroll
        for (int u = 0; u < RPT; ++u)
#pragma unroll
            for (int w = 0; w < W; ++w) {
                const v2u32 v = __builtin_amdgcn_raw_buffer_load_b64(rsrc, tid * (8 * W) + 8 * w, u * (SNT * 8 * W), 0);
                dst[u].r[w] = (u64)v.x | ((u64)v.y << 32);
            }
    };
    RegRec<W> nxt[RPT];
    u64 n_nxt;
    load_part(blockIdx.x, nxt, n_nxt);
    for (u32 p = blockIdx.x; p < n_parts; p += gridDim.x) {
        RegRec<W> rr[RPT];
#pragma unroll
        for (int u = 0; u < RPT; ++u) rr[u] = nxt[u];
        const u64 n = n_nxt;
        load_part(p + gridDim.x, nxt, n_nxt);  // in flight during this partition's rounds
        if (n == 0) continue;
        if (n > (u64)SNT * RPT) {  // uniform: the generic kernel takes it
            if (tid == 0) {
                const u32 k = atomicAdd(spill, 1u);
                if (k < spill_cap) spill[1 + k] = p;
                else atomicOr((unsigned long long*)(out.tot + PPT_ERR), (unsigned long long)ERR_OVF_LOST);
            }
            continue;
        }
        if (tr) atomicAdd((unsigned long long*)out.trace + 5, 1ULL);
        // slot hash bits; a record's round is the low sub_bits of its hash (the partition is the
        // top bits, the slot position the top bits of the low word)
        auto slot_hash = [&](const RegRec<W>& r) -> u32 {
            u64 h = hash_bits(K0, r.le(0, ps_tw(K0)));
            if (K1 >= 0) h = (h * NULL_HASH_VAL) ^ hash_bits(K1, r.le(ps_tw(K0), ps_tw(K1)));
            return (u32)pp_mix(h);
        };
        u32 lo[RPT];  // slot hash bits; the round is the low sub_bits
#pragma unroll
        for (int u = 0; u < RPT; ++u) lo[u] = slot_hash(rr[u]);
        // records this lane holds: register u is row u * SNT + tid (32-bit: n <= SNT * RPT; a 64-bit
        // row test per register had the compiler keep RPT 64-bit row constants live, and spill them)
        const u32 valid = (1u << ((u32)n > tid ? ((u32)n - 1 - tid) / SNT + 1 : 0u)) - 1;
        tick(0);  // the partition's loads landed, hashed
        for (u32 round = 0; round <= smask; ++round) {
            u32 act = 0;
#pragma unroll
            for (int u = 0; u < RPT; ++u) act |= (lo[u] & smask) == round ? (1u << u) : 0u;
            act &= valid;
            while (true) {  // mini-rounds: the round's records, then its probe-window misses
                while (true) {  // stage <= PS_STAGE of them at a time (compacted: every lane busy)
                    // one LDS add per wave for all RPT slots: the ballots first (no memory ops),
                    // then the wave's base, then each slot's running offset (wave-uniform)
                    u64 mb[RPT];
                    u32 wtot = 0;
#pragma unroll
                    for (int u = 0; u < RPT; ++u) {
                        mb[u] = __ballot((act >> u) & 1);
                        wtot += (u32)__popcll(mb[u]);
                    }
                    u32 wbase = 0;
                    if (wtot) {
                        if (lane == 0) wbase = atomicAdd(&scount, wtot);
                        wbase = __builtin_amdgcn_readfirstlane(wbase);
                    }
                    u32 run = wbase;
#pragma unroll
                    for (int u = 0; u < RPT; ++u) {
                        const u64 m = mb[u];
                        const bool on = (act >> u) & 1;
                        const u32 k = run + (u32)__popcll(m & ((1ULL << lane) - 1));
                        run += (u32)__popcll(m);
                        if (on && k < PS_STAGE) {
#pragma unroll
                            for (int w = 0; w < W; ++w) sw_[(size_t)k * W + w] = rr[u].r[w];
                            slo[k] = lo[u];
                            sorg[k] = (u16)((tid << 4) | (u32)u);
                            act &= ~(1u << u);
                        }
                    }
                    tick(1);
                    lds_barrier();
                    tick(4);
                    const u32 ms = min(scount, (u32)PS_STAGE);
                    for (u32 k0 = 0; k0 < ms; k0 += SNT) {
                        const u32 k = k0 + tid;
                        if (k < ms && !insert(k))
                            __hip_atomic_fetch_or(pend + (sorg[k] >> 4), 1u << (sorg[k] & 15), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    }
                    tick(2);
                    lds_barrier();
                    if (tid == 0) scount = 0;
                    const bool more = block_any(act != 0);
                    tick(4);
                    if (!more) break;
                }
                // the round's groups out as result rows, their tags cleared for the next table
                if (tid == 0) gbase = nlist ? atomicAdd((unsigned long long*)(out.tot + PPT_GROUPS), (unsigned long long)nlist) : 0;
                lds_barrier();
                const u32 ng = nlist;
                for (u32 k = tid; k < ng; k += SNT) {
                    const u32 pos = list[k];
                    const l64* e = body + (size_t)pos * BW;
                    const u64 row = gbase + k;
                    // the slot's key words, row count and sums, read where they are stored (narrow slots
                    // widened: a sum of signed arguments sign-extended)
                    auto key_word = [&](u32 w) -> u64 {
                        if constexpr (NW) {
                            const l32* e32 = (const l32*)e;
                            const u64 lo = e32[2 * w], hi = 2 * w + 1 < SH::KW32 ? (u64)e32[2 * w + 1] : 0;
                            return lo | (hi << 32);
                        } else {
                            return e[w];
                        }
                    };
                    auto count_of = [&]() -> u64 {
                        if constexpr (NW) return ((const l32*)e)[SH::KW32];
                        else return e[KW];
                    };
                    auto sum_of = [&](int a) -> u64 {
                        if constexpr (NW) {
                            const u32 v = ((const l32*)e)[SH::sum32(a)];
                            return ps_signed(ps_type(SH::agg(a))) ? (u64)(i64)(int32_t)v : (u64)v;
                        } else {
                            return e[SH::sumw(a)];
                        }
                    };
                    if (MODE == 1) {  // group records in the state-record format: [key words][Spec state words]
                        if (row < out.grec_cap) {
                            u64* d = (u64*)(out.grec + row * SH::REC_BYTES);
#pragma unroll
                            for (u32 w = 0; w < KW; ++w) d[w] = key_word(w);
                            u32 q = KW;
#pragma unroll
                            for (int a = 0; a < 3; ++a) {
                                const int A = SH::agg(a);
                                if (A == 0) continue;
                                if (ps_kind(A) == PS_COUNT) d[q++] = count_of();
                                else if (ps_kind(A) == PS_SUM) d[q++] = sum_of(a);
                                else {
                                    d[q++] = sum_of(a);
                                    d[q++] = count_of();
                                }
                            }
                        }
                    } else if (row < out.cols.cap_groups) {
                        RegRec<KW> kr;
#pragma unroll
                        for (u32 w = 0; w < KW; ++w) kr.r[w] = key_word(w);
                        const u64 cnt = count_of();
                        write_bytes(out.cols.key_data[0], row, ps_tw(K0), kr.le(0, ps_tw(K0)), 0);
                        if (out.cols.key_valid[0]) out.cols.key_valid[0][row] = 1;
                        if (K1 >= 0) {
                            write_bytes(out.cols.key_data[1], row, ps_tw(K1), kr.le(ps_tw(K0), ps_tw(K1)), 0);
                            if (out.cols.key_valid[1]) out.cols.key_valid[1][row] = 1;
                        }
#pragma unroll
                        for (int a = 0; a < 3; ++a) {
                            const int A = SH::agg(a);
                            if (A == 0) continue;
                            u64 v;
                            if (ps_kind(A) == PS_COUNT) {
                                v = cnt;
                            } else if (ps_kind(A) == PS_SUM) {
                                v = sum_of(a);
                            } else {  // AVG: the sum as i64 (u64 for unsigned arguments) / count, as f64
                                const u64 sv = sum_of(a);
                                const double sum = ps_signed(ps_type(A)) ? (double)(i64)sv : (double)sv;
                                v = (u64)__double_as_longlong(sum / (double)cnt);
                            }
                            ((u64*)out.cols.agg_data[a])[row] = v;
                            if (out.cols.agg_valid[a]) out.cols.agg_valid[a][row] = 1;
                        }
                    }
                    tags[pos] = 0;
                }
                tick(3);
                lds_barrier();
                tick(4);
                if (tid == 0) nlist = 0;
                act = pend[tid];
                pend[tid] = 0;
                if (!block_any(act != 0)) break;
                if (tid == 0) atomicAdd((unsigned long long*)(out.tot + PPT_ROUNDS), 1ULL);
            }
        }
    }
}

// The instantiated shapes: C4 (ClickBench Q33) and the one-key COUNT / SUM forms.
#define PS_SHAPES(X)                                                                                          \
    X(2, DBG_INT64, DBG_INT32, PS_AGG(PS_COUNT, 0), PS_AGG(PS_SUM, DBG_INT16), PS_AGG(PS_AVG, DBG_INT16))       \
    X(1, DBG_INT64, -1, PS_AGG(PS_COUNT, 0), 0, 0)                                                             \
    X(2, DBG_INT64, -1, PS_AGG(PS_COUNT, 0), PS_AGG(PS_SUM, DBG_INT64), 0)                                     \
    X(2, DBG_INT64, DBG_INT64, PS_AGG(PS_COUNT, 0), 0, 0)
#define PP_SPEC_RPT 16

static int ps_code(const DAgg& A) {
    if (A.kind == DBG_AGG_COUNT) return A.arg_type < 0 ? PS_AGG(PS_COUNT, 0) : -1;
    if (A.arg_type < 0 || A.arg_nullable || A.sumk != SUMK_I64 || A.res_width != 8) return -1;
    const int t = A.arg_type;
    const bool ints = t == DBG_INT8 || t == DBG_INT16 || t == DBG_INT32 || t == DBG_INT64 || t == DBG_UINT8 || t == DBG_UINT16 ||
                      t == DBG_UINT32 || t == DBG_UINT64;
    if (!ints) return -1;
    if (A.kind == DBG_AGG_SUM) return PS_AGG(PS_SUM, t);
    if (A.kind == DBG_AGG_AVG && !A.avg_round && A.res_type == DBG_FLOAT64) return PS_AGG(PS_AVG, t);
    return -1;
}

template <int K0, int K1, int A0, int A1, int A2>
static bool ps_match(const Spec& S) {
    typedef PsShape<K0, K1, A0, A1, A2> SH;
    const int nk = SH::NK, na = (A0 ? 1 : 0) + (A1 ? 1 : 0) + (A2 ? 1 : 0);
    if (S.pp_str || S.n_keys != nk || S.n_aggs != na || S.flags_word >= 0) return false;
    const int kt[2] = {K0, K1};
    for (int c = 0; c < nk; ++c)
        if (S.key_types[c].type != kt[c] || S.key_types[c].nullable || S.koff[c] != (c == 0 ? 0u : ps_tw(K0))) return false;
    const int ac[3] = {A0, A1, A2};
    for (int a = 0; a < na; ++a) {
        if (ps_code(S.aggs[a]) != ac[a]) return false;
        if (ps_has_arg(ac[a]) && S.pp_aoff[a] != SH::off(a)) return false;
    }
    return S.pp_rw_raw == ((SH::END + 7) & ~7u) && S.pp_kw == 8 * SH::KW && S.pp_rw_state == SH::REC_BYTES;
}

static int ps_literal_shape(const Spec& S, u32* cap, u32* max_records) {
    int id = 0, found = -1;
    u32 bw = 0, w = 0;
#define PS_TRY(WW, K0, K1, A0, A1, A2)                        \
    if (found < 0 && ps_match<K0, K1, A0, A1, A2>(S)) {     \
        found = id;                                         \
        bw = PsShape<K0, K1, A0, A1, A2>::BWL;              \
        w = WW;                                             \
    }                                                       \
    ++id;
    PS_SHAPES(PS_TRY)
#undef PS_TRY
    if (found >= 0) {
        *cap = ps_cap(bw, w, PP_LIT_NT, PS_LDS / PP_LIT_PER_CU);
        *max_records = PP_LIT_NT * PP_LIT_RPT;
    }
    return found;
}

static void launch_ps_literal(hipStream_t s, const Spec& S, int shape, int mode, u32 n_parts, const u64* raw_off, const u8* raw, u32 sub_bits,
                              const PPAggOut& out, u32* spill, u32 spill_cap) {
    if (!n_parts) return;
    const u32 grid = n_parts < 256u * PP_LIT_PER_CU ? n_parts : 256u * PP_LIT_PER_CU;  // persistent workgroups
    // test hook: a smaller LDS table than the plan assumed (probe-window misses, pending rounds)
    const u32 cap_x = S.x_pp_cap;
    int id = 0;
#define PS_LAUNCH(WW, K0, K1, A0, A1, A2)                                                                               \
    if (shape == id) {                                                                                                  \
        const u32 bw = PsShape<K0, K1, A0, A1, A2>::BWL, cap = std::min(ps_cap(bw, WW, PP_LIT_NT, PS_LDS / PP_LIT_PER_CU), cap_x); \
        const size_t lds = ps_lds_bytes(cap, bw, WW, PP_LIT_NT) + 16;                                                   \
        if (mode == 0)                                                                                                  \
            hipLaunchKernelGGL((pp_agg_spec_kernel<0, WW, PP_LIT_RPT, PP_LIT_NT, K0, K1, A0, A1, A2>), dim3(grid),         \
                               dim3(PP_LIT_NT), lds, s, n_parts, raw_off, raw, sub_bits, cap, out, spill, spill_cap);      \
        else                                                                                                            \
            hipLaunchKernelGGL((pp_agg_spec_kernel<1, WW, PP_LIT_RPT, PP_LIT_NT, K0, K1, A0, A1, A2>), dim3(grid),         \
                               dim3(PP_LIT_NT), lds, s, n_parts, raw_off, raw, sub_bits, cap, out, spill, spill_cap);      \
    }                                                                                                                   \
    ++id;
    PS_SHAPES(PS_LAUNCH)
#undef PS_LAUNCH
}

// The class above runs on the descriptor kernel; its most common shapes — C4's (Int64, Int32;
// COUNT, SUM(Int16), AVG(Int16)), one Int64 key with COUNT or COUNT + SUM(Int64), two Int64 keys
// with COUNT — also have fully compile-time instances (pp_agg_spec_kernel, PS_SHAPES), which the
// descriptor kernel cannot match yet (C4 pp_agg 36 ms compile-time, 48-53 ms from the descriptor:
// the emit and insert phases pay for the runtime kinds and widths).  Shape ids: 0.. the literal
// shapes, PS_DESC_ID + W the descriptor kernel.
#define PS_DESC_ID 64
int pp_spec_shape(const Spec& S, u32* cap, u32* max_records) {
    // test hook: the descriptor kernel for a literal shape too (same results)
    const int lit = S.x_pp_desc ? -1 : ps_literal_shape(S, cap, max_records);
    if (lit >= 0) return lit;
    const int w = ps_desc_shape(S, cap, max_records);
    return w >= 0 ? PS_DESC_ID + w : -1;
}

void launch_pp_agg_spec(hipStream_t s, const Spec& S, int shape, int mode, u32 n_parts, const u64* raw_off, const u8* raw,
                        u32 sub_bits, const PPAggOut& out, u32* spill, u32 spill_cap) {
    if (shape >= PS_DESC_ID) launch_ps_desc(s, S, shape - PS_DESC_ID, mode, n_parts, raw_off, raw, sub_bits, out, spill, spill_cap);
    else launch_ps_literal(s, S, shape, mode, n_parts, raw_off, raw, sub_bits, out, spill, spill_cap);
}

// ------------------------------------------------------------------------------------------
// group records -> result columns: per block of PP_GB rows, string bytes per key column; the
// host scans them; the write pass places rows at their index and strings at scanned offsets.
// ------------------------------------------------------------------------------------------
#define PP_GB 2048
#define PP_GNT 256
u64 pp_grec_blocks(u64 n) { return (n + PP_GB - 1) / PP_GB; }

// length of string key column c of a group record's key part (global)
__device__ __forceinline__ StrRef pp_key_str(const Spec& S, const BatchDesc* batches, const u8* k, int c, bool& valid) {
    const u8 klen = gld<u8>(k + 8);
    if (klen == PP_KLEN_LONG) {
        const u64 ref = gld<u64>(k + 16);
        const DCol& col = batches[ref_bid(ref)].keys[c];
        valid = dcol_valid(col, ref_row(ref));
        return valid ? dcol_str(col, ref_row(ref)) : StrRef{nullptr, 0};
    }
    u32 o = 9;
    for (int j = 0; j < S.n_keys; ++j) {
        bool v = true;
        if (S.key_types[j].nullable) v = gld<u8>(k + o++) != 0;
        if (S.key_types[j].type == DBG_STRING) {
            const u32 n = gld<u8>(k + o++);
            if (j == c) {
                valid = v;
                return StrRef{k + o, n};
            }
            o += n;
        } else {
            o += type_width(S.key_types[j].type);
        }
    }
    valid = false;
    return StrRef{nullptr, 0};
}
// fixed-width key column c of a blob key part (global): value bits
__device__ __forceinline__ bool pp_key_fixed(const Spec& S, const BatchDesc* batches, const u8* k, int c, u64& lo, u64& hi) {
    lo = hi = 0;
    if (!S.pp_str) {
        const dbg_datatype& t = S.key_types[c];
        const bool v = !t.nullable || gld<u8>(k + S.voff[c]) != 0;
        if (t.type == DBG_DECIMAL128) {
            lo = ld_le(k + S.koff[c], 8);
            hi = ld_le(k + S.koff[c] + 8, 8);
        } else {
            lo = ld_le(k + S.koff[c], type_width(t.type));
        }
        return v;
    }
    const u8 klen = gld<u8>(k + 8);
    if (klen == PP_KLEN_LONG) {
        const u64 ref = gld<u64>(k + 16);
        const DCol& col = batches[ref_bid(ref)].keys[c];
        const bool v = dcol_valid(col, ref_row(ref));
        if (v) {
            lo = dcol_bits(col, ref_row(ref));
            if (col.type == DBG_DECIMAL128) hi = dcol_hi(col, ref_row(ref));
            else if (col.type == DBG_FLOAT32 || col.type == DBG_FLOAT64) lo = canon_float_bits(col.type, lo);
        }
        return v;
    }
    u32 o = 9;
    for (int j = 0; j < S.n_keys; ++j) {
        bool v = true;
        if (S.key_types[j].nullable) v = gld<u8>(k + o++) != 0;
        const int ty = S.key_types[j].type;
        if (ty == DBG_STRING) {
            o += 1 + gld<u8>(k + o);
            continue;
        }
        const u32 w = type_width(ty);
        if (j == c) {
            if (ty == DBG_DECIMAL128) {
                lo = ld_le(k + o, 8);
                hi = ld_le(k + o + 8, 8);
            } else {
                lo = ld_le(k + o, w);
            }
            return v;
        }
        o += w;
    }
    return false;
}

__global__ void __launch_bounds__(PP_GNT) pp_grec_len_kernel(const Spec* __restrict__ spec, const BatchDesc* __restrict__ batches,
                                                            const u8* __restrict__ grec, const u64* __restrict__ np, u64* __restrict__ blk_len, u64 nblocks) {
    const Spec& S = *spec;
    const u64 n = *np;
    __shared__ unsigned long long acc[DBG_MAX_KEYS];
    if (threadIdx.x < DBG_MAX_KEYS) acc[threadIdx.x] = 0;
    __syncthreads();
    const u64 r0 = (u64)blockIdx.x * PP_GB;
    for (u64 r = r0 + threadIdx.x; r < r0 + PP_GB && r < n; r += PP_GNT) {
        const u8* k = grec + r * S.pp_rw_state;
        for (int c = 0; c < S.n_keys; ++c)
            if (S.key_types[c].type == DBG_STRING) {
                bool v;
                atomicAdd(&acc[c], (unsigned long long)pp_key_str(S, batches, k, c, v).len);
            }
    }
    __syncthreads();
    if (threadIdx.x < (u32)S.n_keys) blk_len[(u64)threadIdx.x * nblocks + blockIdx.x] = acc[threadIdx.x];
}

void launch_pp_grec_lengths(hipStream_t s, const Spec* dspec, const u8* grec, const u64* np, u64* blk_len, u64 nblocks,
                            const BatchDesc* batches) {
    if (!nblocks) return;
    hipLaunchKernelGGL(pp_grec_len_kernel, dim3((u32)nblocks), dim3(PP_GNT), 0, s, dspec, batches, grec, np, blk_len, nblocks);
}

__global__ void __launch_bounds__(PP_GNT) pp_grec_write_kernel(const Spec* __restrict__ spec, const BatchDesc* __restrict__ batches,
                                                              const u8* __restrict__ grec, const u64* __restrict__ np, const u64* __restrict__ str_pos,
                                                              u64 nblocks, OutDesc out, u64* err) {
    const Spec& S = *spec;
    const u64 n = *np;
    __shared__ u32 wtot[PP_GNT / 64];
    u64 srun[DBG_MAX_KEYS];
    for (int c = 0; c < S.n_keys; ++c) srun[c] = S.key_types[c].type == DBG_STRING ? str_pos[(u64)c * nblocks + blockIdx.x] : 0;
    const u64 r0 = (u64)blockIdx.x * PP_GB;
    for (u64 rb = r0; rb < r0 + PP_GB && rb < n; rb += PP_GNT) {  // uniform
        const u64 r = rb + threadIdx.x;
        const bool in = r < n && r < r0 + PP_GB;
        const u8* k = grec + (in ? r : rb) * S.pp_rw_state;
        for (int c = 0; c < S.n_keys; ++c) {
            const dbg_datatype& t = S.key_types[c];
            if (t.type == DBG_STRING) {
                bool v = false;
                StrRef sr = in ? pp_key_str(S, batches, k, c, v) : StrRef{nullptr, 0};
                u32 tot;
                const u32 pre = block_excl_scan((u32)sr.len, wtot, tot);
                if (in && r < out.cap_groups) {
                    const u64 pos = srun[c] + pre;
                    out.key_offsets[c][r] = pos;
                    if (pos + sr.len <= out.cap_str[c]) {
                        u8* d = (u8*)out.key_data[c] + pos;
                        for (u64 j = 0; j < sr.len; ++j) d[j] = gld<u8>(sr.p + j);
                    }
                    if (out.key_valid[c]) out.key_valid[c][r] = v ? 1 : 0;
                }
                srun[c] += tot;
            } else if (in && r < out.cap_groups) {
                u64 lo, hi;
                const bool v = pp_key_fixed(S, batches, k, c, lo, hi);
                write_bytes(out.key_data[c], r, type_width(t.type), lo, hi);
                if (out.key_valid[c]) out.key_valid[c][r] = v ? 1 : 0;
            }
        }
        if (in && r < out.cap_groups) {
            const u64* st = (const u64*)(k + S.pp_kw) - 1;
            for (int a = 0; a < S.n_aggs; ++a) write_agg(S, a, st, r, out, err);
        }
    }
}

void launch_pp_grec_write(hipStream_t s, const Spec* dspec, const BatchDesc* batches, const u8* grec, const u64* np, const u64* str_pos,
                          u64 nblocks, const OutDesc& out, u64* err) {
    if (!nblocks) return;
    hipLaunchKernelGGL(pp_grec_write_kernel, dim3((u32)nblocks), dim3(PP_GNT), 0, s, dspec, batches, grec, np, str_pos, nblocks, out, err);
}

// ------------------------------------------------------------------------------------------
// group records -> exchange records ([hash][validity][keys][state words], strings into
// per-partition blobs) partitioned by hash % n (Payload::scatter) or radix bits [48 - r, 48)
// (PartitionedPayload) — the same record format as the HBM table's export.
// ------------------------------------------------------------------------------------------
#define PP_MAX_PARTS 256
__device__ __forceinline__ u32 pp_part_of(u64 h, u32 n_parts, int scheme, const u32* lpart, u64 r) {
    if (n_parts <= 1) return 0;
    if (scheme == 2) return lpart[r];  // legacy bucket (pp_grec_legacy_bucket_kernel)
    if (scheme == 0) return (u32)(h % n_parts);
    const u32 rb = 31 - __clz(n_parts);
    return (u32)((h >> (48 - rb)) & (n_parts - 1));
}
__device__ __forceinline__ u64 pp_grec_hash(const Spec& S, const u8* k) { return S.pp_str ? gld<u64>(k) : pp_fixed_hash(S, k); }

__global__ void __launch_bounds__(PP_GNT) pp_grec_count_kernel(const Spec* __restrict__ spec, const BatchDesc* __restrict__ batches,
                                                              const u8* __restrict__ grec, u64 n, u32 n_parts, int scheme,
                                                              const u32* __restrict__ lpart, u64* __restrict__ hist,
                                                              u64* __restrict__ str_hist, u64 nblocks) {
    const Spec& S = *spec;
    __shared__ unsigned long long lh[PP_MAX_PARTS];
    __shared__ unsigned long long ls[DBG_MAX_KEYS][PP_MAX_PARTS];
    for (u32 p = threadIdx.x; p < n_parts; p += PP_GNT) {
        lh[p] = 0;
        for (int c = 0; c < S.n_keys; ++c) ls[c][p] = 0;
    }
    __syncthreads();
    const u64 r0 = (u64)blockIdx.x * PP_GB;
    for (u64 r = r0 + threadIdx.x; r < r0 + PP_GB && r < n; r += PP_GNT) {
        const u8* k = grec + r * S.pp_rw_state;
        const u32 p = pp_part_of(scheme == 2 ? 0 : pp_grec_hash(S, k), n_parts, scheme, lpart, r);
        atomicAdd(&lh[p], 1ULL);
        for (int c = 0; c < S.n_keys; ++c)
            if (S.key_types[c].type == DBG_STRING) {
                bool v;
                atomicAdd(&ls[c][p], (unsigned long long)pp_key_str(S, batches, k, c, v).len);
            }
    }
    __syncthreads();
    for (u32 p = threadIdx.x; p < n_parts; p += PP_GNT) {
        hist[(u64)p * nblocks + blockIdx.x] = lh[p];
        for (int c = 0; c < S.n_keys; ++c) str_hist[((u64)p * S.n_keys + c) * nblocks + blockIdx.x] = ls[c][p];
    }
}

void launch_pp_grec_count_parts(hipStream_t s, const Spec* dspec, const BatchDesc* batches, const u8* grec, u64 n, u32 n_parts,
                                int scheme, const u32* lpart, u64* hist, u64* str_hist, u64 nblocks) {
    if (!nblocks) return;
    hipLaunchKernelGGL(pp_grec_count_kernel, dim3((u32)nblocks), dim3(PP_GNT), 0, s, dspec, batches, grec, n, n_parts, scheme, lpart, hist,
                       str_hist, nblocks);
}

__global__ void __launch_bounds__(PP_GNT) pp_grec_export_kernel(const Spec* __restrict__ spec, const BatchDesc* __restrict__ batches,
                                                               const u8* __restrict__ grec, u64 n, u32 n_parts, int scheme,
                                                               const u32* __restrict__ lpart,
                                                               const u64* __restrict__ pos, const u64* __restrict__ str_pos,
                                                               u64 nblocks, u8* rec_out, u8* str_out,
                                                               const u64* __restrict__ part_str_base) {
    const Spec& S = *spec;
    __shared__ unsigned long long cur[PP_MAX_PARTS];
    __shared__ unsigned long long scur[DBG_MAX_KEYS][PP_MAX_PARTS];
    for (u32 p = threadIdx.x; p < n_parts; p += PP_GNT) {
        cur[p] = pos[(u64)p * nblocks + blockIdx.x];
        for (int c = 0; c < S.n_keys; ++c) scur[c][p] = str_pos[((u64)p * S.n_keys + c) * nblocks + blockIdx.x];
    }
    __syncthreads();
    const u64 r0 = (u64)blockIdx.x * PP_GB;
    for (u64 r = r0 + threadIdx.x; r < r0 + PP_GB && r < n; r += PP_GNT) {
        const u8* k = grec + r * S.pp_rw_state;
        const u64 h = pp_grec_hash(S, k);
        const u32 p = pp_part_of(h, n_parts, scheme, lpart, r);
        const u64 ri = atomicAdd(&cur[p], 1ULL);
        u8* rec = rec_out + ri * S.rec_width;
        *(u64*)rec = h;
        for (int c = 0; c < S.n_keys; ++c) {
            const dbg_datatype& t = S.key_types[c];
            u8* kd = rec + S.rec_key_off[c];
            if (t.type == DBG_STRING) {
                bool v = false;
                StrRef sr = pp_key_str(S, batches, k, c, v);
                if (t.nullable) rec[S.rec_val_off[c]] = v ? 1 : 0;
                const u64 o = atomicAdd(&scur[c][p], (unsigned long long)sr.len);
                for (u64 j = 0; j < sr.len; ++j) str_out[o + j] = gld<u8>(sr.p + j);
                ((u64*)kd)[0] = o - part_str_base[p];
                ((u64*)kd)[1] = sr.len;
            } else {
                u64 lo, hi;
                const bool v = pp_key_fixed(S, batches, k, c, lo, hi);
                if (t.nullable) rec[S.rec_val_off[c]] = v ? 1 : 0;
                const u32 w = type_width(t.type);
                for (u32 j = 0; j < w && j < 8; ++j) kd[j] = (u8)(lo >> (8 * j));
                for (u32 j = 8; j < w; ++j) kd[j] = (u8)(hi >> (8 * (j - 8)));
            }
        }
        u64* sw = (u64*)(rec + S.rec_state_off);
        const u64* st = (const u64*)(k + S.pp_kw);
        for (int w = 0; w < S.n_words; ++w) sw[w] = st[w];
    }
}

// Legacy bucket of every group record (enable_experimental_aggregate_hashtable = 0), as
// agg.hip legacy_slot_bucket_kernel does for the HBM table's slots.
__global__ void __launch_bounds__(PP_GNT) pp_grec_legacy_bucket_kernel(const Spec* __restrict__ spec, const BatchDesc* __restrict__ batches,
                                                                      const u8* __restrict__ grec, u64 n, LegacyLayout L,
                                                                      u32* __restrict__ out) {
    const Spec& S = *spec;
    __shared__ u32 tab[256];
    crc_table_init(tab);
    for (u64 r = blockIdx.x * (u64)PP_GNT + threadIdx.x; r < n; r += (u64)gridDim.x * PP_GNT) {
        const u8* k = grec + r * S.pp_rw_state;
        u64 h;
        if (L.binary) {
            bool v;
            const StrRef sr = pp_key_str(S, batches, k, 0, v);
            h = legacy_bytes_hash(tab, sr.p, sr.len);
        } else if (L.serializer) {
            SerCrc sc;
            for (int c = 0; c < S.n_keys; ++c) {
                const dbg_datatype& ty = S.key_types[c];
                if (ty.type == DBG_STRING) {
                    bool v;
                    const StrRef sr = pp_key_str(S, batches, k, c, v);
                    sc.column(tab, ty.type, ty.nullable, v, 0, 0, sr.p, sr.len);
                } else {
                    u64 lo, hi;
                    const bool v = pp_key_fixed(S, batches, k, c, lo, hi);
                    sc.column(tab, ty.type, ty.nullable, v, lo, hi, nullptr, 0);
                }
            }
            h = sc.finish(tab);
        } else {
            u64 kw[4] = {0, 0, 0, 0};
            for (int c = 0; c < S.n_keys; ++c) {
                u64 lo, hi;
                if (!pp_key_fixed(S, batches, k, c, lo, hi)) {
                    const u32 o = (u32)L.null_off[c];
                    kw[o >> 3] |= 1ULL << (8 * (o & 7));
                } else {
                    const u32 w = type_width(S.key_types[c].type);
                    legacy_put(kw, L.off[c], lo, w == 16 ? hi : 0, w);
                }
            }
            h = legacy_fixed_crc(tab, kw, L.words);
        }
        out[r] = legacy_bucket(h, L.bits);
    }
}

void launch_pp_grec_legacy_bucket(hipStream_t s, const Spec* dspec, const BatchDesc* batches, const u8* grec, u64 n,
                                  const LegacyLayout& L, u32* out) {
    if (!n) return;
    u64 blocks = (n + PP_GNT - 1) / PP_GNT;
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL(pp_grec_legacy_bucket_kernel, dim3((u32)blocks), dim3(PP_GNT), 0, s, dspec, batches, grec, n, L, out);
}

void launch_pp_grec_export(hipStream_t s, const Spec* dspec, const BatchDesc* batches, const u8* grec, u64 n, u32 n_parts,
                           int scheme, const u32* lpart, const u64* pos, const u64* str_pos, u64 nblocks, u8* rec_out,
                           u8* str_out, const u64* part_str_base) {
    if (!nblocks) return;
    hipLaunchKernelGGL(pp_grec_export_kernel, dim3((u32)nblocks), dim3(PP_GNT), 0, s, dspec, batches, grec, n, n_parts, scheme, lpart, pos,
                       str_pos, nblocks, rec_out, str_out, part_str_base);
}

// ------------------------------------------------------------------------------------------
// Byte-range gather (payload export / import, abi.hip dbg_agg_payload_*): one workgroup per
// range, 8-byte words (records and their offsets are multiples of 8 bytes).
// ------------------------------------------------------------------------------------------
__global__ void __launch_bounds__(256) copy_ranges_kernel(const u8* __restrict__ src, u8* __restrict__ dst,
                                                          const CopyRange* __restrict__ r, u32 n) {
    for (u32 k = blockIdx.x; k < n; k += gridDim.x) {
        const CopyRange c = r[k];
        const u64* a = (const u64*)(src + c.src);
        u64* b = (u64*)(dst + c.dst);
        for (u64 w = threadIdx.x; w < c.n / 8; w += 256) b[w] = a[w];
    }
}

void launch_copy_ranges(hipStream_t s, const u8* src, u8* dst, const CopyRange* dranges, u32 n) {
    if (!n) return;
    hipLaunchKernelGGL(copy_ranges_kernel, dim3(n < 4096 ? n : 4096), dim3(256), 0, s, src, dst, dranges, n);
}
