// part.hip — radix-partitioned insert for high-cardinality single-key COUNT(*) batches.
//
// The streaming insert (agg_insert_fast) turns every row of a high-cardinality batch into one
// random device-scope atomic on the HBM table (ClickBench Q17 shape: 1e9 rows, 1.3e8 groups, a
// 8.6 GB table): 1e9 random 64-B memory-side read-modify-writes.  Here the same batch is
// reordered first so that the table is touched slice by slice:
//
//   1. m = slot_mix(key) for every row (slot_mix is a bijection of u64), radix-partitioned on
//      the slot bits above the slice size by this file's own LSD radix partition (rp_*): one
//      histogram pass over the keys counts the digits of every pass, then each pass scatters
//      8192-row tiles through LDS — a stable wave-level ranking (8 ballots per digit), the
//      tile's digit counts published for a decoupled look-back over earlier tiles, and the
//      tile written out digit run by digit run;
//   2. part_bounds: the first sorted position of every slice (one binary search per slice);
//   3. part_slice: one workgroup per table slice: slice HBM -> LDS (64 KB) — or, when the table is
//      empty at launch (a reset whose initialisation was deferred), the slice starts EMPTY in
//      LDS and the table is not read at all — every row of the slice probes and counts in LDS
//      (same linear probing as g_find, so the table stays a valid HBM table for every other
//      kernel), LDS -> HBM.  A probe that would leave the slice (its run continues in the next
//      slice, owned by another workgroup) becomes an overflow record [key][1] that part_fixup
//      merges right after — the deferred-overflow protocol of the streaming insert.
//
// This is the reference's own answer to the same problem — AggregateHashTable radix-partitions
// its payload (EAGG/partitioned_payload.rs:100-143) so the final merge works partition by
// partition on cache-sized tables (AGG/transform_aggregate_final.rs:71-156) — applied to the
// 64 KB LDS of a CDNA4 workgroup instead of a CPU core's cache.
#include <algorithm>
#include <cstdio>
#include <cstring>

#include "agg.hpp"

#define PART_NT_DEFAULT 512  // slice-kernel workgroup: 48 KB of LDS, three per CU (DBG_X_SLICE_NT=1024: two)
#define PART_SB 12  // slice = 4096 slots x 16 B = 64 KB of LDS
#define PART_PROBE_CAP 64
#define PART_OVF_LDS 512  // overflow keys gathered per workgroup before one device atomic
#define RB 4  // sorted keys per lane per batch in the slice kernel

namespace {

// ---------------------------------------------------------------------------------------------
// LSD radix partition of m = slot_mix(key) on bits [sb, log2 cap) — 1 to 3 passes of <= 8 bits
// ---------------------------------------------------------------------------------------------
// scatter tile shapes (threads x rows per thread) are template parameters; rp_shape() picks one
#define RP_MAXP 3
#define RP_HIST_NT 256
#define RP_HIST_BLOCKS 2048
// look-back status words: [flag 2 b | count 62 b]; flag 1 = this tile's count, 2 = inclusive prefix
#define RP_AGG (1ULL << 62)
#define RP_INC (2ULL << 62)
#define RP_VAL ((1ULL << 62) - 1)

struct RadixPlan {
    u32 npass;
    u32 shift[RP_MAXP];
    u32 bits[RP_MAXP];
};

template <int W>
__device__ __forceinline__ u64 rp_key(const u8* p, u64 i) {
    if (W == 1) return gld<u8>(p + i);
    if (W == 2) return gld<uint16_t>(p + 2 * i);
    if (W == 4) return gld<uint32_t>(p + 4 * i);
    return gld<u64>(p + 8 * i);
}

// Digit counts of every pass in one read of the keys: per-workgroup LDS histograms, then one
// device atomic per non-empty bin.  hist[p * 256 + d] (u32: a batch holds < 2^32 rows).
template <int W>
__global__ void __launch_bounds__(RP_HIST_NT) rp_hist_kernel(const u8* __restrict__ keys, u64 rows, RadixPlan P,
                                                             u32* __restrict__ hist) {
    __shared__ u32 h[RP_MAXP][256];
    for (u32 i = threadIdx.x; i < RP_MAXP * 256; i += RP_HIST_NT) (&h[0][0])[i] = 0;
    __syncthreads();
    const u64 per = (rows + gridDim.x - 1) / gridDim.x;
    const u64 lo = min<u64>(rows, (u64)blockIdx.x * per), hi = min<u64>(rows, lo + per);
    constexpr int U = 8;  // independent loads in flight per lane
    u64 i = lo + threadIdx.x;
    for (; i + (u64)(U - 1) * RP_HIST_NT < hi; i += (u64)U * RP_HIST_NT) {
        u64 v[U];
#pragma unroll
        for (int k = 0; k < U; ++k) v[k] = rp_key<W>(keys, i + (u64)k * RP_HIST_NT);
#pragma unroll
        for (int k = 0; k < U; ++k) {
            const u64 m = slot_mix(v[k]);
            for (u32 p = 0; p < P.npass; ++p) atomicAdd(&h[p][(m >> P.shift[p]) & ((1u << P.bits[p]) - 1)], 1u);
        }
    }
    for (; i < hi; i += RP_HIST_NT) {
        const u64 m = slot_mix(rp_key<W>(keys, i));
        for (u32 p = 0; p < P.npass; ++p) atomicAdd(&h[p][(m >> P.shift[p]) & ((1u << P.bits[p]) - 1)], 1u);
    }
    __syncthreads();
    for (u32 x = threadIdx.x; x < P.npass * 256; x += RP_HIST_NT) {
        const u32 c = (&h[0][0])[x];
        if (c) atomicAdd(hist + x, c);
    }
}

// Exclusive prefix sum of one value per thread over threads 0..255 (the first four waves; other
// threads pass 0 and get a meaningless result).  Called by every thread of the workgroup (it
// synchronises); tmp: 8 words of LDS.
__device__ __forceinline__ u64 scan256(u64 v, u64* tmp) {
    const u32 lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    u64 x = v;  // inclusive scan inside the wave
#pragma unroll
    for (u32 o = 1; o < 64; o <<= 1) {
        const u64 y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63 && w < 4) tmp[w] = x;
    __syncthreads();
    u64 add = 0;
    for (u32 k = 0; k < w && k < 4; ++k) add += tmp[k];
    __syncthreads();  // tmp may be reused by the caller
    return add + x - v;
}

// One scatter pass.  RAW: the source is the key column (width W; m = slot_mix(key) on the fly),
// else the previous pass's m.  Tiles are taken in order from a device counter, so every tile's
// predecessors are running or done when it looks back (no circular wait).  Rows keep their
// relative order within a digit (LSD needs a stable pass): a wave ranks its 16 rounds of 64
// rows in order, lanes ranked among equal digits by ballot, wave counts prefixed in wave order.
// Measured and not kept (round 6): the next tile's rows loaded into registers while the current
// tile is ranked (a second register set: 168 VGPRs, C3 insert 16.7 -> 19.1 ms) or while it is
// written out (the same registers, but the loads in flight still held them: 138 VGPRs, 19.2 ms).
template <int W, bool RAW, int RP_NT, int RP_IPT>
__global__ void __launch_bounds__(RP_NT) rp_scatter_kernel(const u8* __restrict__ src, u64 rows, u32 shift, u32 bits,
                                                           const u32* __restrict__ hist, u64* __restrict__ status,
                                                           u32* __restrict__ tile_ctr, u64* __restrict__ dst) {
    constexpr int RP_TILE = RP_NT * RP_IPT, RP_WAVES = RP_NT / 64, RP_WROWS = 64 * RP_IPT;
    __shared__ __attribute__((aligned(16))) u64 stage[RP_TILE];
    __shared__ u32 wcnt[RP_WAVES][256];  // per wave: digit counts, then their exclusive prefix over waves
    __shared__ u32 lstart[256];           // tile-local start of every digit
    __shared__ u64 gstart[256];           // global start of every digit's run of this tile
    __shared__ u32 s_tile;
    __shared__ u64 scan_tmp[16];
    const u32 tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const u32 nb = 1u << bits, dmask = nb - 1;
    const u32 ntiles = (u32)((rows + RP_TILE - 1) / RP_TILE);
    // persistent: each workgroup takes tiles in order from the counter, the next one while it
    // works on the current (the grab's latency off the tile's critical path); tiles only ever
    // wait on smaller tiles, so holding a not-yet-started tile cannot deadlock
    if (tid == 0) s_tile = atomicAdd(tile_ctr, 1u);
    __syncthreads();
    u32 tile = s_tile;
    while (tile < ntiles) {
    u32 next_tile = 0;
    if (tid == 0) next_tile = atomicAdd(tile_ctr, 1u);
    for (u32 i = tid; i < RP_WAVES * 256; i += RP_NT) (&wcnt[0][0])[i] = 0;
    __syncthreads();
    const u64 base = (u64)tile * RP_TILE;
    const u64 e0 = base + (u64)w * RP_WROWS + lane;  // this lane's row of round 0
    u64 m[RP_IPT];
#pragma unroll
    for (int r = 0; r < RP_IPT; ++r) {
        const u64 e = e0 + (u64)r * 64;
        if (e < rows) {
            if (RAW) m[r] = rp_key<W>(src, e);
            else m[r] = gld<u64>(src + 8 * e);
        }
    }
    // stable ranking, round by round
    u32 rank[RP_IPT];
    const u64 lt = (1ULL << lane) - 1;
#pragma unroll
    for (int r = 0; r < RP_IPT; ++r) {
        const u64 e = e0 + (u64)r * 64;
        const bool ok = e < rows;
        if (RAW && ok) m[r] = slot_mix(m[r]);
        const u32 d = ok ? (u32)(m[r] >> shift) & dmask : 0;
        u64 peers = __ballot(ok);
        for (u32 b = 0; b < bits; ++b) {
            const u64 bb = __ballot((d >> b) & 1);
            peers &= ((d >> b) & 1) ? bb : ~bb;
        }
        u32 old = 0;
        if (ok) old = wcnt[w][d];
        __builtin_amdgcn_wave_barrier();
        const bool leader = ok && (peers & lt) == 0;
        if (leader) wcnt[w][d] = old + (u32)__popcll(peers);
        __builtin_amdgcn_wave_barrier();
        rank[r] = old + (u32)__popcll(peers & lt);
    }
    __syncthreads();
    // digit totals of the tile, per-wave exclusive prefixes, local digit starts
    u32 tot = 0;
    if (tid < 256) {
        for (u32 x = 0; x < RP_WAVES; ++x) {
            const u32 c = wcnt[x][tid];
            wcnt[x][tid] = tot;
            tot += c;
        }
        if (tid >= nb) tot = 0;
    }
    // publish this tile's counts (a tile without predecessors publishes its inclusive prefix)
    if (tid < nb) {
        u64* st = status + (u64)tile * 256 + tid;
        __hip_atomic_store(st, (tile == 0 ? RP_INC : RP_AGG) | (u64)tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    // exclusive scans over the 256 digits: the tile's counts (local starts) and the pass
    // histogram (the digit's first row in the output)
    const u32 lst = scan256(tid < 256 ? tot : 0u, scan_tmp);
    const u64 hst = scan256(tid < nb ? hist[tid] : 0u, scan_tmp + 8);
    if (tid < 256) lstart[tid] = lst;
    // decoupled look-back: the rows of digit d in every earlier tile
    if (tid < nb) {
        u64 acc = 0;
        if (tile > 0) {
            const u64* sp = status + (u64)(tile - 1) * 256 + tid;
            for (;;) {
                const u64 v = __hip_atomic_load((u64*)sp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                if (v == 0) {
                    __builtin_amdgcn_s_sleep(1);
                    continue;
                }
                acc += v & RP_VAL;
                if (v & RP_INC) break;
                sp -= 256;
            }
            __hip_atomic_store(status + (u64)tile * 256 + tid, RP_INC | (acc + tot), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        gstart[tid] = hst + acc;
    }
    __syncthreads();
    // rows to LDS in digit order
#pragma unroll
    for (int r = 0; r < RP_IPT; ++r) {
        const u64 e = e0 + (u64)r * 64;
        if (e < rows) {
            const u32 d = (u32)(m[r] >> shift) & dmask;
            stage[lstart[d] + wcnt[w][d] + rank[r]] = m[r];
        }
    }
    __syncthreads();
    // LDS -> HBM: consecutive lanes write consecutive words of one digit's run
    const u32 n = (u32)min<u64>(RP_TILE, rows - base);
    for (u32 j = tid; j < n; j += RP_NT) {
        const u64 v = stage[j];
        const u32 d = (u32)(v >> shift) & dmask;
        dst[gstart[d] + (j - lstart[d])] = v;
    }
    if (tid == 0) s_tile = next_tile;
    __syncthreads();  // stage / lstart / gstart are rewritten by the next tile
    tile = s_tile;
    }
}

__device__ __forceinline__ u64 bucket_of(u64 m, u64 mask, u32 sb) { return (m & mask) >> sb; }

// first sorted position of every slice b in [0, n_slices]; bounds[n_slices] = rows
__global__ void __launch_bounds__(256) part_bounds_kernel(const u64* __restrict__ sorted, u64 rows, u64 mask, u32 sb,
                                                          u64 n_slices, u64* __restrict__ bounds) {
    u64 b = blockIdx.x * (u64)blockDim.x + threadIdx.x;
    if (b > n_slices) return;
    u64 lo = 0, hi = rows;  // first index with bucket >= b
    while (lo < hi) {
        u64 mid = lo + (hi - lo) / 2;
        if (bucket_of(sorted[mid], mask, sb) < b) lo = mid + 1;
        else hi = mid;
    }
    bounds[b] = lo;
}

typedef unsigned long long v2u64 __attribute__((ext_vector_type(2)));

// One workgroup per table slice [b * S, (b + 1) * S), S = 2^SB slots.  COUNT(*) only: slot =
// [entry][count].  The slice size is a compile-time constant so that the slice's loads (S / NT
// 16-byte vectors per lane) are all in flight together before the first LDS store waits on
// them: one memory latency per workgroup, not one per load.
// EMPTY: the table holds no group and was not initialised (a deferred reset): the slice starts
// as EMPTY entries with zero counts in LDS, and the kernel writes every slot of it.
template <int SB, bool EMPTY, int PART_NT>
__global__ void __launch_bounds__(PART_NT) part_slice_kernel(const u64* __restrict__ sorted, const u64* __restrict__ bounds,
                                                             TableDesc t) {
    extern __shared__ __attribute__((aligned(16))) u64 lds[];
    __shared__ u32 lclaims, novf;
    __shared__ u64 ovfq[PART_OVF_LDS];
    __shared__ u64 ovf_base;
    constexpr u64 S = 1ULL << SB;
    constexpr int PER = (int)(S / PART_NT);
    static_assert(PER >= 1 && S % PART_NT == 0, "slice size");
    const u64 b = blockIdx.x;
    const u64 s0 = b * S;
    const u64 mask = t.cap - 1;
    const u64 lo = bounds[b], hi = bounds[b + 1];
    // slice -> LDS: keys [S] u64, then this launch's counts [S] u32 (a slice receives < 2^32 rows;
    // the table's own counts stay in registers and are added back at write-out), 48 KB: three
    // workgroups per CU
    const v2u64 __attribute__((address_space(1)))* gsl = (const v2u64 __attribute__((address_space(1)))*)(t.slots + s0 * 2);
    u64* lkey = lds;
    u32* lcnt = (u32*)(lds + S);
    v2u64 sv[PER];
#pragma unroll
    for (int k = 0; k < PER; ++k) {
        if (EMPTY) sv[k] = v2u64{SLOT_EMPTY, 0ULL};
        else sv[k] = gsl[threadIdx.x + k * PART_NT];
    }
    // the slice's first sorted keys are loaded before the slice reaches LDS (independent loads,
    // all in flight together); later batches are loaded one batch ahead of their processing
    const u64 __attribute__((address_space(1)))* src = (const u64 __attribute__((address_space(1)))*)sorted;
    const u64 last = hi > lo ? hi - 1 : 0;
    u64 r = lo + threadIdx.x;
    u64 cur[RB];
#pragma unroll
    for (int k = 0; k < RB; ++k) cur[k] = src[min<u64>(r + (u64)k * PART_NT, last)];
    if (threadIdx.x == 0) lclaims = novf = 0;
#pragma unroll
    for (int k = 0; k < PER; ++k) {
        lkey[threadIdx.x + k * PART_NT] = sv[k].x;
        lcnt[threadIdx.x + k * PART_NT] = 0;
    }
    __syncthreads();
    u32 my_claims = 0;
    auto push_rec = [&](u64 key) {
        u64 k = atomicAdd((unsigned long long*)(t.counters + CNT_OVF_RECS), 1ULL);
        if (k < t.ovf_recs_cap) {
            u64* rec = t.ovf_recs + k * t.stride_words;
            rec[0] = key;
            rec[1] = 1;
        } else {
            atomicOr((unsigned long long*)(t.counters + CNT_ERR), (unsigned long long)ERR_OVF_LOST);
        }
    };
    // Probe state machine with one loop exit (the SQ_INSTS_SALU count of a loop with several
    // divergent returns was ~3x its VALU count: exec-mask bookkeeping per exit).  Plain LDS
    // loads are enough: an entry, once set, never changes, and an EMPTY read that went stale is
    // corrected by the CAS's return value.
    auto one = [&](u64 m) {
        const u64 key = slot_unmix(m);
        u32 ls = (u32)((m & mask) - s0);
        const u32 lim = (u32)min<u64>(S, (u64)ls + PART_PROBE_CAP);
        int st = key == SLOT_EMPTY ? 2 : 0;  // 0 probing, 1 found at ls, 2 sentinel key, 3 overflow
        while (st == 0) {
            wptr<AS_LDS> e = asp<AS_LDS>(lkey + ls);
            u64 ev = *e;
            if (ev == SLOT_EMPTY) {
                const u64 old = at_cas<AS_LDS>(e, SLOT_EMPTY, key);
                my_claims += old == SLOT_EMPTY ? 1u : 0u;
                ev = old == SLOT_EMPTY ? key : old;
            }
            if (ev == key) st = 1;
            else if (++ls >= lim) st = 3;
        }
        if (st == 1) {
            __hip_atomic_fetch_add((__attribute__((address_space(3))) u32*)(lcnt + ls), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        } else if (st == 2) {  // the sentinel slot (index cap) is outside every slice
            wptr<AS_GLB> sent = asp<AS_GLB>(t.slots + t.cap * 2);
            u64 old = at_cas<AS_GLB>(sent, SLOT_EMPTY, 0ULL);
            if (old == SLOT_EMPTY) atomicAdd((unsigned long long*)(t.counters + CNT_CLAIMS), 1ULL);
            at_add<AS_GLB>(sent + 1, 1ULL);
        } else {
            // the run leaves the slice (or is long): an overflow record, merged by part_fixup.
            // Gathered in LDS and reserved with one device atomic per workgroup, not one
            // device-scope atomic per row on a single counter.
            const u32 q = atomicAdd(&novf, 1u);
            if (q < PART_OVF_LDS) ovfq[q] = key;
            else push_rec(key);
        }
    };
    // RB keys per lane in process, the next RB in flight
    while (r < hi) {
        const u64 rn = r + (u64)RB * PART_NT;
        u64 nxt[RB];
        if (rn < hi) {
#pragma unroll
            for (int k = 0; k < RB; ++k) nxt[k] = src[min<u64>(rn + (u64)k * PART_NT, last)];
        }
#pragma unroll
        for (int k = 0; k < RB; ++k)
            if (r + (u64)k * PART_NT < hi) one(cur[k]);
        if (rn >= hi) break;
#pragma unroll
        for (int k = 0; k < RB; ++k) cur[k] = nxt[k];
        r = rn;
    }
    if (my_claims) atomicAdd(&lclaims, my_claims);
    __syncthreads();
    const u32 nq = min<u32>(novf, PART_OVF_LDS);
    if (nq) {
        if (threadIdx.x == 0) ovf_base = atomicAdd((unsigned long long*)(t.counters + CNT_OVF_RECS), (unsigned long long)nq);
        __syncthreads();
        for (u32 i = threadIdx.x; i < nq; i += PART_NT) {
            const u64 k = ovf_base + i;
            if (k < t.ovf_recs_cap) {
                u64* rec = t.ovf_recs + k * t.stride_words;
                rec[0] = ovfq[i];
                rec[1] = 1;
            } else {
                atomicOr((unsigned long long*)(t.counters + CNT_ERR), (unsigned long long)ERR_OVF_LOST);
            }
        }
    }
    v2u64 __attribute__((address_space(1)))* osl = (v2u64 __attribute__((address_space(1)))*)(t.slots + s0 * 2);
#pragma unroll
    for (int k = 0; k < PER; ++k) {
        const u32 i = threadIdx.x + k * PART_NT;
        osl[i] = v2u64{lkey[i], sv[k].y + (u64)lcnt[i]};
    }
    if (threadIdx.x == 0 && lclaims) atomicAdd((unsigned long long*)(t.counters + CNT_CLAIMS), (unsigned long long)lclaims);
}

// Direct variant for a recycled one-shot step (reset -> add_groups -> finalize_into with
// dbg_agg_set_recycle, the table empty when the batch arrived): the groups reach the result
// columns without a table-wide count and write pass.  Two kernels:
//   part_slice_direct_kernel (one workgroup per slice): the slice's LDS table is self-contained
//     (a probe wraps around inside the slice instead of continuing into the next one, so no
//     overflow record is needed); its groups are written compacted, as (key, count) pairs, to the
//     start of the slice's own 64 KB of the table (which the step does not keep: it is left
//     uninitialised, like a reset table), and its group count to counts[b];
//   part_direct_emit_kernel (one workgroup per 64 slices, chunk ids from a ticket): the chunk's
//     group offset by a decoupled look-back over chunk totals (every count is known, so no chunk
//     waits on work), then the pairs copied to the result columns; the last workgroup appends the
//     all-ones key (the table's sentinel slot: only an 8-byte key can take it) and writes the total.
// (One kernel with a look-back per slice measured slower, 8.9 vs 7.6 ms for C3's table stage and
// finalize: a slice's results wait for every earlier slice's rows, so the slowest slice of the
// resident window held up all the others.)
// A slice with more distinct keys than its 4096 slots, or more groups than the result columns
// hold, makes totals[0] = ~0: the host then replays the regular slice kernel from the same sorted
// keys (the table path), which reports short buffers with the table intact.
//   status: [n_slices] counts, [n_chunks] look-back words, then ticket, sentinel rows, fail, done
#define PD_CHUNK 64
template <int SB, int PART_NT>
__global__ void __launch_bounds__(PART_NT) part_slice_direct_kernel(const u64* __restrict__ sorted, const u64* __restrict__ bounds,
                                                                    u64 n_slices, u64 cap, u64* __restrict__ slots, u64* __restrict__ status) {
    extern __shared__ __attribute__((aligned(16))) u64 lds[];
    __shared__ u32 wtot[PART_NT / 64];
    __shared__ u32 s_fail;
    constexpr u32 S = 1u << SB;
    constexpr int PER = (int)(S / PART_NT);
    static_assert(PER >= 1 && S % PART_NT == 0, "slice size");
    const u32 tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const u64 n_chunks = (n_slices + PD_CHUNK - 1) / PD_CHUNK;
    u64* tail = status + n_slices + n_chunks;  // ticket, sentinel rows, fail, done
    u64* lkey = lds;
    u32* lcnt = (u32*)(lds + S);
    if (tid == 0) s_fail = 0;
#pragma unroll
    for (int k = 0; k < PER; ++k) {
        lkey[tid + k * PART_NT] = SLOT_EMPTY;
        lcnt[tid + k * PART_NT] = 0;
    }
    const u64 b = blockIdx.x;
    const u64 s0 = b * S, mask = cap - 1;
    const u64 lo = bounds[b], hi = bounds[b + 1];
    const u64 __attribute__((address_space(1)))* src = (const u64 __attribute__((address_space(1)))*)sorted;
    const u64 last = hi > lo ? hi - 1 : 0;
    u64 r = lo + tid;
    u64 cur[RB];
#pragma unroll
    for (int k = 0; k < RB; ++k) cur[k] = src[min<u64>(r + (u64)k * PART_NT, last)];
    __syncthreads();
    u32 sent = 0;  // rows of the all-ones key seen by this thread
    bool fail = false;
    auto one = [&](u64 m) {
        const u64 key = slot_unmix(m);
        if (key == SLOT_EMPTY) {
            ++sent;
            return;
        }
        u32 ls = (u32)((m & mask) - s0);
        u32 q = 0;
        int st = 0;  // 0 probing, 1 found, 3 slice full
        while (st == 0) {
            wptr<AS_LDS> e = asp<AS_LDS>(lkey + ls);
            u64 ev = *e;
            if (ev == SLOT_EMPTY) {
                const u64 old = at_cas<AS_LDS>(e, SLOT_EMPTY, key);
                ev = old == SLOT_EMPTY ? key : old;
            }
            if (ev == key) st = 1;
            else if (++q >= S) st = 3;
            else ls = (ls + 1) & (S - 1);
        }
        if (st == 1) __hip_atomic_fetch_add((__attribute__((address_space(3))) u32*)(lcnt + ls), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        else fail = true;
    };
    while (r < hi) {
        const u64 rn = r + (u64)RB * PART_NT;
        u64 nxt[RB];
        if (rn < hi) {
#pragma unroll
            for (int k = 0; k < RB; ++k) nxt[k] = src[min<u64>(rn + (u64)k * PART_NT, last)];
        }
#pragma unroll
        for (int k = 0; k < RB; ++k)
            if (r + (u64)k * PART_NT < hi) one(cur[k]);
        if (rn >= hi) break;
#pragma unroll
        for (int k = 0; k < RB; ++k) cur[k] = nxt[k];
        r = rn;
    }
    if (sent) atomicAdd((unsigned long long*)(tail + 1), (unsigned long long)sent);
    if (fail) s_fail = 1;
    __syncthreads();
    // this thread's PER consecutive slots: occupied count, block exclusive scan
    u32 occ = 0;
#pragma unroll
    for (int k = 0; k < PER; ++k) occ += lkey[tid * PER + k] != SLOT_EMPTY ? 1u : 0u;
    u32 x = occ;
#pragma unroll
    for (u32 o = 1; o < 64; o <<= 1) {
        const u32 y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) wtot[wave] = x;
    __syncthreads();
    u32 off = x - occ, total = 0;
#pragma unroll
    for (u32 w = 0; w < PART_NT / 64; ++w) {
        off += w < wave ? wtot[w] : 0u;
        total += wtot[w];
    }
    // the slice's pairs, compacted at the start of its own table region
    v2u64 __attribute__((address_space(1)))* osl = (v2u64 __attribute__((address_space(1)))*)(slots + s0 * 2);
#pragma unroll
    for (int k = 0; k < PER; ++k) {
        const u64 key = lkey[tid * PER + k];
        if (key == SLOT_EMPTY) continue;
        osl[off++] = v2u64{key, (u64)lcnt[tid * PER + k]};
    }
    if (tid == 0) {
        status[b] = total;
        if (s_fail) atomicOr((unsigned long long*)(tail + 2), 1ULL);
    }
}

template <int KW>
__global__ void __launch_bounds__(1024) part_direct_emit_kernel(const u64* __restrict__ slots, u64 n_slices, u64* __restrict__ status,
                                                                u8* __restrict__ out_key, u64* __restrict__ out_cnt, u64 cap_groups,
                                                                u64* __restrict__ totals) {
    constexpr u32 S = 1u << PART_SB;
    __shared__ u64 pre[PD_CHUNK + 1];
    __shared__ u32 s_chunk, s_last;
    __shared__ u64 s_base;
    const u32 tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const u64 n_chunks = (n_slices + PD_CHUNK - 1) / PD_CHUNK;
    u64* look = status + n_slices;
    u64* tail = look + n_chunks;
    if (tid == 0) s_chunk = (u32)atomicAdd((unsigned long long*)tail, 1ULL);
    __syncthreads();
    const u64 q = s_chunk;
    const u64 b0 = q * PD_CHUNK, nb = min<u64>(PD_CHUNK, n_slices - b0);
    if (wave == 0) {  // the chunk's counts, their inclusive scan, the chunk's offset
        u64 c = lane < nb ? status[b0 + lane] : 0, x = c;
#pragma unroll
        for (u32 o = 1; o < 64; o <<= 1) {
            const u64 y = __shfl_up(x, o, 64);
            if (lane >= o) x += y;
        }
        pre[lane] = x - c;
        const u64 tot = __shfl(x, 63, 64);
        if (lane == 0) {
            u64 acc = 0;
            if (q == 0) {
                __hip_atomic_store(look, RP_INC | tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            } else {
                __hip_atomic_store(look + q, RP_AGG | tot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                const u64* sp = look + q - 1;
                for (;;) {
                    const u64 v = __hip_atomic_load((u64*)sp, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    if (v == 0) {
                        __builtin_amdgcn_s_sleep(1);
                        continue;
                    }
                    acc += v & RP_VAL;
                    if (v & RP_INC) break;
                    --sp;
                }
                __hip_atomic_store(look + q, RP_INC | (acc + tot), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            s_base = acc;
            pre[PD_CHUNK] = tot;
        }
    }
    __syncthreads();
    // each wave copies whole slices: lanes stride over the slice's pairs
    for (u32 j = wave; j < nb; j += 1024 / 64) {
        const u64 b = b0 + j;
        const u64 n = (j + 1 < nb ? pre[j + 1] : pre[PD_CHUNK]) - pre[j];
        const u64 row0 = s_base + pre[j];
        const v2u64 __attribute__((address_space(1)))* isl = (const v2u64 __attribute__((address_space(1)))*)(slots + b * S * 2);
        for (u64 i = lane; i < n; i += 64) {
            const v2u64 pr = isl[i];
            const u64 row = row0 + i;
            if (row >= cap_groups) break;
            if (KW == 8) ((u64*)out_key)[row] = pr.x;
            else if (KW == 4) ((u32*)out_key)[row] = (u32)pr.x;
            else if (KW == 2) ((uint16_t*)out_key)[row] = (uint16_t)pr.x;
            else out_key[row] = (u8)pr.x;
            out_cnt[row] = pr.y;
        }
    }
    // the last workgroup: sentinel group, total (or the failure mark ~0)
    if (tid == 0) {
        __threadfence();
        s_last = atomicAdd((unsigned long long*)(tail + 3), 1ULL) == n_chunks - 1;
    }
    __syncthreads();
    if (s_last && tid == 0) {
        __threadfence();
        const u64 grand = __hip_atomic_load(look + n_chunks - 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) & RP_VAL;
        const u64 ns = __hip_atomic_load(tail + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        bool bad = __hip_atomic_load(tail + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0 || grand > cap_groups;
        u64 n = grand;
        if (ns && !bad) {
            if (KW == 8 && grand < cap_groups) {  // only an 8-byte key can be all ones
                ((u64*)out_key)[grand] = SLOT_EMPTY;
                out_cnt[grand] = ns;
                n = grand + 1;
            } else {
                bad = true;
            }
        }
        totals[0] = bad ? ~0ULL : n;
    }
}

// Merge the overflow records of this launch (and any still pending) into the HBM table right
// away, so finalize sees no pending overflow and needs no second round.  Merged records are
// tombstoned (entry = EMPTY, never a record key in inline mode: the all-ones key lives in the
// sentinel slot); the last workgroup clears the record count when nothing failed — otherwise
// the survivors stay for resolve_overflow (growth + agg_retry, which skips tombstones).
// counters[CNT_FIX_FAIL], counters[CNT_FIX_TICKET]: scratch, left at zero.
__global__ void __launch_bounds__(256) part_fixup_kernel(TableDesc t) {
    __shared__ u32 s_claims, s_fails, s_last;
    if (threadIdx.x == 0) s_claims = s_fails = 0;
    __syncthreads();
    const u64 n = min<u64>(ld_sc1(t.counters + CNT_OVF_RECS), t.ovf_recs_cap);
    const u64 mask = t.cap - 1;
    const u32 limit = (u32)min<u64>(t.cap, 4096);
    u32 claims = 0, fails = 0;
    for (u64 k = blockIdx.x * 256ULL + threadIdx.x; k < n; k += (u64)gridDim.x * 256) {
        u64* r = t.ovf_recs + k * t.stride_words;
        const u64 key = r[0];
        if (key == SLOT_EMPTY) continue;
        u64 s = slot_mix(key) & mask;
        bool done = false;
        for (u32 p = 0; p < limit; ++p) {
            wptr<AS_GLB> e = asp<AS_GLB>(t.slots + s * 2);
            u64 ev = vld<AS_GLB>(e);
            if (ev == SLOT_EMPTY) {
                u64 old = at_cas<AS_GLB>(e, SLOT_EMPTY, key);
                if (old == SLOT_EMPTY) claims++;
                ev = old == SLOT_EMPTY ? key : old;
            }
            if (ev == key) {
                at_add<AS_GLB>(e + 1, r[1]);
                done = true;
                break;
            }
            s = (s + 1) & mask;
        }
        if (done) r[0] = SLOT_EMPTY;
        else fails++;
    }
    if (claims) atomicAdd(&s_claims, claims);
    if (fails) atomicAdd(&s_fails, fails);
    __syncthreads();
    if (threadIdx.x == 0) {
        if (s_claims) atomicAdd((unsigned long long*)(t.counters + CNT_CLAIMS), (unsigned long long)s_claims);
        if (s_fails) atomicAdd((unsigned long long*)(t.counters + CNT_FIX_FAIL), (unsigned long long)s_fails);
        __threadfence();
        u64 ticket = atomicAdd((unsigned long long*)(t.counters + CNT_FIX_TICKET), 1ULL);
        s_last = ticket == gridDim.x - 1;
    }
    __syncthreads();
    if (s_last && threadIdx.x == 0) {
        __threadfence();
        if (ld_sc1(t.counters + CNT_FIX_FAIL) == 0) atomicExch((unsigned long long*)(t.counters + CNT_OVF_RECS), 0ULL);
        atomicExch((unsigned long long*)(t.counters + CNT_FIX_FAIL), 0ULL);
        atomicExch((unsigned long long*)(t.counters + CNT_FIX_TICKET), 0ULL);
    }
}

u32 log2u(u64 x) { return 63 - __builtin_clzll(x); }

// Passes over the digit bits [sb, log2 cap): at most 8 bits each, low digit first (LSD).
RadixPlan rp_plan(u32 sb, u64 cap) {
    RadixPlan P;
    memset(&P, 0, sizeof(P));
    const u32 D = log2u(cap) - sb;
    P.npass = (D + 7) / 8;
    u32 sh = sb;
    for (u32 p = 0; p < P.npass; ++p) {
        const u32 left = D - (sh - sb);
        P.bits[p] = (left + (P.npass - p) - 1) / (P.npass - p);  // as even as possible
        P.shift[p] = sh;
        sh += P.bits[p];
    }
    return P;
}

// scatter tile shape: (threads, rows per thread); DBG_X_RP="NT,IPT" overrides it (experiments)
struct RpShape {
    int nt, ipt;
};
RpShape rp_shape() {
    static RpShape sh = [] {
        RpShape r{512, 16};
        if (const char* e = X_ENV("DBG_X_RP")) {
            int a = 0, b = 0;
            if (sscanf(e, "%d,%d", &a, &b) == 2) r = RpShape{a, b};
        }
        return r;
    }();
    return sh;
}
u64 rp_tile_rows() { return (u64)rp_shape().nt * rp_shape().ipt; }
u64 rp_tiles(u64 rows) { return (rows + rp_tile_rows() - 1) / rp_tile_rows(); }

// temp layout: [alt rows u64][status tiles x 256 u64][hist RP_MAXP x 256 u32][tile counters RP_MAXP u32]
size_t rp_status_off(u64 rows) { return (size_t)rows * 8; }
size_t rp_hist_off(u64 rows) { return rp_status_off(rows) + (size_t)rp_tiles(rows) * 256 * 8; }
size_t rp_temp_bytes(u64 rows) { return rp_hist_off(rows) + RP_MAXP * 256 * 4 + RP_MAXP * 4 + 64; }

template <int W>
void rp_launch_hist(hipStream_t s, const u8* keys, u64 rows, const RadixPlan& P, u32* hist) {
    const u32 blocks = (u32)std::max<u64>(1, std::min<u64>(RP_HIST_BLOCKS, (rows + 8191) / 8192));
    hipLaunchKernelGGL(rp_hist_kernel<W>, dim3(blocks), dim3(RP_HIST_NT), 0, s, keys, rows, P, hist);
}

hipError_t rp_sort(hipStream_t s, int width, const u8* keys, u64 rows, const RadixPlan& P, u8* temp, u64* out,
                   const char** step) {
    u64* alt = (u64*)temp;
    u64* status = (u64*)(temp + rp_status_off(rows));
    u32* hist = (u32*)(temp + rp_hist_off(rows));
    u32* ctr = hist + RP_MAXP * 256;
    const u64 tiles = rp_tiles(rows);
    hipError_t e;
    *step = "rp_hist";
    if ((e = hipMemsetAsync(hist, 0, RP_MAXP * 256 * 4 + RP_MAXP * 4, s)) != hipSuccess) return e;
    switch (width) {
        case 1: rp_launch_hist<1>(s, keys, rows, P, hist); break;
        case 2: rp_launch_hist<2>(s, keys, rows, P, hist); break;
        case 4: rp_launch_hist<4>(s, keys, rows, P, hist); break;
        default: rp_launch_hist<8>(s, keys, rows, P, hist); break;
    }
    if ((e = hipGetLastError()) != hipSuccess) return e;
    // the last pass writes `out`: passes alternate between out and alt backwards from it
    for (u32 p = 0; p < P.npass; ++p) {
        *step = "rp_scatter";
        u64* dst = ((P.npass - 1 - p) % 2 == 0) ? out : alt;
        const u8* src = p == 0 ? keys : (const u8*)(((P.npass - p) % 2 == 0) ? out : alt);
        if ((e = hipMemsetAsync(status, 0, (size_t)tiles * 256 * 8, s)) != hipSuccess) return e;
        const dim3 g((u32)std::min<u64>(tiles, 2 * 256));  // persistent: two workgroups per CU
        u32* h = hist + p * 256;
        u32* tc = ctr + p;
        const RpShape sh = rp_shape();
#define RP_GO(WW, RAWF, NTT, IPTT) \
    hipLaunchKernelGGL((rp_scatter_kernel<WW, RAWF, NTT, IPTT>), g, dim3(NTT), 0, s, src, rows, P.shift[p], P.bits[p], h, status, tc, dst)
#define RP_SHAPES(WW, RAWF)                                                      \
    if (sh.nt == 1024 && sh.ipt == 8) RP_GO(WW, RAWF, 1024, 8);                   \
    else if (sh.nt == 256 && sh.ipt == 16) RP_GO(WW, RAWF, 256, 16);              \
    else if (sh.nt == 512 && sh.ipt == 8) RP_GO(WW, RAWF, 512, 8);                \
    else if (sh.nt == 256 && sh.ipt == 32) RP_GO(WW, RAWF, 256, 32);              \
    else RP_GO(WW, RAWF, 512, 16);
        if (p > 0) { RP_SHAPES(8, false) }
        else if (width == 1) { RP_SHAPES(1, true) }
        else if (width == 2) { RP_SHAPES(2, true) }
        else if (width == 4) { RP_SHAPES(4, true) }
        else { RP_SHAPES(8, true) }
#undef RP_SHAPES
#undef RP_GO
        if ((e = hipGetLastError()) != hipSuccess) return e;
    }
    return hipSuccess;
}

}  // namespace

// Host-side shape of a partitioned insert: slice bits (0 = not eligible).
u32 part_slice_bits(const Spec& S, const BatchDesc& hb, u64 rows, u64 cap) {
    if (!S.inline_keys || S.n_keys != 1 || S.key_types[0].nullable || hb.n_nodes != 0) return 0;
    if (!(S.n_aggs == 1 && S.aggs[0].kind == DBG_AGG_COUNT && S.aggs[0].arg_type < 0 && S.aggs[0].w0 == 1 && S.stride_words == 2))
        return 0;
    const DCol& k = hb.keys[0];
    int ty = k.type;
    bool intlike = (ty >= DBG_INT8 && ty <= DBG_UINT64) || ty == DBG_DATE || ty == DBG_TIMESTAMP;
    if (!intlike || k.layout != LAYOUT_ARROW || ((uintptr_t)k.data % k.width)) return 0;
    // below ~1M rows the sort's fixed cost outweighs the streaming insert's HBM atomics
    if (rows < (1ULL << 20) || cap < (1ULL << 20)) return 0;
    // 4096 slots of 16 B per slice (the kernel is instantiated for this size only; at least two
    // slices)
    if (cap < (2ULL << PART_SB)) return 0;
    return PART_SB;
}

size_t part_temp_bytes(int width, u64 rows, u32 sb, u64 cap) {
    (void)width;
    (void)sb;
    (void)cap;
    return rp_temp_bytes(rows);
}

// sorted: rows u64; bounds: (cap >> sb) + 1 u64; temp: part_temp_bytes.  The keys of the batch
// sorted by their slot's slice, and every slice's first sorted position.  *step names the failing
// step on error.
hipError_t launch_part_sort(hipStream_t s, const BatchDesc& hb, u64 rows, u64 cap, u32 sb, void* temp, size_t temp_bytes,
                            u64* sorted, u64* bounds, const char** step) {
    const int width = (int)hb.keys[0].width;
    if (sb != PART_SB || temp_bytes < rp_temp_bytes(rows) || rows >= (1ULL << 32)) return hipErrorInvalidValue;
    const RadixPlan P = rp_plan(sb, cap);
    if (P.npass < 1 || P.npass > RP_MAXP) return hipErrorInvalidValue;
    hipError_t e = rp_sort(s, width, hb.keys[0].data, rows, P, (u8*)temp, sorted, step);
    if (e != hipSuccess) return e;
    const u64 n_slices = cap >> sb;
    *step = "part_bounds";
    hipLaunchKernelGGL(part_bounds_kernel, dim3((u32)((n_slices + 1 + 255) / 256)), dim3(256), 0, s, sorted, rows, cap - 1, sb,
                       n_slices, bounds);
    return hipGetLastError();
}

// The table stage of a sorted batch: one workgroup per slice, then the overflow merge.
// table_empty: the table holds no group and its initialisation was deferred (part_slice writes
// every slot).
hipError_t launch_part_slices(hipStream_t s, const TableDesc& t, u32 sb, const u64* sorted, const u64* bounds, bool table_empty,
                              const char** step) {
    if (sb != PART_SB) return hipErrorInvalidValue;
    const u64 n_slices = t.cap >> sb;
    hipError_t e;
    *step = "part_slice";
    static const int slice_nt = X_ENV("DBG_X_SLICE_NT") ? atoi(X_ENV("DBG_X_SLICE_NT")) : PART_NT_DEFAULT;
    const size_t sh = (size_t)(12ULL << PART_SB);
#define SLICE_GO(EM, NTT) \
    hipLaunchKernelGGL((part_slice_kernel<PART_SB, EM, NTT>), dim3((u32)n_slices), dim3(NTT), sh, s, sorted, bounds, t)
    if (slice_nt == 1024) {
        if (table_empty) SLICE_GO(true, 1024); else SLICE_GO(false, 1024);
    } else {
        if (table_empty) SLICE_GO(true, 512); else SLICE_GO(false, 512);
    }
#undef SLICE_GO
    if ((e = hipGetLastError()) != hipSuccess) return e;
    *step = "part_fixup";
    hipLaunchKernelGGL(part_fixup_kernel, dim3(512), dim3(256), 0, s, t);
    return hipGetLastError();
}

hipError_t launch_part_insert(hipStream_t s, const BatchDesc& hb, u64 rows, const TableDesc& t, u32 sb, void* temp,
                              size_t temp_bytes, u64* sorted, u64* bounds, bool table_empty, const char** step) {
    hipError_t e = launch_part_sort(s, hb, rows, t.cap, sb, temp, temp_bytes, sorted, bounds, step);
    if (e != hipSuccess) return e;
    return launch_part_slices(s, t, sb, sorted, bounds, table_empty, step);
}

u64 part_direct_status_words(u64 cap, u32 sb) {
    const u64 n = cap >> sb;
    return n + (n + PD_CHUNK - 1) / PD_CHUNK + 4;
}

// The direct stage (part_slice_direct_kernel + part_direct_emit_kernel) of a sorted batch into
// result columns: keys of key_width bytes, u64 counts; totals[0] = groups, or ~0 when the host must
// replay the table path.  status: part_direct_status_words() words.  The table's slots are
// scratch here (left to be initialised, like a reset table).
hipError_t launch_part_direct(hipStream_t s, const TableDesc& t, u32 sb, const u64* sorted, const u64* bounds, u64* status, int key_width,
                              void* out_key, u64* out_cnt, u64 cap_groups, u64* totals) {
    if (sb != PART_SB) return hipErrorInvalidValue;
    const u64 n_slices = t.cap >> sb, n_chunks = (n_slices + PD_CHUNK - 1) / PD_CHUNK;
    hipError_t e = hipMemsetAsync(status + n_slices, 0, (n_chunks + 4) * 8, s);
    if (e != hipSuccess) return e;
    const size_t sh = (size_t)(12ULL << PART_SB);
    hipLaunchKernelGGL((part_slice_direct_kernel<PART_SB, PART_NT_DEFAULT>), dim3((u32)n_slices), dim3(PART_NT_DEFAULT), sh, s, sorted,
                       bounds, n_slices, t.cap, t.slots, status);
    if ((e = hipGetLastError()) != hipSuccess) return e;
#define EMIT_GO(KW)                                                                                                                \
    hipLaunchKernelGGL((part_direct_emit_kernel<KW>), dim3((u32)n_chunks), dim3(1024), 0, s, t.slots, n_slices, status, (u8*)out_key, \
                       out_cnt, cap_groups, totals)
    switch (key_width) {
        case 1: EMIT_GO(1); break;
        case 2: EMIT_GO(2); break;
        case 4: EMIT_GO(4); break;
        case 8: EMIT_GO(8); break;
        default: return hipErrorInvalidValue;
    }
#undef EMIT_GO
    return hipGetLastError();
}
