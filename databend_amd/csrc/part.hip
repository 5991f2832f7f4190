// part.hip — radix-partitioned insert for high-cardinality single-key COUNT(*) batches.
//
// The streaming insert (agg_insert_fast) turns every row of a high-cardinality batch into one
// random device-scope atomic on the HBM table (ClickBench Q17 shape: 1e9 rows, 1.3e8 groups, a
// 8.6 GB table): 1e9 random 64-B memory-side read-modify-writes.  Here the same batch is
// reordered first so that the table is touched slice by slice:
//
//   1. m = slot_mix(key) for every row (slot_mix is a bijection of u64), radix-partitioned on
//      the slot bits above the slice size — rocPRIM's onesweep radix sort over bits
//      [slice_bits, log2 cap), input read through a transform iterator (no staging pass);
//   2. part_bounds: the first sorted position of every slice (one binary search per slice);
//   3. part_slice: one workgroup per table slice: slice HBM -> LDS (64 KB), every row of the
//      slice probes and counts in LDS (same linear probing as g_find, so the table stays a valid
//      HBM table for every other kernel), LDS -> HBM.  A probe that would leave the slice (its
//      run continues in the next slice, owned by another workgroup) becomes an overflow record
//      [key][1] that agg_retry merges after the launch — the deferred-overflow protocol of the
//      streaming insert.
//
// This is the reference's own answer to the same problem — AggregateHashTable radix-partitions
// its payload (EAGG/partitioned_payload.rs:100-143) so the final merge works partition by
// partition on cache-sized tables (AGG/transform_aggregate_final.rs:71-156) — applied to the
// 64 KB LDS of a CDNA4 workgroup instead of a CPU core's cache.
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/iterator/transform_iterator.hpp>

#include <cstdio>

#include "agg.hpp"

#define PART_NT 1024
#define PART_SB 12  // slice = 4096 slots x 16 B = 64 KB of LDS
#define PART_PROBE_CAP 64
#define PART_OVF_LDS 512  // overflow keys gathered per workgroup before one device atomic
#define RB 4  // sorted keys per lane per batch in the slice kernel

namespace {

template <typename U>
struct MixOf {
    __host__ __device__ u64 operator()(U v) const { return slot_mix((u64)v); }
};

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
template <int SB>
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
    // slice -> LDS (16-byte loads; the slot stride is 2 words)
    const v2u64 __attribute__((address_space(1)))* gsl = (const v2u64 __attribute__((address_space(1)))*)(t.slots + s0 * 2);
    v2u64* lsl = (v2u64*)lds;
    v2u64 sv[PER];
#pragma unroll
    for (int k = 0; k < PER; ++k) sv[k] = gsl[threadIdx.x + k * PART_NT];
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
    for (int k = 0; k < PER; ++k) lsl[threadIdx.x + k * PART_NT] = sv[k];
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
            wptr<AS_LDS> e = asp<AS_LDS>(lds + (u64)ls * 2);
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
            at_add<AS_LDS>(asp<AS_LDS>(lds + (u64)ls * 2 + 1), 1ULL);
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
    for (int k = 0; k < PER; ++k) osl[threadIdx.x + k * PART_NT] = lsl[threadIdx.x + k * PART_NT];
    if (threadIdx.x == 0 && lclaims) atomicAdd((unsigned long long*)(t.counters + CNT_CLAIMS), (unsigned long long)lclaims);
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

template <typename U>
hipError_t sort_t(void* temp, size_t& temp_bytes, const void* keys, u64* out, u64 rows, u32 b0, u32 b1, hipStream_t s) {
    auto it = rocprim::make_transform_iterator((const U*)keys, MixOf<U>());
    hipError_t e = rocprim::radix_sort_keys(temp, temp_bytes, it, out, (size_t)rows, b0, b1, s);
    return e;
}

hipError_t sort_any(int width, void* temp, size_t& temp_bytes, const void* keys, u64* out, u64 rows, u32 b0, u32 b1,
                    hipStream_t s) {
    switch (width) {
        case 1: return sort_t<uint8_t>(temp, temp_bytes, keys, out, rows, b0, b1, s);
        case 2: return sort_t<uint16_t>(temp, temp_bytes, keys, out, rows, b0, b1, s);
        case 4: return sort_t<uint32_t>(temp, temp_bytes, keys, out, rows, b0, b1, s);
        default: return sort_t<u64>(temp, temp_bytes, keys, out, rows, b0, b1, s);
    }
}

u32 log2u(u64 x) { return 63 - __builtin_clzll(x); }

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
    size_t bytes = 0;
    if (sort_any(width, nullptr, bytes, nullptr, nullptr, rows, sb, log2u(cap), 0) != hipSuccess) return 0;
    return bytes;
}

// sorted: rows u64; bounds: (cap >> sb) + 1 u64; temp: part_temp_bytes.  *step names the
// failing step on error.
hipError_t launch_part_insert(hipStream_t s, const BatchDesc& hb, u64 rows, const TableDesc& t, u32 sb, void* temp,
                              size_t temp_bytes, u64* sorted, u64* bounds, const char** step) {
    const int width = (int)hb.keys[0].width;
    const u32 cb = log2u(t.cap);
    // rocPRIM's return code is authoritative: it makes calls whose failure it tolerates (HIP's
    // last-error slot then holds a stale code), so the slot is not consulted for the sort
    *step = "rocprim radix_sort_keys";
    (void)hipGetLastError();  // rocPRIM reads the last-error slot after its launches: start it clean
    hipError_t e = sort_any(width, temp, temp_bytes, hb.keys[0].data, sorted, rows, sb, cb, s);
    if (e != hipSuccess) return e;
    (void)hipGetLastError();
    const u64 n_slices = t.cap >> sb;
    *step = "part_bounds";
    hipLaunchKernelGGL(part_bounds_kernel, dim3((u32)((n_slices + 1 + 255) / 256)), dim3(256), 0, s, sorted, rows, t.cap - 1, sb,
                       n_slices, bounds);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    *step = "part_slice";
    if (sb != PART_SB) return hipErrorInvalidValue;
    hipLaunchKernelGGL(part_slice_kernel<PART_SB>, dim3((u32)n_slices), dim3(PART_NT), (size_t)(16ULL << PART_SB), s, sorted, bounds,
                       t);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    *step = "part_fixup";
    hipLaunchKernelGGL(part_fixup_kernel, dim3(512), dim3(256), 0, s, t);
    return hipGetLastError();
}
