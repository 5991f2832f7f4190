// sort.hip — ORDER BY <one column> LIMIT k on device: the sort that ends every ClickBench
// GROUP BY query, applied to the aggregate's result columns while they are still in HBM.
//
// Reference: DataBlock::sort (EXP/kernels/sort.rs:79-107) with one sort column and a limit goes
// to arrow's sort_to_indices -> indices_sorted_unstable_by
// (src/common/arrow/src/arrow/compute/sort/common.rs:95-174): NULLs are placed first or last in
// ascending row order; the valid rows are ordered by ord::total_cmp (integers) or
// total_cmp_f32/f64 (floats: IEEE 754 totalOrder on the raw bits, array/ord.rs:36-56), reversed
// for DESC, and cut with select_nth_unstable_by(limit) + sort_unstable_by — ties at equal keys
// come out in an unspecified order there; here they come out in ascending row order, one of the
// orders the reference may produce.
//
// MI355X shape: an MSD radix select over the composite key (null rank 1 bit | order key 64 bits |
// row 32 bits), one 8-bit digit per pass: each pass is one streaming read of the column with an
// LDS histogram per workgroup (HBM-bound, 8 B/row for 64-bit columns), and the host picks the
// digit bucket holding the limit-th row.  Passes stop as soon as that bucket is taken whole, and
// one AND/OR reduction pass finds the key bytes every row shares (the high bytes of a COUNT
// column), whose passes are skipped.  The <= limit selected rows are then compacted and ordered by
// one workgroup's bitonic sort in LDS; inputs of <= 2048 rows go straight to that sort.
#include <cstring>
#include <string>

#include "device.hpp"
#include "sort.hpp"

#define SBLOCK 256
#define SORT_NT 1024

struct SortSel {  // rows whose masked composite key equals (nr_val, ok_val, ix_val) are "in play"
    u32 nr_mask, nr_val;
    u64 ok_mask, ok_val;
    u32 ix_mask, ix_val;
};

// Order key: ascending u64 order == the reference's value order (ASC); DESC flips it.
__device__ __forceinline__ u64 sort_key(const DCol& c, u64 i, bool desc) {
    u64 b = dcol_bits(c, i), k;
    switch (c.type) {
        case DBG_FLOAT64: k = (b >> 63) ? ~b : (b | 0x8000000000000000ULL); break;  // total_cmp_f64
        case DBG_FLOAT32: {
            u32 x = (u32)b;
            k = (x >> 31) ? (u64)(~x) : (u64)(x | 0x80000000u);  // total_cmp_f32
            break;
        }
        case DBG_INT8: case DBG_INT16: case DBG_INT32: case DBG_DATE: case DBG_INT64: case DBG_TIMESTAMP:
            k = (u64)dcol_i64(c, i) ^ 0x8000000000000000ULL;
            break;
        default: k = b;  // unsigned, boolean
    }
    return desc ? ~k : k;
}

// Null rank: 0 sorts before 1.  nulls_first -> NULL rows rank 0; otherwise valid rows rank 0.
__device__ __forceinline__ u32 null_rank(const DCol& c, u64 i, bool nulls_first) {
    return dcol_valid(c, i) == nulls_first ? 1u : 0u;
}

__device__ __forceinline__ void row_key(const DCol& c, u64 i, bool desc, bool nulls_first, u32& nr, u64& ok) {
    nr = null_rank(c, i, nulls_first);
    ok = dcol_valid(c, i) ? sort_key(c, i, desc) : 0ULL;
}

__device__ __forceinline__ bool in_play(const SortSel& s, u32 nr, u64 ok, u32 ix) {
    return (nr & s.nr_mask) == s.nr_val && (ok & s.ok_mask) == s.ok_val && (ix & s.ix_mask) == s.ix_val;
}

// level 0: null rank; 1..8: order-key bytes, most significant first; 9..12: row bytes.
__global__ void __launch_bounds__(SBLOCK) sort_hist_kernel(DCol c, u64 rows, int desc, int nulls_first, SortSel s,
                                                           int level, u32* hist) {
    __shared__ u32 h[256];
    for (u32 t = threadIdx.x; t < 256; t += SBLOCK) h[t] = 0;
    __syncthreads();
    for (u64 i = blockIdx.x * (u64)SBLOCK + threadIdx.x; i < rows; i += (u64)gridDim.x * SBLOCK) {
        u32 nr;
        u64 ok;
        row_key(c, i, desc, nulls_first, nr, ok);
        const u32 ix = (u32)i;
        if (!in_play(s, nr, ok, ix)) continue;
        u32 d;
        if (level == 0) d = nr;
        else if (level <= 8) d = (u32)(ok >> (8 * (8 - level))) & 255u;
        else d = (ix >> (8 * (12 - level))) & 255u;
        atomicAdd(&h[d], 1u);
    }
    __syncthreads();
    for (u32 t = threadIdx.x; t < 256; t += SBLOCK)
        if (h[t]) atomicAdd(&hist[t], h[t]);
}

// Bitwise AND / OR of the order keys of the rows in play: a byte on which they agree is common
// to every row in play (and to every subset of them), so its radix pass can be skipped.
__global__ void __launch_bounds__(SBLOCK) sort_andor_kernel(DCol c, u64 rows, int desc, int nulls_first, SortSel s,
                                                            u64* andor) {
    u64 a = ~0ULL, o = 0ULL;
    for (u64 i = blockIdx.x * (u64)SBLOCK + threadIdx.x; i < rows; i += (u64)gridDim.x * SBLOCK) {
        u32 nr;
        u64 ok;
        row_key(c, i, desc, nulls_first, nr, ok);
        if (!in_play(s, nr, ok, (u32)i)) continue;
        a &= ok;
        o |= ok;
    }
    for (int off = 32; off > 0; off >>= 1) {
        a &= __shfl_xor(a, off);
        o |= __shfl_xor(o, off);
    }
    if ((threadIdx.x & 63) == 0) {
        atomicAnd((unsigned long long*)andor, (unsigned long long)a);
        atomicOr((unsigned long long*)(andor + 1), (unsigned long long)o);
    }
}

// Rows whose masked composite key is <= the threshold: exactly the first `limit` rows.
__global__ void __launch_bounds__(SBLOCK) sort_select_kernel(DCol c, u64 rows, int desc, int nulls_first, SortSel s,
                                                             u64* cand_ok, u64* cand_lo, u32* counter, u32 cap) {
    for (u64 i = blockIdx.x * (u64)SBLOCK + threadIdx.x; i < rows; i += (u64)gridDim.x * SBLOCK) {
        u32 nr;
        u64 ok;
        row_key(c, i, desc, nulls_first, nr, ok);
        const u32 ix = (u32)i;
        const u32 a = nr & s.nr_mask;
        const u64 b = ok & s.ok_mask;
        const u32 x = ix & s.ix_mask;
        const bool le = a != s.nr_val ? a < s.nr_val : (b != s.ok_val ? b < s.ok_val : x <= s.ix_val);
        if (!le) continue;
        u32 p = atomicAdd(counter, 1u);
        if (p < cap) {
            cand_ok[p] = ok;
            cand_lo[p] = ((u64)nr << 32) | ix;
        }
    }
}

// One workgroup: bitonic sort of n <= SORT_CAP (null rank, order key, row) triples in LDS.
__device__ __forceinline__ bool sort_less(u64 ao, u64 al, u64 bo, u64 bl) {
    u32 an = (u32)(al >> 32), bn = (u32)(bl >> 32);
    if (an != bn) return an < bn;
    if (ao != bo) return ao < bo;
    return (u32)al < (u32)bl;
}

__global__ void __launch_bounds__(SORT_NT) sort_small_kernel(const u64* cand_ok, const u64* cand_lo, u32 n, u32 n_out,
                                                            u32* idx_out) {
    __shared__ u64 ko[SORT_CAP], kl[SORT_CAP];
    u32 m = 1;
    while (m < n) m <<= 1;
    for (u32 t = threadIdx.x; t < m; t += SORT_NT) {
        ko[t] = t < n ? cand_ok[t] : ~0ULL;
        kl[t] = t < n ? cand_lo[t] : (3ULL << 32);  // null rank 3: after every real row
    }
    __syncthreads();
    for (u32 size = 2; size <= m; size <<= 1) {
        for (u32 stride = size >> 1; stride > 0; stride >>= 1) {
            for (u32 t = threadIdx.x; t < m; t += SORT_NT) {
                u32 p = t ^ stride;
                if (p > t) {
                    const bool up = (t & size) == 0;
                    const bool sw = up ? sort_less(ko[p], kl[p], ko[t], kl[t]) : sort_less(ko[t], kl[t], ko[p], kl[p]);
                    if (sw) {
                        u64 a = ko[t], b = kl[t];
                        ko[t] = ko[p];
                        kl[t] = kl[p];
                        ko[p] = a;
                        kl[p] = b;
                    }
                }
            }
            __syncthreads();
        }
    }
    for (u32 t = threadIdx.x; t < n_out; t += SORT_NT) idx_out[t] = (u32)kl[t];
}

int sort_limit_run(hipStream_t s, const DCol& c, u64 rows, int asc, int nulls_first, u64 limit, u32* idx_out,
                   u64* n_out, std::string& err) {
    *n_out = 0;
    const u64 need_total = limit < rows ? limit : rows;
    if (need_total == 0) return DBG_OK;
    if (need_total > SORT_CAP) {
        err = "sort limit: at most " + std::to_string(SORT_CAP) + " rows";
        return DBG_ERR_UNSUPPORTED;
    }
    if (rows >= 0xFFFFFFFFULL) {
        err = "sort limit: row indices are u32";
        return DBG_ERR_UNSUPPORTED;
    }
    // one allocation: hist[256] u32 | counter u32 (+pad) | cand_ok | cand_lo | and/or u64 x 2
    char* buf = nullptr;
    const size_t bytes = 256 * 4 + 16 + 2 * (size_t)SORT_CAP * 8 + 16;
    if (hipMalloc((void**)&buf, bytes) != hipSuccess) {
        err = "sort limit: device allocation failed";
        return DBG_ERR_OOM;
    }
    u32* hist = (u32*)buf;
    u32* counter = (u32*)(buf + 1024);
    u64* cand_ok = (u64*)(buf + 1024 + 16);
    u64* cand_lo = cand_ok + SORT_CAP;
    u64* andor = cand_lo + SORT_CAP;
    const int desc = asc ? 0 : 1;
    const bool has_nulls = c.nullable && c.validity != nullptr;
    u64 blocks = (rows + SBLOCK * 8 - 1) / (SBLOCK * 8);
    if (blocks > 4096) blocks = 4096;
    if (blocks < 1) blocks = 1;

    SortSel sel;
    memset(&sel, 0, sizeof(sel));
    int level = 0;
    if (!has_nulls) {  // every row has the valid rank
        sel.nr_mask = 1;
        sel.nr_val = nulls_first ? 1u : 0u;
        level = 1;
    }
    int rc = DBG_OK;
    u64 need = need_total;
    u32 h[256];
    u64 common = 0, common_val = 0;  // order-key bits shared by every row in play
    bool have_common = false;
    if (rows <= SORT_CAP) level = 13;  // every row is a candidate: no select passes
    for (; level <= 12; ++level) {
        if (level >= 1 && level <= 8 && !have_common) {
            const u64 init[2] = {~0ULL, 0ULL};
            hipMemcpyAsync(andor, init, 16, hipMemcpyHostToDevice, s);
            hipLaunchKernelGGL(sort_andor_kernel, dim3((u32)blocks), dim3(SBLOCK), 0, s, c, rows, desc, nulls_first, sel, andor);
            u64 ao[2];
            hipMemcpyAsync(ao, andor, 16, hipMemcpyDeviceToHost, s);
            if (hipStreamSynchronize(s) != hipSuccess) {
                err = "sort limit: and/or pass failed";
                rc = DBG_ERR_DEVICE;
                break;
            }
            common = ~(ao[0] ^ ao[1]);
            common_val = ao[0];
            have_common = true;
        }
        if (level >= 1 && level <= 8) {
            const int sh = 8 * (8 - level);
            if (((common >> sh) & 255ULL) == 255ULL) {  // one bucket holds every row in play
                sel.ok_mask |= 255ULL << sh;
                sel.ok_val |= common_val & (255ULL << sh);
                continue;
            }
        }
        hipMemsetAsync(hist, 0, 1024, s);
        hipLaunchKernelGGL(sort_hist_kernel, dim3((u32)blocks), dim3(SBLOCK), 0, s, c, rows, desc, nulls_first, sel, level, hist);
        hipMemcpyAsync(h, hist, sizeof(h), hipMemcpyDeviceToHost, s);
        hipError_t e = hipStreamSynchronize(s);
        if (e != hipSuccess) {
            err = std::string("sort limit: ") + hipGetErrorString(e);
            rc = DBG_ERR_DEVICE;
            break;
        }
        u64 cum = 0;
        u32 d = 0;
        for (; d < 256; ++d) {
            if (cum + h[d] >= need) break;
            cum += h[d];
        }
        if (d == 256) {  // fewer rows in play than needed: cannot happen for a consistent column
            err = "sort limit: inconsistent histogram";
            rc = DBG_ERR_INTERNAL;
            break;
        }
        if (level == 0) {
            sel.nr_mask = 1;
            sel.nr_val = d;
        } else if (level <= 8) {
            const int sh = 8 * (8 - level);
            sel.ok_mask |= 255ULL << sh;
            sel.ok_val |= (u64)d << sh;
        } else {
            const int sh = 8 * (12 - level);
            sel.ix_mask |= 255u << sh;
            sel.ix_val |= d << sh;
        }
        need -= cum;
        if (h[d] == need) break;  // the whole bucket is in: the threshold is this prefix
    }
    if (rc == DBG_OK) {
        hipMemsetAsync(counter, 0, 4, s);
        hipLaunchKernelGGL(sort_select_kernel, dim3((u32)blocks), dim3(SBLOCK), 0, s, c, rows, desc, nulls_first, sel,
                           cand_ok, cand_lo, counter, (u32)SORT_CAP);
        const u64 n_cand = rows <= SORT_CAP ? rows : need_total;
        hipLaunchKernelGGL(sort_small_kernel, dim3(1), dim3(SORT_NT), 0, s, cand_ok, cand_lo, (u32)n_cand, (u32)need_total, idx_out);
        u32 got = 0;
        hipMemcpyAsync(&got, counter, 4, hipMemcpyDeviceToHost, s);
        hipError_t e = hipStreamSynchronize(s);
        if (e != hipSuccess) {
            err = std::string("sort limit: ") + hipGetErrorString(e);
            rc = DBG_ERR_DEVICE;
        } else if (got != n_cand) {
            err = "sort limit: selected " + std::to_string(got) + " rows, expected " + std::to_string(n_cand);
            rc = DBG_ERR_INTERNAL;
        } else {
            *n_out = need_total;
        }
    }
    hipFree(buf);
    return rc;
}
