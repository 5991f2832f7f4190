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
#include <vector>

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

// ------------------------------------------------------------------------------------------
// ORDER BY <c1 [ASC|DESC] [NULLS FIRST|LAST], c2 ...> LIMIT k over numbers, Decimal128 and
// String columns (DataBlock::sort with several descriptions -> arrow lexsort_to_indices, EXP/
// kernels/sort.rs:79-107; values by ord of each column: integers, IEEE totalOrder floats, i128
// decimals, byte-wise strings).
//
// Each row's sort key is one order-preserving byte string, read 8 bytes (one u64 word, big-endian)
// at a time straight from the columns, never materialised for the whole input: per column a null
// marker byte when the column is nullable (the rank nulls_first asks for; DESC does not move
// NULLs), then the value — 8 bytes of the order key for numbers, 16 for Decimal128, and for a
// String its bytes in groups of 8, each followed by a marker byte (9 = more groups follow, else the
// group's byte count), which makes the encoding prefix-free and byte-wise comparison equal to
// (bytes, length) order; DESC inverts the value bytes.  A NULL's value bytes are 0.  The radix
// select of the single-column path then runs over (key words..., row index): per word an AND/OR
// pass finds the bytes every row in play shares, one histogram pass per remaining byte picks the
// bucket of the limit-th row, and words already decided are matched whole.  The <= limit rows
// selected are ordered by one workgroup's bitonic sort over their key words (gathered into a
// scratch buffer), ties by row index.
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ u32 mkey_col_len(const MKeyDesc& K, int c, u64 row) {
    const DCol& col = K.cols[c];
    u32 n = col.nullable ? 1u : 0u;
    if (col.type == DBG_STRING) {
        const u64 len = dcol_str(col, row).len;
        return n + 9u * (u32)(len ? (len + 7) / 8 : 1);
    }
    return n + (col.type == DBG_DECIMAL128 ? 16u : 8u);
}

// byte q of column c's encoding (q < mkey_col_len)
__device__ __forceinline__ u32 mkey_col_byte(const MKeyDesc& K, int c, u64 row, u32 q) {
    const DCol& col = K.cols[c];
    const bool valid = dcol_valid(col, row);
    if (col.nullable) {
        if (q == 0) return valid == (K.nulls_first[c] != 0) ? 1u : 0u;
        --q;
    }
    if (!valid) return 0u;
    const u32 inv = K.desc[c] ? 0xFFu : 0u;
    if (col.type == DBG_STRING) {
        const StrRef s = dcol_str(col, row);
        const u64 g = q / 9, r = q % 9;
        if (r < 8) return (g * 8 + r < s.len ? (u32)gld<u8>(s.p + g * 8 + r) : 0u) ^ inv;
        const u64 groups = s.len ? (s.len + 7) / 8 : 1;
        return (g + 1 < groups ? 9u : (u32)(s.len - g * 8)) ^ inv;
    }
    if (col.type == DBG_DECIMAL128) {
        const u64 hi = dcol_hi(col, row) ^ 0x8000000000000000ULL, lo = dcol_bits(col, row);
        const u64 w = q < 8 ? hi : lo;
        return ((u32)(w >> (8 * (7 - (q & 7)))) & 0xFFu) ^ inv;
    }
    return (u32)(sort_key(col, row, K.desc[c] != 0) >> (8 * (7 - q))) & 0xFFu;  // sort_key applies DESC
}

// word w (bytes [8w, 8w + 8), big-endian) of the row's key; 0 past its end
__device__ u64 mkey_word(const MKeyDesc& K, u64 row, u32 w) {
    const u32 lo = 8 * w, hi = lo + 8;
    u64 out = 0;
    u32 pos = 0;
    for (int c = 0; c < K.n && pos < hi; ++c) {
        const u32 len = mkey_col_len(K, c, row);
        if (pos + len > lo) {
            const u32 a = pos > lo ? pos : lo, b = pos + len < hi ? pos + len : hi;
            for (u32 p = a; p < b; ++p) out |= (u64)mkey_col_byte(K, c, row, p - pos) << (8 * (7 - (p - lo)));
        }
        pos += len;
    }
    return out;
}

struct MSel {  // rows whose words [0, nw) equal prefix and whose masked word nw / row match
    const u64* prefix;
    u32 nw;
    u64 mask, val;  // on word nw (nw < W)
    u32 ix_mask, ix_val;
};

// -1 / 0 / 1: the row's (prefix words, masked word, masked row) against the selection's
__device__ __forceinline__ int msel_cmp(const MKeyDesc& K, const MSel& s, u32 W, u64 row) {
    for (u32 j = 0; j < s.nw; ++j) {
        const u64 k = mkey_word(K, row, j), p = s.prefix[j];
        if (k != p) return k < p ? -1 : 1;
    }
    if (s.nw < W) {
        const u64 k = mkey_word(K, row, s.nw) & s.mask;
        if (k != s.val) return k < s.val ? -1 : 1;
    }
    const u32 x = (u32)row & s.ix_mask;
    return x == s.ix_val ? 0 : (x < s.ix_val ? -1 : 1);
}

__global__ void __launch_bounds__(SBLOCK) mkey_maxlen_kernel(MKeyDesc K, u64 rows, u64* maxlen) {
    u64 m = 0;
    for (u64 i = blockIdx.x * (u64)SBLOCK + threadIdx.x; i < rows; i += (u64)gridDim.x * SBLOCK) {
        u64 t = 0;
        for (int c = 0; c < K.n; ++c) t += mkey_col_len(K, c, i);
        m = t > m ? t : m;
    }
    for (int off = 32; off > 0; off >>= 1) {
        const u64 o = __shfl_xor(m, off);
        m = o > m ? o : m;
    }
    if ((threadIdx.x & 63) == 0) atomicMax((unsigned long long*)maxlen, (unsigned long long)m);
}

__global__ void __launch_bounds__(SBLOCK) mkey_andor_kernel(MKeyDesc K, u64 rows, u32 W, MSel s, u64* andor) {
    u64 a = ~0ULL, o = 0ULL;
    for (u64 i = blockIdx.x * (u64)SBLOCK + threadIdx.x; i < rows; i += (u64)gridDim.x * SBLOCK) {
        if (msel_cmp(K, s, W, i) != 0) continue;
        const u64 k = mkey_word(K, i, s.nw);
        a &= k;
        o |= k;
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

// digit `byte` (0 = most significant) of word s.nw, or of the row index once every word is decided
__global__ void __launch_bounds__(SBLOCK) mkey_hist_kernel(MKeyDesc K, u64 rows, u32 W, MSel s, int byte, u32* hist) {
    __shared__ u32 h[256];
    for (u32 t = threadIdx.x; t < 256; t += SBLOCK) h[t] = 0;
    __syncthreads();
    for (u64 i = blockIdx.x * (u64)SBLOCK + threadIdx.x; i < rows; i += (u64)gridDim.x * SBLOCK) {
        if (msel_cmp(K, s, W, i) != 0) continue;
        const u32 d = s.nw < W ? (u32)(mkey_word(K, i, s.nw) >> (8 * (7 - byte))) & 255u
                               : ((u32)i >> (8 * (3 - byte))) & 255u;
        atomicAdd(&h[d], 1u);
    }
    __syncthreads();
    for (u32 t = threadIdx.x; t < 256; t += SBLOCK)
        if (h[t]) atomicAdd(&hist[t], h[t]);
}

__global__ void __launch_bounds__(SBLOCK) mkey_select_kernel(MKeyDesc K, u64 rows, u32 W, MSel s, u32* cand, u32* counter,
                                                             u32 cap) {
    for (u64 i = blockIdx.x * (u64)SBLOCK + threadIdx.x; i < rows; i += (u64)gridDim.x * SBLOCK) {
        if (msel_cmp(K, s, W, i) > 0) continue;
        const u32 p = atomicAdd(counter, 1u);
        if (p < cap) cand[p] = (u32)i;
    }
}

__global__ void __launch_bounds__(SBLOCK) mkey_gather_kernel(MKeyDesc K, const u32* cand, u32 n, u32 W, u64* words) {
    for (u64 t = blockIdx.x * (u64)SBLOCK + threadIdx.x; t < (u64)n * W; t += (u64)gridDim.x * SBLOCK)
        words[t] = mkey_word(K, cand[t / W], (u32)(t % W));
}

__device__ __forceinline__ bool mkey_less(const u64* words, const u32* cand, u32 W, u32 a, u32 b) {
    const u64* x = words + (u64)a * W;
    const u64* y = words + (u64)b * W;
    for (u32 w = 0; w < W; ++w)
        if (x[w] != y[w]) return x[w] < y[w];
    return cand[a] < cand[b];
}

// one workgroup: bitonic sort of the candidate positions (n <= SORT_CAP) by their key words
__global__ void __launch_bounds__(SORT_NT) mkey_sort_kernel(const u64* words, const u32* cand, u32 n, u32 W, u32* idx_out) {
    __shared__ u32 pos[SORT_CAP];
    u32 m = 1;
    while (m < n) m <<= 1;
    for (u32 t = threadIdx.x; t < m; t += SORT_NT) pos[t] = t < n ? t : 0xFFFFFFFFu;
    __syncthreads();
    for (u32 size = 2; size <= m; size <<= 1) {
        for (u32 stride = size >> 1; stride > 0; stride >>= 1) {
            for (u32 t = threadIdx.x; t < m; t += SORT_NT) {
                const u32 p = t ^ stride;
                if (p > t) {
                    const u32 a = pos[t], b = pos[p];
                    // padding (0xFFFFFFFF) sorts after every candidate
                    const bool b_lt_a = b != 0xFFFFFFFFu && (a == 0xFFFFFFFFu || mkey_less(words, cand, W, b, a));
                    const bool a_lt_b = a != 0xFFFFFFFFu && (b == 0xFFFFFFFFu || mkey_less(words, cand, W, a, b));
                    if ((t & size) == 0 ? b_lt_a : a_lt_b) {
                        pos[t] = b;
                        pos[p] = a;
                    }
                }
            }
            __syncthreads();
        }
    }
    for (u32 t = threadIdx.x; t < n; t += SORT_NT) idx_out[t] = cand[pos[t]];
}

int sort_multi_limit_run(hipStream_t s, const MKeyDesc& K, u64 rows, u64 limit, u32* idx_out, u64* n_out, std::string& err) {
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
    u64 blocks = (rows + SBLOCK * 8 - 1) / (SBLOCK * 8);
    if (blocks > 4096) blocks = 4096;
    if (blocks < 1) blocks = 1;
    // scratch: hist[256] u32 | counter | maxlen, and/or u64 x 2 | cand u32 x SORT_CAP; prefix and
    // candidate words allocated once W is known
    char* buf = nullptr;
    const size_t head = 1024 + 16 + 32 + (size_t)SORT_CAP * 4;
    if (hipMalloc((void**)&buf, head) != hipSuccess) {
        err = "sort limit: device allocation failed";
        return DBG_ERR_OOM;
    }
    u32* hist = (u32*)buf;
    u32* counter = (u32*)(buf + 1024);
    u64* maxlen = (u64*)(buf + 1024 + 16);
    u64* andor = maxlen + 2;
    u32* cand = (u32*)(buf + 1024 + 16 + 32);
    u64* pref = nullptr;
    u64* words = nullptr;
    int rc = DBG_OK;
    u32 W = 0;
    {
        hipMemsetAsync(maxlen, 0, 8, s);
        hipLaunchKernelGGL(mkey_maxlen_kernel, dim3((u32)blocks), dim3(SBLOCK), 0, s, K, rows, maxlen);
        u64 ml = 0;
        hipMemcpyAsync(&ml, maxlen, 8, hipMemcpyDeviceToHost, s);
        if (hipStreamSynchronize(s) != hipSuccess) {
            err = "sort limit: key length pass failed";
            rc = DBG_ERR_DEVICE;
        }
        W = (u32)((ml + 7) / 8);
        const u64 n_max = rows <= SORT_CAP ? rows : need_total;
        if (rc == DBG_OK && (hipMalloc((void**)&pref, (size_t)(W + 1) * 8) != hipSuccess ||
                             hipMalloc((void**)&words, (size_t)n_max * (W ? W : 1) * 8) != hipSuccess)) {
            err = "sort limit: device allocation failed";
            rc = DBG_ERR_OOM;
        }
    }
    MSel sel;
    memset(&sel, 0, sizeof(sel));
    sel.prefix = pref;
    std::vector<u64> hpref;
    hpref.reserve(W + 1);  // stable addresses: the prefix words are copied from it asynchronously
    u64 need = need_total;
    bool done = rows <= SORT_CAP;  // every row is a candidate
    for (u32 w = 0; rc == DBG_OK && !done && w <= W; ++w) {
        sel.nw = w;
        sel.mask = sel.val = 0;
        u64 common = 0, common_val = 0;
        if (w < W) {
            const u64 init[2] = {~0ULL, 0ULL};
            hipMemcpyAsync(andor, init, 16, hipMemcpyHostToDevice, s);
            hipLaunchKernelGGL(mkey_andor_kernel, dim3((u32)blocks), dim3(SBLOCK), 0, s, K, rows, W, sel, andor);
            u64 ao[2];
            hipMemcpyAsync(ao, andor, 16, hipMemcpyDeviceToHost, s);
            if (hipStreamSynchronize(s) != hipSuccess) {
                err = "sort limit: and/or pass failed";
                rc = DBG_ERR_DEVICE;
                break;
            }
            common = ~(ao[0] ^ ao[1]);
            common_val = ao[0];
        }
        const int nbytes = w < W ? 8 : 4;
        for (int b = 0; b < nbytes; ++b) {
            if (w < W) {
                const int sh = 8 * (7 - b);
                if (((common >> sh) & 255ULL) == 255ULL) {  // one bucket holds every row in play
                    sel.mask |= 255ULL << sh;
                    sel.val |= common_val & (255ULL << sh);
                    continue;
                }
            }
            hipMemsetAsync(hist, 0, 1024, s);
            hipLaunchKernelGGL(mkey_hist_kernel, dim3((u32)blocks), dim3(SBLOCK), 0, s, K, rows, W, sel, b, hist);
            u32 h[256];
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
            if (d == 256) {
                err = "sort limit: inconsistent histogram";
                rc = DBG_ERR_INTERNAL;
                break;
            }
            if (w < W) {
                const int sh = 8 * (7 - b);
                sel.mask |= 255ULL << sh;
                sel.val |= (u64)d << sh;
            } else {
                const int sh = 8 * (3 - b);
                sel.ix_mask |= 255u << sh;
                sel.ix_val |= d << sh;
            }
            need -= cum;
            if (h[d] == need) {  // the whole bucket is in: the threshold is this prefix
                done = true;
                break;
            }
        }
        if (rc != DBG_OK || done) break;
        if (w < W) {  // word w decided whole: it joins the matched prefix
            hpref.push_back(sel.val);
            hipMemcpyAsync(pref + w, &hpref[w], 8, hipMemcpyHostToDevice, s);
        }
    }
    if (rc == DBG_OK && !done && rows > SORT_CAP) {
        err = "sort limit: selection did not converge";
        rc = DBG_ERR_INTERNAL;
    }
    if (rc == DBG_OK) {
        if (rows <= SORT_CAP) {  // no select passes: every row
            sel.nw = 0;
            sel.mask = sel.val = 0;
            sel.ix_mask = 0;
            sel.ix_val = 0;
        }
        hipMemsetAsync(counter, 0, 4, s);
        hipLaunchKernelGGL(mkey_select_kernel, dim3((u32)blocks), dim3(SBLOCK), 0, s, K, rows, W, sel, cand, counter, (u32)SORT_CAP);
        const u64 n_cand = rows <= SORT_CAP ? rows : need_total;
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
            if (W) {
                u64 gb = ((u64)got * W + SBLOCK - 1) / SBLOCK;
                hipLaunchKernelGGL(mkey_gather_kernel, dim3((u32)(gb > 4096 ? 4096 : gb)), dim3(SBLOCK), 0, s, K, cand, got, W, words);
            }
            // the n_cand candidates sorted; the first need_total written
            u32* sorted = idx_out;
            u32* tmp = nullptr;
            if (n_cand > need_total) {
                if (hipMalloc((void**)&tmp, n_cand * 4) != hipSuccess) {
                    err = "sort limit: device allocation failed";
                    rc = DBG_ERR_OOM;
                }
                sorted = tmp;
            }
            if (rc == DBG_OK) {
                hipLaunchKernelGGL(mkey_sort_kernel, dim3(1), dim3(SORT_NT), 0, s, words, cand, (u32)n_cand, W, sorted);
                if (tmp) hipMemcpyAsync(idx_out, tmp, need_total * 4, hipMemcpyDeviceToDevice, s);
                e = hipStreamSynchronize(s);
                if (e != hipSuccess) {
                    err = std::string("sort limit: ") + hipGetErrorString(e);
                    rc = DBG_ERR_DEVICE;
                } else {
                    *n_out = need_total;
                }
            }
            if (tmp) hipFree(tmp);
        }
    }
    if (words) hipFree(words);
    if (pref) hipFree(pref);
    hipFree(buf);
    return rc;
}
