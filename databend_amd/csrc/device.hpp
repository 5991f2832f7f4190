// device.hpp — device-side building blocks of the gfx950 GROUP BY path.
//
// Shared by agg.hip / filter.hip (device) and abi.hip (host, to fill the descriptors).
//  * DCol: a column as the kernels see it — Databend's arrow layout (EXP/values.rs:157-176) or a
//    strided view into a partial-state record buffer.
//  * the group-hash family of EAGG/group_hash.rs:39-265, bit-exact (partition routing depends on it)
//  * key equality with row_match_columns semantics (EAGG/payload_row.rs:169-528)
//  * predicate programs with SQL three-valued logic (EXP/filter/selector.rs)
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/dbgpu_agg.h"

#define DBG_MAX_KEYS 8
#define DBG_MAX_AGGS 32
#define DBG_MAX_FCOLS 8
#define DBG_MAX_NODES 24
#define DBG_MAX_WORDS 96  // state words per slot

typedef uint64_t u64;
typedef int64_t i64;
typedef uint32_t u32;
typedef uint8_t u8;
typedef uint16_t u16;

// ------------------------------------------------------------------------------------------
// Column descriptor
// ------------------------------------------------------------------------------------------
enum { LAYOUT_ARROW = 0, LAYOUT_RECORD = 1 };

struct DCol {
    int32_t type;      // dbg_type
    uint8_t precision, scale, nullable, layout;
    uint32_t width;    // value bytes (0 for strings)
    uint32_t stride;   // bytes between rows (LAYOUT_RECORD); == width for arrow fixed-width
    const u8* data;    // values / string bytes / record base + column offset
    const u64* offsets;   // arrow strings
    const u8* validity;   // arrow: bitmap; record: byte at row*stride (relative to record base)
    u64 validity_offset;  // arrow: bit offset; record: unused
    u64 data_offset;      // arrow booleans: bit offset
    const u8* strings;    // record layout: string blob base (key part holds (offset,len) u64 pairs)
};

__host__ __device__ inline uint32_t type_width(int t) {
    switch (t) {
        case DBG_INT8: case DBG_UINT8: case DBG_BOOLEAN: return 1;
        case DBG_INT16: case DBG_UINT16: return 2;
        case DBG_INT32: case DBG_UINT32: case DBG_FLOAT32: case DBG_DATE: return 4;
        case DBG_INT64: case DBG_UINT64: case DBG_FLOAT64: case DBG_TIMESTAMP: return 8;
        case DBG_DECIMAL128: return 16;
        default: return 0;
    }
}

// Loads of column data through a descriptor: the pointers come out of device memory, so the
// compiler cannot infer their address space and would emit flat loads (which also count against
// lgkmcnt and retire out of order, serialising LDS work behind them).  Column buffers are always
// global memory (device or mapped host), so read them through address-space-1 views.
template <typename V>
__device__ __forceinline__ V gld(const void* p) {
    return *(const V __attribute__((address_space(1)))*)p;
}

__device__ __forceinline__ bool dcol_valid(const DCol& c, u64 i) {
    if (!c.nullable) return true;
    if (c.layout == LAYOUT_RECORD) return gld<u8>(c.validity + i * c.stride) != 0;
    if (c.validity == nullptr) return true;
    u64 b = c.validity_offset + i;
    return (gld<u8>(c.validity + (b >> 3)) >> (b & 7)) & 1;
}

// Raw value bits of a fixed-width cell, zero-extended to 64 bits (Decimal128: low word).
__device__ __forceinline__ u64 dcol_bits(const DCol& c, u64 i) {
    if (c.type == DBG_BOOLEAN) {
        if (c.layout == LAYOUT_RECORD) return gld<u8>(c.data + i * c.stride) != 0;
        u64 b = c.data_offset + i;
        return (gld<u8>(c.data + (b >> 3)) >> (b & 7)) & 1;
    }
    const u8* p = c.data + i * (u64)c.stride;
    switch (c.width) {
        case 1: return gld<u8>(p);
        case 2: return gld<uint16_t>(p);
        case 4: return gld<uint32_t>(p);
        default: return gld<u64>(p);
    }
}
__device__ __forceinline__ u64 dcol_hi(const DCol& c, u64 i) {  // Decimal128 high word
    return gld<u64>(c.data + i * (u64)c.stride + 8);
}

struct StrRef {
    const u8* p;
    u64 len;
};
__device__ __forceinline__ StrRef dcol_str(const DCol& c, u64 i) {
    if (c.layout == LAYOUT_RECORD) {
        const u8* pr = c.data + i * (u64)c.stride;
        return StrRef{c.strings + gld<u64>(pr), gld<u64>(pr + 8)};
    }
    u64 a = gld<u64>(c.offsets + i), b = gld<u64>(c.offsets + i + 1);
    return StrRef{c.data + a, b - a};
}

// Sign-/zero-extended integer value of a number column (for SUM/MIN/MAX/filters).
__device__ __forceinline__ i64 dcol_i64(const DCol& c, u64 i) {
    u64 b = dcol_bits(c, i);
    switch (c.type) {
        case DBG_INT8: return (i64)(int8_t)b;
        case DBG_INT16: return (i64)(int16_t)b;
        case DBG_INT32: case DBG_DATE: return (i64)(int32_t)b;
        default: return (i64)b;
    }
}
__device__ __forceinline__ double dcol_f64(const DCol& c, u64 i) {
    u64 b = dcol_bits(c, i);
    if (c.type == DBG_FLOAT32) return (double)__uint_as_float((u32)b);
    return __longlong_as_double((long long)b);
}

// ------------------------------------------------------------------------------------------
// Group hash — EAGG/group_hash.rs
// ------------------------------------------------------------------------------------------
#define NULL_HASH_VAL 0xd1cefa08eb382d69ULL  // group_hash.rs:39

__host__ __device__ __forceinline__ u64 hash_prim(u64 x) {  // group_hash.rs:194-218
    x ^= x >> 32;
    x *= 0xd6e8feb86659fd93ULL;
    x ^= x >> 32;
    x *= 0xd6e8feb86659fd93ULL;
    x ^= x >> 32;
    return x;
}

__device__ __forceinline__ u64 load_u64_unaligned(const u8* p) {
    // two aligned 8-byte loads funnelled together (the second only when the bytes straddle)
    uintptr_t a = (uintptr_t)p;
    u32 off = (u32)(a & 7);
    const u8* base = (const u8*)(a & ~(uintptr_t)7);
    u64 w0 = gld<u64>(base);
    if (off == 0) return w0;
    u64 w1 = gld<u64>(base + 8);
    return (w0 >> (8 * off)) | (w1 << (64 - 8 * off));
}

// The first r (1..8) bytes at p as a little-endian word (upper bytes unspecified): aligned loads
// only, and only of words that hold at least one of the r bytes (so never past the buffer's page).
__device__ __forceinline__ u64 load_partial(const u8* p, u64 r) {
    uintptr_t a = (uintptr_t)p;
    u32 off = (u32)(a & 7);
    const u8* base = (const u8*)(a & ~(uintptr_t)7);
    u64 w = gld<u64>(base) >> (8 * off);
    if (off + r > 8) w |= gld<u64>(base + 8) << (64 - 8 * off);
    return w;
}

// impl AggHash for [u8] (group_hash.rs:161-192)
__device__ __forceinline__ u64 hash_bytes(const u8* p, u64 len) {
    const u64 M = 0xc6a4a7935bd1e995ULL, R = 47;
    u64 h = 0xe17a1465ULL ^ (len * M);
    u64 nb = len >> 3;
    for (u64 i = 0; i < nb; ++i) {
        u64 k = load_u64_unaligned(p + i * 8);
        k *= M;
        k ^= k >> R;
        k *= M;
        h ^= k;
        h *= M;
    }
    u64 tl = len & 7;
    // tail: h ^= b[i] << 8 * (tl - 1 - i), i.e. the tail bytes big-endian
    if (tl) h ^= __builtin_bswap64(load_partial(p + nb * 8, tl)) >> (8 * (8 - tl));
    h ^= h >> R;
    h *= M;
    h ^= h >> R;
    return h;
}
// Decimal128: hash of i128::to_le_bytes — two full 8-byte blocks, no tail.
__device__ __forceinline__ u64 hash_i128(u64 lo, u64 hi) {
    const u64 M = 0xc6a4a7935bd1e995ULL, R = 47;
    u64 h = 0xe17a1465ULL ^ (16ULL * M);
    u64 k = lo * M;
    k ^= k >> R;
    k *= M;
    h ^= k;
    h *= M;
    k = hi * M;
    k ^= k >> R;
    k *= M;
    h ^= k;
    h *= M;
    h ^= h >> R;
    h *= M;
    h ^= h >> R;
    return h;
}

// Canonical bits of a float key: NaN -> f32::NAN / f64::NAN (group_hash.rs:238-258).
__device__ __forceinline__ u64 canon_float_bits(int type, u64 b) {
    if (type == DBG_FLOAT32) {
        u32 x = (u32)b;
        if ((x & 0x7f800000u) == 0x7f800000u && (x & 0x007fffffu)) return 0x7fc00000u;
        return x;
    }
    if ((b & 0x7ff0000000000000ULL) == 0x7ff0000000000000ULL && (b & 0x000fffffffffffffULL)) return 0x7ff8000000000000ULL;
    return b;
}

// AggHash of one non-null cell.
__device__ __forceinline__ u64 hash_cell(const DCol& c, u64 i) {
    switch (c.type) {
        case DBG_STRING: {
            StrRef s = dcol_str(c, i);
            return hash_bytes(s.p, s.len);
        }
        case DBG_DECIMAL128: return hash_i128(dcol_bits(c, i), dcol_hi(c, i));
        case DBG_BOOLEAN: return dcol_bits(c, i);
        case DBG_FLOAT32: case DBG_FLOAT64: return hash_prim(canon_float_bits(c.type, dcol_bits(c, i)));
        case DBG_INT8: case DBG_INT16: case DBG_INT32: case DBG_DATE:
            return hash_prim((u64)dcol_i64(c, i));  // `*self as u64` sign-extends
        default: return hash_prim(dcol_bits(c, i));
    }
}

// group_hash_columns + combine_group_hash_column (group_hash.rs:41-150)
__device__ __forceinline__ u64 group_hash(const DCol* keys, int nk, u64 i) {
    u64 h = 0;
    for (int k = 0; k < nk; ++k) {
        u64 v = dcol_valid(keys[k], i) ? hash_cell(keys[k], i) : NULL_HASH_VAL;
        h = k == 0 ? v : (h * NULL_HASH_VAL) ^ v;
    }
    return h;
}

// ------------------------------------------------------------------------------------------
// Key equality (row_match_columns): nulls equal nulls, floats by canonical bits, strings by bytes.
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ bool bytes_equal(const u8* a, const u8* b, u64 n) {
    u64 i = 0;
    for (; i + 8 <= n; i += 8)
        if (load_u64_unaligned(a + i) != load_u64_unaligned(b + i)) return false;
    if (i == n) return true;
    const u64 r = n - i;  // 1..7
    return ((load_partial(a + i, r) ^ load_partial(b + i, r)) & ((1ULL << (8 * r)) - 1)) == 0;
}

__device__ __forceinline__ bool cell_equal(const DCol& a, u64 i, const DCol& b, u64 j) {
    bool va = dcol_valid(a, i), vb = dcol_valid(b, j);
    if (!va || !vb) return va == vb;
    switch (a.type) {
        case DBG_STRING: {
            StrRef x = dcol_str(a, i), y = dcol_str(b, j);
            return x.len == y.len && bytes_equal(x.p, y.p, x.len);
        }
        case DBG_DECIMAL128: return dcol_bits(a, i) == dcol_bits(b, j) && dcol_hi(a, i) == dcol_hi(b, j);
        case DBG_FLOAT32: case DBG_FLOAT64:
            return canon_float_bits(a.type, dcol_bits(a, i)) == canon_float_bits(b.type, dcol_bits(b, j));
        default: return dcol_bits(a, i) == dcol_bits(b, j);
    }
}

// ------------------------------------------------------------------------------------------
// Predicate programs (postfix, three-valued)
// ------------------------------------------------------------------------------------------
struct DNode {
    int32_t op, cmp, col, col2;
    i64 i64v;
    double f64v;
    u64 lo;
    i64 hi;
    const u8* str;  // device copy of the constant
    u64 str_len;
};

__device__ __forceinline__ int cmp3_i64(i64 a, i64 b) { return a < b ? -1 : (a > b ? 1 : 0); }
__device__ __forceinline__ int cmp3_u64(u64 a, u64 b) { return a < b ? -1 : (a > b ? 1 : 0); }
__device__ __forceinline__ int cmp3_f64(double a, double b) {  // OrderedFloat: NaN greatest, NaN == NaN
    bool an = a != a, bn = b != b;
    if (an || bn) return an == bn ? 0 : (an ? 1 : -1);
    return a < b ? -1 : (a > b ? 1 : 0);
}
__device__ __forceinline__ int cmp3_i128(u64 alo, i64 ahi, u64 blo, i64 bhi) {
    if (ahi != bhi) return ahi < bhi ? -1 : 1;
    return cmp3_u64(alo, blo);
}
__device__ __forceinline__ int cmp3_bytes(const u8* a, u64 la, const u8* b, u64 lb) {
    u64 n = la < lb ? la : lb;
    for (u64 k = 0; k < n; ++k) {
        u8 x = gld<u8>(a + k), y = gld<u8>(b + k);
        if (x != y) return x < y ? -1 : 1;
    }
    return la < lb ? -1 : (la > lb ? 1 : 0);
}
__device__ __forceinline__ bool apply_cmp(int c, int o) {
    switch (c) {
        case DBG_CMP_EQ: return o == 0;
        case DBG_CMP_NE: return o != 0;
        case DBG_CMP_LT: return o < 0;
        case DBG_CMP_LE: return o <= 0;
        case DBG_CMP_GT: return o > 0;
        default: return o >= 0;
    }
}
__device__ __forceinline__ bool is_unsigned_t(int t) { return t == DBG_UINT8 || t == DBG_UINT16 || t == DBG_UINT32 || t == DBG_UINT64; }
__device__ __forceinline__ bool is_float_t(int t) { return t == DBG_FLOAT32 || t == DBG_FLOAT64; }

__device__ __forceinline__ int cmp_const(const DCol& c, u64 i, const DNode& n) {
    int t = c.type;
    if (t == DBG_STRING) {
        StrRef s = dcol_str(c, i);
        return cmp3_bytes(s.p, s.len, n.str, n.str_len);
    }
    if (is_float_t(t)) return cmp3_f64(dcol_f64(c, i), n.f64v);
    if (t == DBG_DECIMAL128) return cmp3_i128(dcol_bits(c, i), (i64)dcol_hi(c, i), n.lo, n.hi);
    if (is_unsigned_t(t)) return cmp3_u64(dcol_bits(c, i), (u64)n.i64v);
    return cmp3_i64(dcol_i64(c, i), n.i64v);  // signed ints, date, timestamp, boolean
}
__device__ __forceinline__ int cmp_cols(const DCol& a, const DCol& b, u64 i) {
    int t = a.type;
    if (t == DBG_STRING) {
        StrRef x = dcol_str(a, i), y = dcol_str(b, i);
        return cmp3_bytes(x.p, x.len, y.p, y.len);
    }
    if (is_float_t(t)) return cmp3_f64(dcol_f64(a, i), dcol_f64(b, i));
    if (t == DBG_DECIMAL128) return cmp3_i128(dcol_bits(a, i), (i64)dcol_hi(a, i), dcol_bits(b, i), (i64)dcol_hi(b, i));
    if (is_unsigned_t(t)) return cmp3_u64(dcol_bits(a, i), dcol_bits(b, i));
    return cmp3_i64(dcol_i64(a, i), dcol_i64(b, i));
}

// Evaluate the program on row i; TRUE keeps the row.  Values: 0 false, 1 true, 2 null.
__device__ __forceinline__ bool eval_pred(const DNode* nodes, int n_nodes, const DCol* cols, u64 i) {
    u32 st = 0;  // 2-bit stack, 16 deep
    int sp = 0;
    for (int k = 0; k < n_nodes; ++k) {
        const DNode& n = nodes[k];
        u32 v = 0;
        switch (n.op) {
            case DBG_PRED_TRUE: v = 1; break;
            case DBG_PRED_CMP_CONST:
                v = !dcol_valid(cols[n.col], i) ? 2u : (apply_cmp(n.cmp, cmp_const(cols[n.col], i, n)) ? 1u : 0u);
                break;
            case DBG_PRED_CMP_COLS:
                v = (!dcol_valid(cols[n.col], i) || !dcol_valid(cols[n.col2], i))
                        ? 2u : (apply_cmp(n.cmp, cmp_cols(cols[n.col], cols[n.col2], i)) ? 1u : 0u);
                break;
            case DBG_PRED_IS_NULL: v = dcol_valid(cols[n.col], i) ? 0u : 1u; break;
            case DBG_PRED_IS_NOT_NULL: v = dcol_valid(cols[n.col], i) ? 1u : 0u; break;
            case DBG_PRED_NOT: {
                u32 a = (st >> (2 * (sp - 1))) & 3u;
                sp -= 1;
                v = a == 2u ? 2u : (a ^ 1u);
                break;
            }
            case DBG_PRED_AND: case DBG_PRED_OR: {
                u32 b = (st >> (2 * (sp - 1))) & 3u, a = (st >> (2 * (sp - 2))) & 3u;
                sp -= 2;
                if (n.op == DBG_PRED_AND) v = (a == 0u || b == 0u) ? 0u : ((a == 1u && b == 1u) ? 1u : 2u);
                else v = (a == 1u || b == 1u) ? 1u : ((a == 0u && b == 0u) ? 0u : 2u);
                break;
            }
        }
        st = (st & ~(3u << (2 * sp))) | (v << (2 * sp));
        sp += 1;
    }
    return sp > 0 && ((st >> (2 * (sp - 1))) & 3u) == 1u;
}

// ------------------------------------------------------------------------------------------
// Aggregate states
// ------------------------------------------------------------------------------------------
// How one aggregate updates its state words.
enum {
    SUMK_I64 = 0,  // wrapping 64-bit add (i8..i64 -> Int64, u8..u64 -> UInt64)
    SUMK_F64 = 1,  // f64 add
    SUMK_I128 = 2  // 128-bit add with carry (Decimal128)
};
enum {
    MMK_I64 = 0,  // signed (ints, date, timestamp, Decimal128 with precision <= 18)
    MMK_U64 = 1,  // unsigned
    MMK_F64 = 2,  // OrderedFloat order via the monotone u64 transform
    MMK_I128 = 3  // Decimal128 with precision > 18: [seq, lo, hi] under a seqlock (agg.hpp at_minmax128)
};

struct DAgg {
    int32_t kind;      // dbg_agg_kind
    int32_t arg_type;  // -1 for count(*)
    int32_t sumk;      // SUMK_* (SUM / AVG)
    int32_t mmk;       // MMK_* (MIN / MAX)
    int32_t w0;        // first state word (slot word index, entry = word 0)
    int32_t nwords;
    int32_t flag_bit;  // bit in the flags word, -1 if the result validity is implied
    int32_t arg_nullable;
    // result
    int32_t res_type;
    uint8_t res_precision, res_scale, res_nullable, dec_check;  // dec_check: SUM p<=18 range check
    int32_t scale_add;  // AVG decimal
    int32_t res_width;
    int32_t avg_round;  // AVG_SQL on Decimal128: round-half-away divide (kind is DBG_AGG_AVG)
    int32_t ser_flags;  // serialized state (AggregateMeta::Serialized): SER_* bits
};
enum {
    SER_OR_NULL = 1,   // AggregateFunctionOrNullAdaptor appends its flag byte
    SER_NULL_ADPT = 2  // AggregateNullUnaryAdaptor<true> (nullable argument) appends its flag byte
};

// Monotone map of OrderedFloat<f64> onto u64 (NaN canonical & greatest).
__device__ __forceinline__ u64 f64_order_key(double d) {
    u64 b = (u64)__double_as_longlong(d);
    b = canon_float_bits(DBG_FLOAT64, b);
    return (b >> 63) ? ~b : (b | 0x8000000000000000ULL);
}
__device__ __forceinline__ double f64_from_order_key(u64 k) {
    u64 b = (k >> 63) ? (k & 0x7fffffffffffffffULL) : ~k;
    return __longlong_as_double((long long)b);
}

__host__ __device__ inline u64 state_init_word(const DAgg& a, int w) {
    if ((a.kind == DBG_AGG_MIN || a.kind == DBG_AGG_MAX) && a.mmk == MMK_I128) {
        // identity: i128::MAX for MIN, i128::MIN for MAX; word 0 is the sequence counter
        if (w == 0) return 0ULL;
        const bool mn = a.kind == DBG_AGG_MIN;
        if (w == 1) return mn ? ~0ULL : 0ULL;
        return mn ? 0x7fffffffffffffffULL : 0x8000000000000000ULL;
    }
    if (a.kind == DBG_AGG_MIN) {
        if (a.mmk == MMK_I64) return 0x7fffffffffffffffULL;
        return ~0ULL;  // U64 / F64-order
    }
    if (a.kind == DBG_AGG_MAX) {
        if (a.mmk == MMK_I64) return 0x8000000000000000ULL;
        return 0ULL;
    }
    return 0ULL;
}
