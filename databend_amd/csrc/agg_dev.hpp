// agg_dev.hpp — device helpers shared by agg.hip (HBM table) and pp.hip (partitioned payload):
// packed-key hashing, state updates (accumulate_keys / merge_states) and results (merge_result).
#pragma once
#include "agg.hpp"

__device__ __forceinline__ u64 width_mask(u32 w) { return w >= 8 ? ~0ULL : ((1ULL << (8 * w)) - 1); }

// AggHash of a cell from its raw bits (inline keys / records).
__device__ __forceinline__ u64 hash_bits(int type, u64 b) {
    switch (type) {
        case DBG_BOOLEAN: return b & 1;
        case DBG_FLOAT32: case DBG_FLOAT64: return hash_prim(canon_float_bits(type, b));
        case DBG_INT8: return hash_prim((u64)(i64)(int8_t)b);
        case DBG_INT16: return hash_prim((u64)(i64)(int16_t)b);
        case DBG_INT32: case DBG_DATE: return hash_prim((u64)(i64)(int32_t)b);
        default: return hash_prim(b);
    }
}

__device__ __forceinline__ u32 ref_bid(u64 e) { return (u32)((e >> 32) & 0xFFFF); }
__device__ __forceinline__ u32 ref_row(u64 e) { return (u32)e; }

// ------------------------------------------------------------------------------------------
// State updates on an LDS (AS_LDS) or HBM (AS_GLB) slot.  The address space is a template
// parameter, never inferred: a slot pointer that may be either (a phi of the LDS and the HBM
// branch) compiles to FLAT atomics, which count against vmcnt as well as lgkmcnt — every LDS
// wait then drains all global loads in flight and the streaming pipeline collapses.
// ------------------------------------------------------------------------------------------
// wptr / asp / at_* / vld live in agg.hpp (shared with part.hip)

template <int AS>
__device__ __forceinline__ void add128(wptr<AS> p, u64 lo, u64 hi) {
    u64 old = at_add<AS>(p, lo);
    u64 carry = (old + lo) < old ? 1ULL : 0ULL;
    u64 h = hi + carry;
    if (h) at_add<AS>(p + 1, h);
}

template <int AS>
__device__ __forceinline__ void set_flag(wptr<AS> st, int fw, int bit) {
    u64 m = 1ULL << bit;
    if (!(st[fw] & m)) at_or<AS>(st + fw, m);
}

// accumulate_keys of every aggregate for input row i into the slot at st (word 0 = entry).
template <int AS>
__device__ __forceinline__ void apply_row(const Spec& S, wptr<AS> st, const BatchDesc& B, u64 i) {
    for (int a = 0; a < S.n_aggs; ++a) {
        const DAgg& A = S.aggs[a];
        const DCol& c = B.args[a];
        if (A.arg_type >= 0 && A.arg_nullable && !dcol_valid(c, i)) continue;
        wptr<AS> w = st + A.w0;
        switch (A.kind) {
            case DBG_AGG_COUNT: at_add<AS>(w, 1ULL); break;
            case DBG_AGG_SUM: case DBG_AGG_AVG: {
                if (A.sumk == SUMK_I64) at_add<AS>(w, (u64)dcol_i64(c, i));
                else if (A.sumk == SUMK_F64) at_addf<AS>(w, dcol_f64(c, i));
                else add128<AS>(w, dcol_bits(c, i), dcol_hi(c, i));
                if (A.kind == DBG_AGG_AVG) at_add<AS>(w + (A.sumk == SUMK_I128 ? 2 : 1), 1ULL);
                break;
            }
            case DBG_AGG_MIN: case DBG_AGG_MAX: {
                bool mn = A.kind == DBG_AGG_MIN;
                if (A.mmk == MMK_I128) at_minmax128<AS>(w, dcol_bits(c, i), dcol_hi(c, i), mn, S.err);
                else if (A.mmk == MMK_I64) at_minmax<AS>(w, (u64)dcol_i64(c, i), mn, true);
                else at_minmax<AS>(w, A.mmk == MMK_U64 ? dcol_bits(c, i) : f64_order_key(dcol_f64(c, i)), mn, false);
                break;
            }
        }
        if (A.flag_bit >= 0) set_flag<AS>(st, S.flags_word, A.flag_bit);
    }
}

// merge_states of a partial state (word array r, same layout) into st.  SC1: read r with sc1
// loads (words parked by another workgroup in this launch, see block_flush).
// RAS: address space of r (LDS table rows being flushed, or global records / parked rows)
template <bool SC1, int RAS>
__device__ __forceinline__ u64 rdw(const u64* p) { return SC1 ? ld_sc1(p) : *asp<RAS>(p); }

// merge_states with the partial state's word w given by get(w) (memory or registers)
template <int AS, typename G>
__device__ __forceinline__ void apply_state_get(const Spec& S, wptr<AS> st, G get) {
    for (int a = 0; a < S.n_aggs; ++a) {
        const DAgg& A = S.aggs[a];
        wptr<AS> w = st + A.w0;
        const int x = A.w0;
        const u64 x0 = get(x);
        switch (A.kind) {
            case DBG_AGG_COUNT: if (x0) at_add<AS>(w, x0); break;
            case DBG_AGG_SUM: case DBG_AGG_AVG: {
                if (A.sumk == SUMK_I64) { if (x0) at_add<AS>(w, x0); }
                else if (A.sumk == SUMK_F64) at_addf<AS>(w, __longlong_as_double((long long)x0));
                else add128<AS>(w, x0, get(x + 1));
                if (A.kind == DBG_AGG_AVG) {
                    int k = A.sumk == SUMK_I128 ? 2 : 1;
                    u64 xk = get(x + k);
                    if (xk) at_add<AS>(w + k, xk);
                }
                break;
            }
            case DBG_AGG_MIN: case DBG_AGG_MAX:
                if (A.mmk == MMK_I128) at_minmax128<AS>(w, get(x + 1), get(x + 2), A.kind == DBG_AGG_MIN, S.err);
                else at_minmax<AS>(w, x0, A.kind == DBG_AGG_MIN, A.mmk == MMK_I64);
                break;
        }
    }
    if (S.flags_word >= 0) {
        u64 f = get(S.flags_word);
        if (f) at_or<AS>(st + S.flags_word, f);
    }
}

template <int AS, bool SC1 = false, int RAS = AS_GLB>
__device__ __forceinline__ void apply_state(const Spec& S, wptr<AS> st, const u64* r) {
    apply_state_get<AS>(S, st, [&](int w) { return rdw<SC1, RAS>(r + w); });
}

struct U128 {
    u64 lo, hi;
};
__device__ __forceinline__ U128 u128_neg(U128 a) {
    U128 r;
    r.lo = ~a.lo + 1;
    r.hi = ~a.hi + (r.lo == 0 ? 1 : 0);
    return r;
}
// magnitude * 10 with overflow detection (> limit)
__device__ __forceinline__ bool u128_mul10(U128& a) {
    u64 lo_hi = __umul64hi(a.lo, 10ULL);
    u64 lo = a.lo * 10ULL;
    u64 hi_hi = __umul64hi(a.hi, 10ULL);
    u64 hi = a.hi * 10ULL;
    u64 nhi = hi + lo_hi;
    bool ovf = hi_hi != 0 || nhi < hi;
    a.lo = lo;
    a.hi = nhi;
    return ovf;
}
// (a / d) truncating, d > 0
__device__ __forceinline__ U128 u128_div_u64(U128 a, u64 d) {
    U128 q{0, 0};
    q.hi = a.hi / d;
    u64 r = a.hi % d;
    u64 lo = 0;
    if (d <= 0xFFFFFFFFULL) {  // two 64/32 long-division steps instead of 64 iterations
        const u64 c1 = (r << 32) | (a.lo >> 32);
        const u64 q1 = c1 / d;
        const u64 c0 = ((c1 - q1 * d) << 32) | (a.lo & 0xFFFFFFFFULL);
        q.lo = (q1 << 32) | (c0 / d);
        return q;
    }
    for (int b = 63; b >= 0; --b) {
        u64 top = r >> 63;
        r = (r << 1) | ((a.lo >> b) & 1);
        if (top || r >= d) {
            r -= d;
            lo |= 1ULL << b;
        }
    }
    q.lo = lo;
    return q;
}
// (hi:lo) / d for hi < d: the quotient fits 64 bits; *r = remainder
__device__ __forceinline__ u64 div128_64(u64 hi, u64 lo, u64 d, u64* r) {
    u64 q = 0, rr = hi;
    for (int b = 63; b >= 0; --b) {
        u64 top = rr >> 63;
        rr = (rr << 1) | ((lo >> b) & 1);
        if (top || rr >= d) {
            rr -= d;
            q |= 1ULL << b;
        }
    }
    *r = rr;
    return q;
}
// SQL avg's decimal divide: do_round_div(sum, count, k) (EXP/types/decimal.rs:480-489) — in
// 256-bit arithmetic (sum * 10^k +- count / 2) / count, truncated toward zero, low 128 bits.
// |sum| * 10^k (k <= 12) spans at most 192 bits; count > 0.
__device__ __forceinline__ U128 dec_round_div(u64 lo, u64 hi, int k, u64 d) {
    const bool neg = (i64)hi < 0;
    U128 m{lo, hi};
    if (neg) m = u128_neg(m);
    u64 p = 1;
    for (int i = 0; i < k; ++i) p *= 10;
    // 192-bit product [l0, l1, l2]
    u64 l0 = m.lo * p, c0 = __umul64hi(m.lo, p);
    u64 t1 = m.hi * p, l2 = __umul64hi(m.hi, p);
    u64 l1 = t1 + c0;
    l2 += l1 < t1 ? 1 : 0;
    // + d / 2 (same magnitude rounding for both signs: truncation is symmetric)
    const u64 half = d >> 1;
    u64 n0 = l0 + half;
    if (n0 < l0) {
        l1 += 1;
        if (l1 == 0) l2 += 1;
    }
    u64 r;
    if (d <= 0xFFFFFFFFULL) {  // a count below 2^32 (always, in practice): six 64/32 long-division
                               // steps instead of 192 shift-subtract iterations
        const u32 dig[6] = {(u32)(l2 >> 32), (u32)l2, (u32)(l1 >> 32), (u32)l1, (u32)(n0 >> 32), (u32)n0};
        u32 qd[6];
        r = 0;
#pragma unroll
        for (int j = 0; j < 6; ++j) {
            const u64 cur = (r << 32) | dig[j];
            qd[j] = (u32)(cur / d);
            r = cur - (u64)qd[j] * d;
        }
        U128 q{((u64)qd[4] << 32) | qd[5], ((u64)qd[2] << 32) | qd[3]};
        return neg ? u128_neg(q) : q;
    }
    div128_64(0, l2, d, &r);  // the quotient's top limb is dropped (low 128 bits)
    u64 q1 = div128_64(r, l1, d, &r);
    u64 q0 = div128_64(r, n0, d, &r);
    U128 q{q0, q1};
    return neg ? u128_neg(q) : q;
}
// 10^38 - 1 = 0x4B3B4CA85A86C47A_098A223FFFFFFFFF
#define DEC38_MAX_HI 0x4B3B4CA85A86C47AULL
#define DEC38_MAX_LO 0x098A223FFFFFFFFFULL
__device__ __forceinline__ bool dec38_out_of_range(u64 lo, u64 hi) {
    U128 m{lo, hi};
    if ((i64)hi < 0) m = u128_neg(m);
    if (m.hi != DEC38_MAX_HI) return m.hi > DEC38_MAX_HI;
    return m.lo > DEC38_MAX_LO;
}

// AggregateFunction::serialize of one state (AggregateMeta::Serialized, EAGG/payload_flush.rs:
// 129-164): the borsh encoding of the reference's state struct — NumberSumState {value} (8 B of
// the sum type), DecimalSumState {value: i128}, Number/DecimalAvgState {value, count: u64},
// AggregateCountState's u64, MinMaxAnyState {value: Option<T>} (tag byte, then T's own width) —
// then the flag byte of AggregateNullUnaryAdaptor<true> (nullable argument: "had a non-NULL
// input", aggregate_null_unary_adaptor.rs:200-207) and of AggregateFunctionOrNullAdaptor (1: the
// group received rows, aggregate_ornull_adaptor.rs:135-163, 175-179).  Returns the byte count.
__device__ __forceinline__ u32 agg_serialize(const Spec& S, const DAgg& A, const u64* st, u8* d) {
    const u64* w = st + A.w0;
    u32 n = 0;
    auto put = [&](u64 v, u32 bytes) {
        for (u32 b = 0; b < bytes; ++b) d[n++] = (u8)(v >> (8 * b));
    };
    bool has = true;  // the null adaptor's flag: a non-NULL input reached the state
    switch (A.kind) {
        case DBG_AGG_COUNT: put(w[0], 8); return n;
        case DBG_AGG_SUM:
            put(w[0], 8);
            if (A.sumk == SUMK_I128) put(w[1], 8);
            if (A.flag_bit >= 0) has = (st[S.flags_word] >> A.flag_bit) & 1;
            break;
        case DBG_AGG_AVG: {
            const int k = A.sumk == SUMK_I128 ? 2 : 1;
            put(w[0], 8);
            if (k == 2) put(w[1], 8);
            put(w[k], 8);
            has = w[k] != 0;
            break;
        }
        default: {  // MIN / MAX
            if (A.flag_bit >= 0) has = (st[S.flags_word] >> A.flag_bit) & 1;
            put(has ? 1 : 0, 1);
            if (has) {
                const u32 aw = type_width(A.arg_type);
                if (A.mmk == MMK_I128) {
                    put(w[1], 8);
                    put(w[2], 8);
                } else if (A.mmk == MMK_F64) {
                    const double x = f64_from_order_key(w[0]);
                    if (A.arg_type == DBG_FLOAT32) put((u64)__float_as_uint((float)x), 4);
                    else put((u64)__double_as_longlong(x), 8);
                } else if (aw == 16) {  // Decimal128 with precision <= 18: i64 state, i128 bytes
                    put(w[0], 8);
                    put((i64)w[0] < 0 ? ~0ULL : 0ULL, 8);
                } else {
                    put(w[0], aw);  // low bytes of the (sign-extended) value: T's own width
                }
            }
        }
    }
    if (A.ser_flags & SER_NULL_ADPT) put(has ? 1 : 0, 1);
    if (A.ser_flags & SER_OR_NULL) put(1, 1);
    return n;
}

__device__ __forceinline__ void write_bytes(void* dst, u64 pos, u32 w, u64 lo, u64 hi) {
    u8* p = (u8*)dst + pos * w;
    switch (w) {
        case 1: *p = (u8)lo; break;
        case 2: *(uint16_t*)p = (uint16_t)lo; break;
        case 4: *(u32*)p = (u32)lo; break;
        case 8: *(u64*)p = lo; break;
        default: ((u64*)p)[0] = lo; ((u64*)p)[1] = hi; break;
    }
}

// Result value of aggregate A from its state words; returns validity.
__device__ __forceinline__ bool agg_result(const Spec& S, const DAgg& A, const u64* st, u64& lo, u64& hi, u64* err) {
    const u64* w = st + A.w0;
    bool valid = true;
    if (A.res_nullable) {
        if (A.kind == DBG_AGG_AVG) valid = w[A.sumk == SUMK_I128 ? 2 : 1] != 0;
        else if (A.flag_bit >= 0) valid = (st[S.flags_word] >> A.flag_bit) & 1;
    }
    hi = 0;
    switch (A.kind) {
        case DBG_AGG_COUNT: lo = w[0]; break;
        case DBG_AGG_SUM:
            lo = w[0];
            if (A.sumk == SUMK_I128) {
                hi = w[1];
                if (valid && A.dec_check && dec38_out_of_range(lo, hi)) atomicOr((unsigned long long*)err, (unsigned long long)ERR_DEC_OVERFLOW);
            }
            if (!valid) lo = hi = 0;
            break;
        case DBG_AGG_AVG: {
            u64 cnt = w[A.sumk == SUMK_I128 ? 2 : 1];
            if (!valid || cnt == 0) {
                lo = hi = 0;
                break;
            }
            if (A.avg_round) {  // SQL avg on Decimal128: SUM's range check, then the rounding divide
                if (A.dec_check && dec38_out_of_range(w[0], w[1])) atomicOr((unsigned long long*)err, (unsigned long long)ERR_DEC_OVERFLOW);
                U128 q = dec_round_div(w[0], w[1], A.scale_add, cnt);
                lo = q.lo;
                hi = q.hi;
            } else if (A.sumk == SUMK_I128) {
                U128 m{w[0], w[1]};
                bool neg = (i64)w[1] < 0;
                if (neg) m = u128_neg(m);
                bool ovf = false;
                for (int k = 0; k < A.scale_add; ++k) ovf |= u128_mul10(m);
                // checked_mul fits i128 iff magnitude <= 2^127 - 1 (+1 when negative)
                if (m.hi >> 63) ovf |= !(neg && m.hi == 0x8000000000000000ULL && m.lo == 0);
                if (ovf) atomicOr((unsigned long long*)err, (unsigned long long)ERR_DEC_OVERFLOW);
                U128 q = u128_div_u64(m, cnt);
                if (neg) q = u128_neg(q);
                lo = q.lo;
                hi = q.hi;
            } else {
                double sum;
                if (A.sumk == SUMK_F64) sum = __longlong_as_double((long long)w[0]);
                else if (A.arg_type == DBG_UINT8 || A.arg_type == DBG_UINT16 || A.arg_type == DBG_UINT32 || A.arg_type == DBG_UINT64)
                    sum = (double)w[0];
                else sum = (double)(i64)w[0];
                double r = sum / (double)cnt;
                lo = (u64)__double_as_longlong(r);
            }
            break;
        }
        case DBG_AGG_MIN: case DBG_AGG_MAX: {
            if (!valid) {
                lo = hi = 0;
                break;
            }
            u64 v = w[0];
            if (A.mmk == MMK_I128) {
                lo = w[1];
                hi = w[2];
            } else if (A.mmk == MMK_F64) {
                double d = f64_from_order_key(v);
                if (A.res_type == DBG_FLOAT32) lo = (u64)__float_as_uint((float)d);
                else lo = (u64)__double_as_longlong(d);
            } else {
                lo = v;
                if (A.res_type == DBG_DECIMAL128) hi = (i64)v < 0 ? ~0ULL : 0ULL;
            }
            break;
        }
    }
    return valid;
}

// One aggregate's output for group row `row`: its result (merge_result) or, in serialize mode,
// its serialized state.
__device__ __forceinline__ void write_agg(const Spec& S, int a, const u64* st, u64 row, const OutDesc& out, u64* err) {
    const DAgg& A = S.aggs[a];
    if (out.ser) {
        const u32 len = agg_serialize(S, A, st, (u8*)out.agg_data[a] + row * out.ser_stride[a]);
        out.agg_valid[a][row] = (u8)len;
        return;
    }
    u64 lo, hi;
    const bool v = agg_result(S, A, st, lo, hi, err);
    write_bytes(out.agg_data[a], row, A.res_width, lo, hi);
    if (out.agg_valid[a]) out.agg_valid[a][row] = v ? 1 : 0;
}
