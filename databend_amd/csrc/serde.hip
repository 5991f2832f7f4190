// serde.hip — ingest of serialized partial states (AggregateMeta::Serialized) on gfx950.
//
// The reference's final stage re-inserts a Serialized block [Binary state per aggregate...,
// group columns...] with AggregateHashTable::add_groups(.., agg_states) — probe, then
// AggregateFunction::batch_merge of each state column (EAGG/aggregate_function.rs:96-103) —
// from SerializedPayload::convert_to_aggregate_table (AGG/aggregate_meta.rs:57-101).  Here one
// pass turns every row into an exchange record ([group hash][key part][state words], the layout
// dbg_agg_record_layout describes): the group hash of its key columns and the borsh state bytes
// decoded into the table's state words.  The records then merge through the same record insert
// as dbg_agg_merge_records (merge_states), so a serialized row and an exported record of the same
// group are indistinguishable to the table.
//
// One thread per row: the work is a handful of dependent byte loads per aggregate, HBM-bound on
// the state bytes (≈ 9-26 B per aggregate per row) plus the record write.
#include "agg_dev.hpp"
#include "serde.hpp"

// Little-endian value of `n` (<= 8) bytes at p (unaligned: borsh rows are packed).
__device__ __forceinline__ u64 ld_le(const u8* p, u32 n) {
    u64 v = 0;
    for (u32 b = 0; b < n; ++b) v |= (u64)gld<u8>(p + b) << (8 * b);
    return v;
}

// One aggregate's serialized state (borsh struct, then AggregateNullUnaryAdaptor's flag byte for a
// nullable argument, then AggregateFunctionOrNullAdaptor's flag byte) -> the state words of a
// record (w = record state words, 0-based: word j of the slot is w[j - 1]).
// Returns 0, ERR_SER_MALFORMED (length does not match the state) or ERR_SER_UNREP (a NULL result
// the state words cannot carry: OrNull flag 0 / None without a nullable argument — states the
// reference's own partial never writes, aggregate_ornull_adaptor.rs:133-171).
__device__ __forceinline__ u32 ser_decode(const Spec& S, const DAgg& A, const u8* p, u64 len, u64* w, u64* flags) {
    u64 body = len;
    bool or_flag = true, has = true;
    if (A.ser_flags & SER_OR_NULL) {  // merge: flag = place flag || reader flag (:181-187)
        if (body < 1) return ERR_SER_MALFORMED;
        or_flag = gld<u8>(p + body - 1) > 0;
        body--;
    }
    if (A.ser_flags & SER_NULL_ADPT) {  // merge: nested merge only when the flag is 1 (:210-224)
        if (body < 1) return ERR_SER_MALFORMED;
        has = gld<u8>(p + body - 1) == 1;
        body--;
    }
    u64* x = w + (A.w0 - 1);
    switch (A.kind) {
        case DBG_AGG_COUNT:  // AggregateCountState: u64 (aggregate_count.rs:152-162)
            if (body != 8) return ERR_SER_MALFORMED;
            x[0] = ld_le(p, 8);
            return 0;
        case DBG_AGG_SUM: {  // NumberSumState {TSum} / DecimalSumState {i128}
            const u32 n = A.sumk == SUMK_I128 ? 16 : 8;
            if (body != n) return ERR_SER_MALFORMED;
            if (has) {
                x[0] = ld_le(p, 8);
                if (n == 16) x[1] = ld_le(p + 8, 8);
            }
            break;
        }
        case DBG_AGG_AVG: {  // Number/DecimalAvgState {value, count: u64}
            const u32 k = A.sumk == SUMK_I128 ? 2 : 1;
            if (body != 8 * k + 8) return ERR_SER_MALFORMED;
            if (has) {
                x[0] = ld_le(p, 8);
                if (k == 2) x[1] = ld_le(p + 8, 8);
                x[k] = ld_le(p + 8 * k, 8);
            }
            // a NULL AVG is count == 0; OrNull 0 with a count cannot be carried
            if (!or_flag && has && x[k] != 0) return ERR_SER_UNREP;
            return 0;
        }
        default: {  // MIN / MAX: MinMaxAnyState {Option<T>}, T in its own width
            if (body < 1) return ERR_SER_MALFORMED;
            const u8 tag = gld<u8>(p);
            const u32 aw = type_width(A.arg_type);
            if (tag > 1 || body != (tag ? 1u + aw : 1u)) return ERR_SER_MALFORMED;
            if (!tag) has = false;
            if (has) {
                const u8* v = p + 1;
                if (A.mmk == MMK_I128) {
                    x[0] = 0;  // even sequence word
                    x[1] = ld_le(v, 8);
                    x[2] = ld_le(v + 8, 8);
                } else if (A.mmk == MMK_F64) {
                    const double d = A.arg_type == DBG_FLOAT32 ? (double)__uint_as_float((u32)ld_le(v, 4))
                                                               : __longlong_as_double((long long)ld_le(v, 8));
                    x[0] = f64_order_key(d);
                } else {
                    u64 b = ld_le(v, aw < 8 ? aw : 8);  // Decimal128 (p <= 18): the low word holds it
                    if (A.mmk == MMK_I64 && aw < 8 && ((b >> (8 * aw - 1)) & 1)) b |= ~0ULL << (8 * aw);
                    x[0] = b;
                }
            }
            break;
        }
    }
    // SUM / MIN / MAX: result validity lives in the flags word when the argument is nullable
    if (A.flag_bit >= 0) {
        if (has && or_flag) *flags |= 1ULL << A.flag_bit;
    } else if (!(has && or_flag)) {
        return ERR_SER_UNREP;
    }
    return 0;
}

__global__ void __launch_bounds__(256) ser_ingest_kernel(const Spec* __restrict__ spec, SerIngest in, u64 n, u8* __restrict__ rec_out,
                                                         u64* __restrict__ err) {
    const Spec& S = *spec;
    u32 e = 0;
    for (u64 i = blockIdx.x * (u64)blockDim.x + threadIdx.x; i < n; i += (u64)gridDim.x * blockDim.x) {
        u8* rec = rec_out + i * S.rec_width;
        *(u64*)rec = group_hash(in.keys, S.n_keys, i);
        for (int c = 0; c < S.n_keys; ++c) {
            const DCol& kc = in.keys[c];
            const bool v = dcol_valid(kc, i);
            if (S.key_types[c].nullable) rec[S.rec_val_off[c]] = v ? 1 : 0;
            u64* kd = (u64*)(rec + S.rec_key_off[c]);
            if (kc.type == DBG_STRING) {  // (offset into the column's own bytes, len)
                const u64 a = gld<u64>(kc.offsets + i), b = gld<u64>(kc.offsets + i + 1);
                kd[0] = a;
                kd[1] = b - a;
            } else {
                kd[0] = dcol_bits(kc, i);
                if (kc.type == DBG_DECIMAL128) kd[1] = dcol_hi(kc, i);
            }
        }
        u64* w = (u64*)(rec + S.rec_state_off);
        for (int k = 1; k <= S.n_words; ++k) w[k - 1] = S.slot_init[k];
        u64 flags = 0;
        for (int a = 0; a < S.n_aggs; ++a) {
            const u64 o0 = gld<u64>(in.st_offs[a] + i), o1 = gld<u64>(in.st_offs[a] + i + 1);
            e |= ser_decode(S, S.aggs[a], in.st_data[a] + o0, o1 - o0, w, &flags);
        }
        if (S.flags_word >= 0) w[S.flags_word - 1] = flags;
    }
    if (e) atomicOr((unsigned long long*)err, (unsigned long long)e);
}

void launch_ser_ingest(hipStream_t s, const Spec* dspec, const SerIngest& in, u64 n, u8* rec_out, u64* err) {
    if (!n) return;
    u64 blocks = (n + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL(ser_ingest_kernel, dim3((u32)blocks), dim3(256), 0, s, dspec, in, n, rec_out, err);
}
