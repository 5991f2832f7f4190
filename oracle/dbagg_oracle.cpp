// ============================================================================================
// ORACLE — TEST INFRASTRUCTURE ONLY.
//
// A CPU restatement (C++17) of Databend's vectorized filter + hash GROUP BY path, written from
// the reference's Rust sources (sundy-li/databend @ 2024-10-24; no Rust toolchain exists in this
// image, so the reference itself cannot be built — SURVEY.md §8c).  Only tests/,
// __graft_entry__.smoke() and bench.py's cpu_baseline leg may load it, and only as the checker or
// the timed CPU baseline ("restated Databend CPU aggregator").  The product path
// (libdbgpu_agg.so) never links or calls it.
//
// Parity pinning: tests/test_oracle_golden.py checks this restatement against the reference's own
// golden files (src/query/functions/tests/it/aggregates/testdata/agg_group_by.txt), the closed
// form of agg_hashtable.rs:57-182 and the numbers()-based expectations of
// tests/sqllogictests/suites/base/03_common/03_0043_new_agg_hashtable.test.  Hash values and
// `hash % n` routing are pinned by no reference test: parity of those rests on this restatement
// of EAGG/group_hash.rs (marked "parity unpinned" in DESIGN.md).
//
// Path aliases: EAGG = src/query/expression/src/aggregate, FUN = src/query/functions/src/aggregates,
// AGG = src/query/service/src/pipelines/processors/transforms/aggregator, EXP = src/query/expression/src
// ============================================================================================
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "../include/dbgpu_agg.h"
#include "../include/dbgpu_datagen.h"

typedef uint8_t u8;
typedef uint32_t u32;
typedef uint64_t u64;
typedef int64_t i64;
typedef __int128 i128;
typedef unsigned __int128 u128;

namespace orc {

struct OverflowError : std::runtime_error {
    explicit OverflowError(const std::string& m) : std::runtime_error(m) {}
};
struct UnsupportedError : std::runtime_error {
    explicit UnsupportedError(const std::string& m) : std::runtime_error(m) {}
};

static thread_local std::string g_err;

// ------------------------------------------------------------------------------------------
// Column access (EXP/values.rs:157-176, arrow Bitmap LSB-first with offset)
// ------------------------------------------------------------------------------------------
static inline bool bit_at(const u8* bits, u64 off, u64 i) {
    u64 b = off + i;
    return (bits[b >> 3] >> (b & 7)) & 1;
}
static inline bool is_valid(const dbg_column& c, u64 i) {
    if (!c.dt.nullable || c.validity == nullptr) return true;
    return bit_at(c.validity, c.validity_offset, i);
}
template <class T>
static inline T val(const dbg_column& c, u64 i) {
    T v;
    memcpy(&v, (const u8*)c.data + i * sizeof(T), sizeof(T));
    return v;
}
static inline bool bool_val(const dbg_column& c, u64 i) { return bit_at((const u8*)c.data, c.data_offset, i); }
static inline const u8* str_ptr(const dbg_column& c, u64 i) { return (const u8*)c.data + c.offsets[i]; }
static inline u64 str_len(const dbg_column& c, u64 i) { return c.offsets[i + 1] - c.offsets[i]; }

static size_t fixed_width(int t) {
    switch (t) {
        case DBG_INT8: case DBG_UINT8: case DBG_BOOLEAN: return 1;
        case DBG_INT16: case DBG_UINT16: return 2;
        case DBG_INT32: case DBG_UINT32: case DBG_FLOAT32: case DBG_DATE: return 4;
        case DBG_INT64: case DBG_UINT64: case DBG_FLOAT64: case DBG_TIMESTAMP: return 8;
        case DBG_DECIMAL128: return 16;
        case DBG_STRING: return 0;
    }
    throw UnsupportedError("unknown type");
}

// ------------------------------------------------------------------------------------------
// Group hash (EAGG/group_hash.rs:39-265)
// ------------------------------------------------------------------------------------------
static const u64 NULL_HASH_VAL = 0xd1cefa08eb382d69ULL;  // group_hash.rs:39

// impl_agg_hash_for_primitive_types (group_hash.rs:194-218): `*self as u64` then the mixer.
static inline u64 hash_prim(u64 x) {
    x ^= x >> 32;
    x *= 0xd6e8feb86659fd93ULL;
    x ^= x >> 32;
    x *= 0xd6e8feb86659fd93ULL;
    x ^= x >> 32;
    return x;
}

// impl AggHash for [u8] (group_hash.rs:161-192): Murmur-like, tail bytes first-most-significant,
// no multiply after the tail.
static inline u64 hash_bytes(const u8* p, u64 len) {
    const u64 M = 0xc6a4a7935bd1e995ULL, SEED = 0xe17a1465ULL, R = 47;
    u64 h = SEED ^ (len * M);
    u64 nb = len / 8;
    for (u64 i = 0; i < nb; ++i) {
        u64 k;
        memcpy(&k, p + i * 8, 8);
        k *= M;
        k ^= k >> R;
        k *= M;
        h ^= k;
        h *= M;
    }
    const u8* t = p + nb * 8;
    u64 tl = len - nb * 8;
    for (u64 i = 0; i < tl; ++i) h ^= (u64)t[i] << (8 * (tl - i - 1));
    h ^= h >> R;
    h *= M;
    h ^= h >> R;
    return h;
}

// AggHash of one (non-null) cell of column c.
static inline u64 hash_cell(const dbg_column& c, u64 i) {
    switch (c.dt.type) {
        case DBG_INT8: return hash_prim((u64)(i64)val<int8_t>(c, i));   // sign-extending `as u64`
        case DBG_INT16: return hash_prim((u64)(i64)val<int16_t>(c, i));
        case DBG_INT32: case DBG_DATE: return hash_prim((u64)(i64)val<int32_t>(c, i));
        case DBG_INT64: case DBG_TIMESTAMP: return hash_prim((u64)val<int64_t>(c, i));
        case DBG_UINT8: return hash_prim((u64)val<uint8_t>(c, i));
        case DBG_UINT16: return hash_prim((u64)val<uint16_t>(c, i));
        case DBG_UINT32: return hash_prim((u64)val<uint32_t>(c, i));
        case DBG_UINT64: return hash_prim(val<uint64_t>(c, i));
        case DBG_FLOAT32: {  // OrderedFloat<f32>: NaN -> f32::NAN bits (group_hash.rs:238-247)
            float f = val<float>(c, i);
            u32 b;
            if (std::isnan(f)) b = 0x7fc00000u; else memcpy(&b, &f, 4);
            return hash_prim((u64)b);
        }
        case DBG_FLOAT64: {  // group_hash.rs:249-258
            double f = val<double>(c, i);
            u64 b;
            if (std::isnan(f)) b = 0x7ff8000000000000ULL; else memcpy(&b, &f, 8);
            return hash_prim(b);
        }
        case DBG_DECIMAL128: return hash_bytes((const u8*)c.data + i * 16, 16);  // i128::to_le_bytes
        case DBG_STRING: return hash_bytes(str_ptr(c, i), str_len(c, i));
        case DBG_BOOLEAN: return (u64)bool_val(c, i);  // group_hash.rs:220-224
    }
    throw UnsupportedError("hash: unsupported type");
}

// group_hash_columns (group_hash.rs:41-48) + combine_group_hash_column (:59-150) for rows
// [start, start+n) of every column.
static void group_hash_columns(const dbg_column* cols, int ncols, u64 start, u64 n, u64* out) {
    for (int k = 0; k < ncols; ++k) {
        const dbg_column& c = cols[k];
        for (u64 r = 0; r < n; ++r) {
            u64 i = start + r;
            bool ok = is_valid(c, i);
            if (k == 0) {
                out[r] = ok ? hash_cell(c, i) : NULL_HASH_VAL;
            } else {
                out[r] = out[r] * NULL_HASH_VAL ^ (ok ? hash_cell(c, i) : NULL_HASH_VAL);
            }
        }
    }
}

// ------------------------------------------------------------------------------------------
// Owned columns (results, flushed group columns, filtered blocks)
// ------------------------------------------------------------------------------------------
struct OwnedColumn {
    dbg_datatype dt{};
    std::vector<u8> data;
    std::vector<u64> offsets;   // strings
    std::vector<u8> valid;      // one byte per row (1 = valid)
    std::vector<u8> vbits;      // packed validity for the dbg_column view
    std::vector<u8> bbits;      // packed booleans for the dbg_column view
    u64 rows = 0;
    void clear() { data.clear(); offsets.assign(1, 0); valid.clear(); rows = 0; }
    dbg_column view() {
        dbg_column c{};
        c.dt = dt;
        c.len = rows;
        if (dt.type == DBG_BOOLEAN) {
            bbits.assign((rows + 7) / 8, 0);
            for (u64 i = 0; i < rows; ++i)
                if (data[i]) bbits[i >> 3] |= (u8)(1u << (i & 7));
            c.data = bbits.data();
        } else {
            c.data = data.data();
        }
        c.offsets = dt.type == DBG_STRING ? offsets.data() : nullptr;
        if (dt.nullable) {
            vbits.assign((rows + 7) / 8, 0);
            for (u64 i = 0; i < rows; ++i)
                if (valid[i]) vbits[i >> 3] |= (u8)(1u << (i & 7));
            c.validity = vbits.data();
        }
        return c;
    }
};

// Append row i of c to o (the `take` kernel, EXP/kernels/take.rs).
static void append_cell(OwnedColumn& o, const dbg_column& c, u64 i) {
    if (c.dt.type == DBG_STRING) {
        u64 l = str_len(c, i);
        const u8* p = str_ptr(c, i);
        o.data.insert(o.data.end(), p, p + l);
        o.offsets.push_back(o.data.size());
    } else if (c.dt.type == DBG_BOOLEAN) {
        o.data.push_back(bool_val(c, i) ? 1 : 0);
    } else {
        size_t w = fixed_width(c.dt.type);
        const u8* p = (const u8*)c.data + i * w;
        o.data.insert(o.data.end(), p, p + w);
    }
    o.valid.push_back(is_valid(c, i) ? 1 : 0);
    o.rows++;
}

// ------------------------------------------------------------------------------------------
// Bump arena (bumpalo stand-in: states and string keys live here)
// ------------------------------------------------------------------------------------------
struct Bump {
    std::vector<std::unique_ptr<u8[]>> chunks;
    size_t cap = 0, used = 0;
    u8* cur = nullptr;
    size_t allocated = 0;
    u8* alloc(size_t size, size_t align) {
        size_t off = (used + align - 1) & ~(align - 1);
        if (cur == nullptr || off + size > cap) {
            size_t sz = std::max<size_t>(size + align, 1 << 20);
            chunks.emplace_back(new u8[sz]);
            cur = chunks.back().get();
            cap = sz;
            used = 0;
            off = ((uintptr_t)cur + align - 1) / align * align - (uintptr_t)cur;
        }
        u8* p = cur + off;
        used = off + size;
        allocated += size;
        return p;
    }
};

// ------------------------------------------------------------------------------------------
// Aggregate functions (EAGG/aggregate_function.rs:34-168; FUN/*)
// ------------------------------------------------------------------------------------------
static i128 pow10_i128(int n) {
    i128 r = 1;
    for (int i = 0; i < n; ++i) r *= 10;
    return r;
}
static i128 dec_max() { return pow10_i128(38) - 1; }  // i128::MAX for Decimal (EXP/types/decimal.rs:653-655)

// Result column builder: push value bytes or a null.
struct Builder {
    OwnedColumn* col;
    template <class T>
    void push(T v) {
        const u8* p = (const u8*)&v;
        col->data.insert(col->data.end(), p, p + sizeof(T));
        col->valid.push_back(1);
        col->rows++;
    }
    void push_null(size_t width) {  // push_default + validity false
        col->data.insert(col->data.end(), width, 0);
        col->valid.push_back(0);
        col->rows++;
    }
};

struct AggFn {
    virtual ~AggFn() {}
    virtual size_t size() const = 0;
    virtual size_t align() const = 0;
    virtual void init_state(u8* p) const = 0;
    // AggregateFunction::accumulate_keys(places, offset, columns, rows): row k of the batch is
    // row (start + k) of `arg`.
    virtual void accumulate_keys(u8* const* places, size_t off, const dbg_column* arg, u64 start, u64 n) const = 0;
    virtual void accumulate_row(u8* place, const dbg_column* arg, u64 row) const = 0;
    virtual void merge_states(u8* place, u8* rhs) const = 0;
    virtual void merge_result(u8* place, Builder& b) const = 0;
    virtual dbg_datatype return_type() const = 0;
    virtual size_t result_width() const = 0;
    // AggregateFunction::serialize / merge (EAGG/aggregate_function.rs:88-105): the borsh bytes of
    // the state struct (FUN/aggregator_common.rs:159-170) — little-endian fixed-width integers and
    // floats, Option<T> = tag byte + T — and the inverse, merging a serialized state into place.
    virtual void serialize(const u8* place, std::vector<u8>& w) const = 0;
    virtual void merge(u8* place, const u8* r, size_t len) const = 0;
};

template <class T>
static inline void put_le(std::vector<u8>& w, T v, size_t bytes = sizeof(T)) {
    u8 b[16];
    memcpy(b, &v, sizeof(T));
    w.insert(w.end(), b, b + bytes);
}
// borsh_deserialize_state: a reader that must hold exactly the state's bytes
static inline void need(size_t len, size_t want) {
    if (len != want) throw UnsupportedError("serialized state: " + std::to_string(len) + " bytes, expected " + std::to_string(want));
}

// AggregateCountFunction (FUN/aggregate_count.rs:37-214): u64 state, counts rows / valid args.
struct CountFn : AggFn {
    bool has_arg;
    explicit CountFn(bool a) : has_arg(a) {}
    size_t size() const override { return 8; }
    size_t align() const override { return 8; }
    void init_state(u8* p) const override { *(u64*)p = 0; }
    void accumulate_keys(u8* const* places, size_t off, const dbg_column* arg, u64 start, u64 n) const override {
        for (u64 k = 0; k < n; ++k)
            if (!has_arg || is_valid(*arg, start + k)) *(u64*)(places[k] + off) += 1;
    }
    void accumulate_row(u8* place, const dbg_column* arg, u64 row) const override {
        if (!has_arg || is_valid(*arg, row)) *(u64*)place += 1;
    }
    void merge_states(u8* p, u8* r) const override { *(u64*)p += *(u64*)r; }
    void merge_result(u8* p, Builder& b) const override { b.push<u64>(*(u64*)p); }
    dbg_datatype return_type() const override { return dbg_datatype{DBG_UINT64, 0, 0, 0, 0}; }
    size_t result_width() const override { return 8; }
    // aggregate_count.rs:152-162: borsh u64
    void serialize(const u8* p, std::vector<u8>& w) const override { put_le<u64>(w, *(const u64*)p); }
    void merge(u8* p, const u8* r, size_t len) const override {
        need(len, 8);
        u64 x;
        memcpy(&x, r, 8);
        *(u64*)p += x;
    }
};

// Read an argument as a signed/unsigned/f64/i128 value.
template <class T>
static inline T arg_as(const dbg_column& c, u64 i);
template <> inline i64 arg_as<i64>(const dbg_column& c, u64 i) {
    switch (c.dt.type) {
        case DBG_INT8: return val<int8_t>(c, i);
        case DBG_INT16: return val<int16_t>(c, i);
        case DBG_INT32: case DBG_DATE: return val<int32_t>(c, i);
        default: return val<int64_t>(c, i);
    }
}
template <> inline u64 arg_as<u64>(const dbg_column& c, u64 i) {
    switch (c.dt.type) {
        case DBG_UINT8: return val<uint8_t>(c, i);
        case DBG_UINT16: return val<uint16_t>(c, i);
        case DBG_UINT32: return val<uint32_t>(c, i);
        case DBG_BOOLEAN: return bool_val(c, i) ? 1 : 0;
        default: return val<uint64_t>(c, i);
    }
}
template <> inline double arg_as<double>(const dbg_column& c, u64 i) {
    if (c.dt.type == DBG_FLOAT32) return (double)val<float>(c, i);
    return val<double>(c, i);
}
template <> inline i128 arg_as<i128>(const dbg_column& c, u64 i) { return val<i128>(c, i); }

// NumberSumState<TSum> (FUN/aggregate_sum.rs:64-113): wrapping `+=` (release overflow-checks off,
// Cargo.toml:353-358).  S = i64 (signed ints), u64 (unsigned), double (floats).
template <class S>
struct SumNumFn : AggFn {
    dbg_datatype rt;
    explicit SumNumFn(dbg_datatype r) : rt(r) {}
    size_t size() const override { return 8; }
    size_t align() const override { return 8; }
    void init_state(u8* p) const override { *(S*)p = 0; }
    static inline void add(S& s, S x) {
        if constexpr (std::is_integral<S>::value) s = (S)((u64)s + (u64)x); else s += x;
    }
    void accumulate_keys(u8* const* places, size_t off, const dbg_column* arg, u64 start, u64 n) const override {
        for (u64 k = 0; k < n; ++k) add(*(S*)(places[k] + off), arg_as<S>(*arg, start + k));
    }
    void accumulate_row(u8* place, const dbg_column* arg, u64 row) const override { add(*(S*)place, arg_as<S>(*arg, row)); }
    void merge_states(u8* p, u8* r) const override { add(*(S*)p, *(S*)r); }
    void merge_result(u8* p, Builder& b) const override { b.push<S>(*(S*)p); }
    dbg_datatype return_type() const override { return rt; }
    size_t result_width() const override { return 8; }
    // NumberSumState {value: TSum} (aggregate_sum.rs:64-113, derive(BorshSerialize))
    void serialize(const u8* p, std::vector<u8>& w) const override { put_le<S>(w, *(const S*)p); }
    void merge(u8* p, const u8* r, size_t len) const override {
        need(len, 8);
        S x;
        memcpy(&x, r, 8);
        add(*(S*)p, x);
    }
};

// DecimalSumState<OVERFLOW, Decimal128> (FUN/aggregate_sum.rs:115-170): i128 `+=` (wrapping in
// release) and, when OVERFLOW (input precision <= 18, :203-222), the range check after every add.
struct SumDecFn : AggFn {
    bool overflow;
    dbg_datatype rt;
    SumDecFn(bool o, dbg_datatype r) : overflow(o), rt(r) {}
    size_t size() const override { return 16; }
    size_t align() const override { return 16; }
    void init_state(u8* p) const override { i128 z = 0; memcpy(p, &z, 16); }
    void add(u8* p, i128 x) const {
        i128 s;
        memcpy(&s, p, 16);
        s = (i128)((u128)s + (u128)x);
        memcpy(p, &s, 16);
        if (overflow && (s > dec_max() || s < -dec_max())) throw OverflowError("Decimal overflow");
    }
    void accumulate_keys(u8* const* places, size_t off, const dbg_column* arg, u64 start, u64 n) const override {
        for (u64 k = 0; k < n; ++k) add(places[k] + off, arg_as<i128>(*arg, start + k));
    }
    void accumulate_row(u8* place, const dbg_column* arg, u64 row) const override { add(place, arg_as<i128>(*arg, row)); }
    void merge_states(u8* p, u8* r) const override {
        i128 x;
        memcpy(&x, r, 16);
        add(p, x);
    }
    void merge_result(u8* p, Builder& b) const override {
        i128 s;
        memcpy(&s, p, 16);
        b.push<i128>(s);
    }
    dbg_datatype return_type() const override { return rt; }
    size_t result_width() const override { return 16; }
    // DecimalSumState {value: i128}; merge = add (aggregate_sum.rs:158-160, range-checked)
    void serialize(const u8* p, std::vector<u8>& w) const override { w.insert(w.end(), p, p + 16); }
    void merge(u8* p, const u8* r, size_t len) const override {
        need(len, 16);
        i128 x;
        memcpy(&x, r, 16);
        add(p, x);
    }
};

// NumberAvgState<T, TSum> (FUN/aggregate_avg.rs:38-99): {value: TSum, count: u64};
// result = (value as f64) / (count as f64).
template <class S>
struct AvgNumFn : AggFn {
    size_t size() const override { return 16; }
    size_t align() const override { return 8; }
    void init_state(u8* p) const override {
        *(S*)p = 0;
        *(u64*)(p + 8) = 0;
    }
    static inline void add(u8* p, S x, u64 c) {
        *(u64*)(p + 8) += c;
        if constexpr (std::is_integral<S>::value) *(S*)p = (S)((u64) * (S*)p + (u64)x); else *(S*)p += x;
    }
    void accumulate_keys(u8* const* places, size_t off, const dbg_column* arg, u64 start, u64 n) const override {
        for (u64 k = 0; k < n; ++k) add(places[k] + off, arg_as<S>(*arg, start + k), 1);
    }
    void accumulate_row(u8* place, const dbg_column* arg, u64 row) const override { add(place, arg_as<S>(*arg, row), 1); }
    void merge_states(u8* p, u8* r) const override { add(p, *(S*)r, *(u64*)(r + 8)); }
    void merge_result(u8* p, Builder& b) const override {
        double v = (double)(*(S*)p) / (double)(*(u64*)(p + 8));
        b.push<double>(v);
    }
    dbg_datatype return_type() const override { return dbg_datatype{DBG_FLOAT64, 0, 0, 0, 0}; }
    size_t result_width() const override { return 8; }
    // NumberAvgState {value: TSum, count: u64} (aggregate_avg.rs:38-88)
    void serialize(const u8* p, std::vector<u8>& w) const override { w.insert(w.end(), p, p + 16); }
    void merge(u8* p, const u8* r, size_t len) const override {
        need(len, 16);
        S x;
        u64 c;
        memcpy(&x, r, 8);
        memcpy(&c, r + 8, 8);
        add(p, x, c);
    }
};

// DecimalAvgState<OVERFLOW, Decimal128> (FUN/aggregate_avg.rs:113-201): {value: i128, count};
// OVERFLOW when input precision > 18 (:235); result = value.checked_mul(10^scale_add)
// .checked_div(count) (truncating), None -> ErrorCode::Overflow.  Result Decimal(38, max(s,4)).
struct AvgDecFn : AggFn {
    bool overflow;
    int scale_add;
    dbg_datatype rt;
    AvgDecFn(bool o, int sa, dbg_datatype r) : overflow(o), scale_add(sa), rt(r) {}
    size_t size() const override { return 32; }
    size_t align() const override { return 16; }
    void init_state(u8* p) const override {
        memset(p, 0, 32);
    }
    void add(u8* p, i128 x, u64 c) const {
        *(u64*)(p + 16) += c;
        i128 s;
        memcpy(&s, p, 16);
        s = (i128)((u128)s + (u128)x);
        memcpy(p, &s, 16);
        if (overflow && (s > dec_max() || s < -dec_max())) throw OverflowError("Decimal overflow");
    }
    void accumulate_keys(u8* const* places, size_t off, const dbg_column* arg, u64 start, u64 n) const override {
        for (u64 k = 0; k < n; ++k) add(places[k] + off, arg_as<i128>(*arg, start + k), 1);
    }
    void accumulate_row(u8* place, const dbg_column* arg, u64 row) const override { add(place, arg_as<i128>(*arg, row), 1); }
    void merge_states(u8* p, u8* r) const override {
        i128 x;
        memcpy(&x, r, 16);
        add(p, x, *(u64*)(r + 16));
    }
    void merge_result(u8* p, Builder& b) const override {
        i128 s;
        memcpy(&s, p, 16);
        u64 c = *(u64*)(p + 16);
        i128 m = pow10_i128(scale_add);
        i128 prod;
        if (__builtin_mul_overflow(s, m, &prod)) throw OverflowError("Decimal overflow: mul");
        if (c == 0) throw OverflowError("Decimal overflow: div");
        b.push<i128>(prod / (i128)c);
    }
    dbg_datatype return_type() const override { return rt; }
    size_t result_width() const override { return 16; }
    // DecimalAvgState {value: i128, count: u64} (aggregate_avg.rs:113-171)
    void serialize(const u8* p, std::vector<u8>& w) const override { w.insert(w.end(), p, p + 24); }
    void merge(u8* p, const u8* r, size_t len) const override {
        need(len, 24);
        i128 x;
        u64 c;
        memcpy(&x, r, 16);
        memcpy(&c, r + 16, 8);
        add(p, x, c);
    }
};

// SQL avg(x) after the planner's rewrite sum(x) / if(count(x) = 0, 1, count(x))
// (SQL/planner/semantic/aggregate_rewriter.rs:145-208), Decimal128 argument: the sum is
// DecimalSumState<OVERFLOW = p <= 18> (as SumDecFn), the count UInt64 viewed as Decimal(20, 0),
// and the decimal divide (FUNCS/scalars/decimal/arithmetic.rs:87-112) has result scale
// max(s, min(s + 6, 12)) (EXP/types/decimal.rs:1015-1018) and value do_round_div(sum, count,
// scale - s) (EXP/types/decimal.rs:480-489): (sum * 10^k + count/2) / count when sum >= 0,
// (sum * 10^k - count/2) / count otherwise, in i256 (truncating), low 128 bits.
// (Numbers: the rewrite's f64 / f64 equals NumberAvgState's result, so AvgNumFn serves.)
struct SqlAvgDecFn : AggFn {
    SumDecFn sum;
    int k;
    dbg_datatype rt;
    SqlAvgDecFn(bool o, int kk, dbg_datatype r) : sum(o, r), k(kk), rt(r) {}
    size_t size() const override { return 32; }
    size_t align() const override { return 16; }
    void init_state(u8* p) const override { memset(p, 0, 32); }
    void accumulate_keys(u8* const* places, size_t off, const dbg_column* arg, u64 start, u64 n) const override {
        for (u64 j = 0; j < n; ++j) accumulate_row(places[j] + off, arg, start + j);
    }
    void accumulate_row(u8* place, const dbg_column* arg, u64 row) const override {
        sum.add(place, arg_as<i128>(*arg, row));
        *(u64*)(place + 16) += 1;
    }
    void merge_states(u8* p, u8* r) const override {
        i128 x;
        memcpy(&x, r, 16);
        sum.add(p, x);
        *(u64*)(p + 16) += *(u64*)(r + 16);
    }
    void merge_result(u8* p, Builder& b) const override {
        i128 s;
        memcpy(&s, p, 16);
        u64 c = *(u64*)(p + 16);
        if (c == 0) c = 1;  // if(count = 0, 1, count)
        const bool neg = s < 0;
        u128 m = neg ? (u128)0 - (u128)s : (u128)s;
        u64 mul = 1;
        for (int i = 0; i < k; ++i) mul *= 10;
        // |s| * 10^k as three 64-bit limbs, then + c / 2, then long division by c
        u128 lo_p = (u128)(u64)m * mul, hi_p = (u128)(u64)(m >> 64) * mul;
        u64 l0 = (u64)lo_p;
        u128 mid = (lo_p >> 64) + (u128)(u64)hi_p;
        u64 l1 = (u64)mid;
        u64 l2 = (u64)(hi_p >> 64) + (u64)(mid >> 64);
        u128 t = (u128)l0 + (c / 2);
        l0 = (u64)t;
        u128 t1 = (u128)l1 + (u64)(t >> 64);
        l1 = (u64)t1;
        l2 += (u64)(t1 >> 64);
        u128 r = l2 % c;
        u128 x1 = (r << 64) | l1;
        u64 q1 = (u64)(x1 / c);
        r = x1 % c;
        u128 x0 = (r << 64) | l0;
        u64 q0 = (u64)(x0 / c);
        u128 q = ((u128)q1 << 64) | q0;
        if (neg) q = (u128)0 - q;
        b.push<i128>((i128)q);
    }
    dbg_datatype return_type() const override { return rt; }
    size_t result_width() const override { return 16; }
    // the SQL rewrite has two reference states (sum, count), not one
    void serialize(const u8*, std::vector<u8>&) const override { throw UnsupportedError("serialized SQL avg"); }
    void merge(u8*, const u8*, size_t) const override { throw UnsupportedError("serialized SQL avg"); }
};

// MinMaxAnyState<T, CmpMin/CmpMax> (FUN/aggregate_min_max_any.rs:46-115,
// FUN/aggregate_scalar_state.rs:60-104): Option<T>; replace when l.partial_cmp(r) is Greater (MIN)
// / Less (MAX).  Floats are OrderedFloat (NaN greatest, all NaNs equal, -0 == +0).
template <class T>
struct MinMaxFn : AggFn {
    bool is_min;
    dbg_datatype rt;
    MinMaxFn(bool m, dbg_datatype r) : is_min(m), rt(r) {}
    size_t size() const override { return 32; }
    size_t align() const override { return 16; }
    void init_state(u8* p) const override { memset(p, 0, 32); }
    static int ord(T a, T b) {
        if constexpr (std::is_floating_point<T>::value) {
            bool an = std::isnan(a), bn = std::isnan(b);
            if (an || bn) return an == bn ? 0 : (an ? 1 : -1);
        }
        return a < b ? -1 : (a > b ? 1 : 0);
    }
    void add(u8* p, T x) const {
        T cur;
        memcpy(&cur, p + 16, sizeof(T));
        if (!p[0]) {
            p[0] = 1;
            memcpy(p + 16, &x, sizeof(T));
        } else {
            int o = ord(cur, x);
            if ((is_min && o > 0) || (!is_min && o < 0)) memcpy(p + 16, &x, sizeof(T));
        }
    }
    static T read(const dbg_column& c, u64 i) {
        if constexpr (std::is_same<T, double>::value) return arg_as<double>(c, i);
        else if constexpr (std::is_same<T, i128>::value) return val<i128>(c, i);
        else if constexpr (std::is_same<T, u64>::value) return arg_as<u64>(c, i);
        else return arg_as<i64>(c, i);
    }
    void accumulate_keys(u8* const* places, size_t off, const dbg_column* arg, u64 start, u64 n) const override {
        for (u64 k = 0; k < n; ++k) add(places[k] + off, read(*arg, start + k));
    }
    void accumulate_row(u8* place, const dbg_column* arg, u64 row) const override { add(place, read(*arg, row)); }
    void merge_states(u8* p, u8* r) const override {
        if (r[0]) {
            T x;
            memcpy(&x, r + 16, sizeof(T));
            add(p, x);
        }
    }
    void merge_result(u8* p, Builder& b) const override {
        T v;
        memcpy(&v, p + 16, sizeof(T));
        if (!p[0]) memset(&v, 0, sizeof(T));  // push_default
        // narrow back to the argument's width
        size_t w = fixed_width(rt.type);
        if (rt.type == DBG_FLOAT32) {
            float f = (float)(double)v;
            b.push<float>(f);
            return;
        }
        u8 buf[16];
        memcpy(buf, &v, sizeof(T));
        b.col->data.insert(b.col->data.end(), buf, buf + w);
        b.col->valid.push_back(1);
        b.col->rows++;
    }
    dbg_datatype return_type() const override { return rt; }
    size_t result_width() const override { return fixed_width(rt.type); }
    // MinMaxAnyState {value: Option<T>} in T's own width (aggregate_min_max_any.rs:46-56):
    // merge = add(rhs value) when Some (:95-100)
    void serialize(const u8* p, std::vector<u8>& w) const override {
        w.push_back(p[0] ? 1 : 0);
        if (!p[0]) return;
        T v;
        memcpy(&v, p + 16, sizeof(T));
        if (rt.type == DBG_FLOAT32) put_le<float>(w, (float)(double)v);
        else put_le<T>(w, v, fixed_width(rt.type));
    }
    void merge(u8* p, const u8* r, size_t len) const override {
        if (len < 1) need(len, 1);
        if (r[0] == 0) {
            need(len, 1);
            return;
        }
        const size_t wd = fixed_width(rt.type);
        need(len, 1 + wd);
        T x;
        if (rt.type == DBG_FLOAT32) {
            float f;
            memcpy(&f, r + 1, 4);
            x = (T)(double)f;
        } else if constexpr (std::is_same<T, double>::value) {
            memcpy(&x, r + 1, 8);
        } else if constexpr (std::is_same<T, i128>::value) {
            memcpy(&x, r + 1, 16);
        } else {
            u64 raw = 0;
            memcpy(&raw, r + 1, wd);
            if (std::is_signed<T>::value && wd < 8 && ((raw >> (8 * wd - 1)) & 1)) raw |= ~0ULL << (8 * wd);
            x = (T)raw;
        }
        add(p, x);
    }
};

// AggregateNullUnaryAdaptor<NULLABLE_RESULT=true> (FUN/adaptors/aggregate_null_unary_adaptor.rs):
// skip NULL args, flag byte after the nested state, NULL result when no valid input.
struct NullUnaryAdaptor : AggFn {
    std::unique_ptr<AggFn> inner;
    explicit NullUnaryAdaptor(AggFn* i) : inner(i) {}
    size_t size() const override { return inner->size() + inner->align(); }
    size_t align() const override { return inner->align(); }
    void init_state(u8* p) const override {
        p[inner->size()] = 0;
        inner->init_state(p);
    }
    void accumulate_keys(u8* const* places, size_t off, const dbg_column* arg, u64 start, u64 n) const override {
        for (u64 k = 0; k < n; ++k) {
            if (is_valid(*arg, start + k)) {
                places[k][off + inner->size()] = 1;
                inner->accumulate_row(places[k] + off, arg, start + k);
            }
        }
    }
    void accumulate_row(u8* place, const dbg_column* arg, u64 row) const override {
        if (is_valid(*arg, row)) {
            place[inner->size()] = 1;
            inner->accumulate_row(place, arg, row);
        }
    }
    void merge_states(u8* p, u8* r) const override {
        if (p[inner->size()] == 0) inner->init_state(p);
        if (r[inner->size()] == 1) {
            p[inner->size()] = 1;
            inner->merge_states(p, r);
        }
    }
    void merge_result(u8* p, Builder& b) const override {
        if (p[inner->size()] == 1) inner->merge_result(p, b);
        else b.push_null(inner->result_width());
    }
    // aggregate_null_unary_adaptor.rs:200-224: nested state, then the flag byte
    void serialize(const u8* p, std::vector<u8>& w) const override {
        inner->serialize(p, w);
        w.push_back(p[inner->size()]);
    }
    void merge(u8* p, const u8* r, size_t len) const override {
        if (len < 1) need(len, 1);
        if (p[inner->size()] == 0) inner->init_state(p);
        if (r[len - 1] == 1) {
            p[inner->size()] = 1;
            inner->merge(p, r, len - 1);
        }
    }
    dbg_datatype return_type() const override {
        dbg_datatype t = inner->return_type();
        t.nullable = 1;
        return t;
    }
    size_t result_width() const override { return inner->result_width(); }
};

// AggregateFunctionOrNullAdaptor (FUN/adaptors/aggregate_ornull_adaptor.rs:43-239).
struct OrNullAdaptor : AggFn {
    std::unique_ptr<AggFn> inner;
    bool inner_nullable;
    explicit OrNullAdaptor(AggFn* i) : inner(i), inner_nullable(i->return_type().nullable != 0) {}
    size_t size() const override { return inner->size() + inner->align(); }
    size_t align() const override { return inner->align(); }
    void init_state(u8* p) const override {
        p[inner->size()] = 0;
        inner->init_state(p);
    }
    void accumulate_keys(u8* const* places, size_t off, const dbg_column* arg, u64 start, u64 n) const override {
        inner->accumulate_keys(places, off, arg, start, n);
        for (u64 k = 0; k < n; ++k) places[k][off + inner->size()] = 1;
    }
    void accumulate_row(u8* place, const dbg_column* arg, u64 row) const override {
        inner->accumulate_row(place, arg, row);
        place[inner->size()] = 1;
    }
    void merge_states(u8* p, u8* r) const override {
        inner->merge_states(p, r);
        p[inner->size()] = (p[inner->size()] > 0 || r[inner->size()] > 0) ? 1 : 0;
    }
    void merge_result(u8* p, Builder& b) const override {
        if (p[inner->size()] == 0) b.push_null(inner->result_width());
        else inner->merge_result(p, b);
    }
    // aggregate_ornull_adaptor.rs:175-187: inner state, then the flag byte
    void serialize(const u8* p, std::vector<u8>& w) const override {
        inner->serialize(p, w);
        w.push_back(p[inner->size()]);
    }
    void merge(u8* p, const u8* r, size_t len) const override {
        if (len < 1) need(len, 1);
        const bool flag = p[inner->size()] > 0 || r[len - 1] > 0;
        inner->merge(p, r, len - 1);
        p[inner->size()] = flag ? 1 : 0;
    }
    dbg_datatype return_type() const override {
        dbg_datatype t = inner->return_type();
        t.nullable = 1;
        return t;
    }
    size_t result_width() const override { return inner->result_width(); }
};

static bool is_signed_int(int t) { return t == DBG_INT8 || t == DBG_INT16 || t == DBG_INT32 || t == DBG_INT64; }
static bool is_unsigned_int(int t) { return t == DBG_UINT8 || t == DBG_UINT16 || t == DBG_UINT32 || t == DBG_UINT64; }
static bool is_float(int t) { return t == DBG_FLOAT32 || t == DBG_FLOAT64; }

// AggregateFunctionFactory::get (FUN/aggregate_function_factory.rs:157-220).
static AggFn* make_fn(const dbg_agg_spec& s) {
    int t = s.arg.type;
    AggFn* base = nullptr;
    if (s.kind == DBG_AGG_COUNT) return new CountFn(t >= 0);  // never wrapped (returns_default_when_only_null)
    if (t < 0) throw UnsupportedError("aggregate needs an argument");
    if (s.kind == DBG_AGG_SUM) {
        // ResultTypeOfUnary::Sum (EXP/utils/arithmetics_type.rs)
        if (is_signed_int(t)) base = new SumNumFn<i64>(dbg_datatype{DBG_INT64, 0, 0, 0, 0});
        else if (is_unsigned_int(t)) base = new SumNumFn<u64>(dbg_datatype{DBG_UINT64, 0, 0, 0, 0});
        else if (is_float(t)) base = new SumNumFn<double>(dbg_datatype{DBG_FLOAT64, 0, 0, 0, 0});
        else if (t == DBG_DECIMAL128)
            base = new SumDecFn(s.arg.precision <= 18, dbg_datatype{DBG_DECIMAL128, 38, s.arg.scale, 0, 0});
    } else if (s.kind == DBG_AGG_AVG) {
        if (is_signed_int(t)) base = new AvgNumFn<i64>();
        else if (is_unsigned_int(t)) base = new AvgNumFn<u64>();
        else if (is_float(t)) base = new AvgNumFn<double>();
        else if (t == DBG_DECIMAL128) {
            int sc = std::max<int>(s.arg.scale, 4);
            base = new AvgDecFn(s.arg.precision > 18, sc - s.arg.scale, dbg_datatype{DBG_DECIMAL128, 38, (u8)sc, 0, 0});
        }
    } else if (s.kind == DBG_AGG_AVG_SQL) {
        if (is_signed_int(t)) base = new AvgNumFn<i64>();
        else if (is_unsigned_int(t)) base = new AvgNumFn<u64>();
        else if (is_float(t)) base = new AvgNumFn<double>();
        else if (t == DBG_DECIMAL128) {
            int sc = std::max<int>(s.arg.scale, std::min<int>(s.arg.scale + 6, 12));
            base = new SqlAvgDecFn(s.arg.precision <= 18, sc - s.arg.scale, dbg_datatype{DBG_DECIMAL128, 38, (u8)sc, 0, 0});
        }
    } else if (s.kind == DBG_AGG_MIN || s.kind == DBG_AGG_MAX) {
        bool mn = s.kind == DBG_AGG_MIN;
        dbg_datatype rt{t, s.arg.precision, s.arg.scale, 0, 0};
        if (is_signed_int(t) || t == DBG_DATE || t == DBG_TIMESTAMP) base = new MinMaxFn<i64>(mn, rt);
        else if (is_unsigned_int(t) || t == DBG_BOOLEAN) base = new MinMaxFn<u64>(mn, rt);  // bool: false < true
        else if (is_float(t)) base = new MinMaxFn<double>(mn, rt);
        else if (t == DBG_DECIMAL128) base = new MinMaxFn<i128>(mn, rt);
    }
    if (base == nullptr) throw UnsupportedError("unsupported aggregate/argument type");
    AggFn* f = base;
    if (s.arg.nullable) f = new NullUnaryAdaptor(f);  // AggregateFunctionCombinatorNull
    if (s.or_null) f = new OrNullAdaptor(f);
    return f;
}

// get_layout_offsets (EAGG/aggregate_function_state.rs:113-133).
static size_t layout_offsets(const std::vector<AggFn*>& fns, std::vector<size_t>& offs, size_t& align) {
    size_t total = 0;
    align = 8;
    for (auto* f : fns) {
        size_t a = f->align();
        total = (total + a - 1) / a * a;
        offs.push_back(total);
        total += f->size();
        align = std::max(align, a);
    }
    return (total + align - 1) / align * align;
}

// ------------------------------------------------------------------------------------------
// Row format + Payload (EAGG/payload.rs:41-432, EAGG/payload_row.rs:43-528)
// ------------------------------------------------------------------------------------------
static const size_t BATCH_SIZE = 2048;          // EAGG/mod.rs:48
static const double LOAD_FACTOR = 1.5;          // EAGG/mod.rs:49
static const size_t MAX_PAGE_SIZE = 256 * 1024; // EAGG/mod.rs:50

static size_t rowformat_size(const dbg_datatype& t) {  // payload_row.rs:43-65
    if (t.type == DBG_STRING) return 4 + 8;
    return fixed_width(t.type);
}

struct Layout {
    std::vector<dbg_datatype> group_types;
    std::vector<AggFn*> aggs;
    std::vector<size_t> validity_offsets, group_offsets, group_sizes, state_addr_offsets;
    size_t hash_offset = 0, state_offset = 0, tuple_size = 0, row_per_page = 0;
    size_t state_size = 0, state_align = 8;
    void init(const std::vector<dbg_datatype>& g, const std::vector<AggFn*>& a) {
        group_types = g;
        aggs = a;
        size_t ts = 0;
        for (auto& t : g) {
            if (t.nullable) { validity_offsets.push_back(ts); ts += 1; }
            else validity_offsets.push_back(0);
        }
        for (auto& t : g) {
            group_offsets.push_back(ts);
            size_t s = rowformat_size(t);
            group_sizes.push_back(s);
            ts += s;
        }
        hash_offset = ts;
        ts += 8;
        state_offset = ts;
        if (!a.empty()) ts += 8;
        tuple_size = ts;
        row_per_page = std::max<size_t>(1, std::min<size_t>(65535, MAX_PAGE_SIZE / ts));
        if (!a.empty()) state_size = layout_offsets(a, state_addr_offsets, state_align);
    }
};

struct Page {
    std::vector<u8> data;
    size_t rows = 0, capacity = 0;
};

template <class T>
static inline T rd(const u8* p) {
    T v;
    memcpy(&v, p, sizeof(T));
    return v;
}
template <class T>
static inline void wr(u8* p, T v) { memcpy(p, &v, sizeof(T)); }

struct Payload {
    const Layout* L;
    std::shared_ptr<Bump> arena;
    std::vector<std::unique_ptr<Page>> pages;
    size_t total_rows = 0, current_write_page = 0;
    Payload(const Layout* l, std::shared_ptr<Bump> a) : L(l), arena(std::move(a)) {}
    size_t memory_size() const { return total_rows * L->tuple_size; }
    Page* writable_page() {
        if (current_write_page == 0 || pages[current_write_page - 1]->rows == pages[current_write_page - 1]->capacity) {
            current_write_page += 1;
            if (current_write_page > pages.size()) {
                auto p = std::make_unique<Page>();
                p->capacity = L->row_per_page;
                p->data.resize(L->row_per_page * L->tuple_size);
                pages.push_back(std::move(p));
            }
        }
        return pages[current_write_page - 1].get();
    }
    // reserve_append_rows + append_rows (payload.rs:177-305)
    void reserve_append_rows(const size_t* sel, const u64* hashes, u8** address, size_t n,
                             const dbg_column* cols, u64 start) {
        Page* page = writable_page();
        for (size_t k = 0; k < n; ++k) {
            size_t idx = sel[k];
            address[idx] = page->data.data() + page->rows * L->tuple_size;
            page->rows += 1;
            if (page->rows == page->capacity) page = writable_page();
        }
        total_rows += n;
        size_t g = L->group_types.size();
        for (size_t k = 0; k < n; ++k) {
            size_t idx = sel[k];
            u8* row = address[idx];
            for (size_t c = 0; c < g; ++c) {
                const dbg_column& col = cols[c];
                u64 i = start + idx;
                if (L->group_types[c].nullable) row[L->validity_offsets[c]] = is_valid(col, i) ? 1 : 0;
                u8* dst = row + L->group_offsets[c];
                if (col.dt.type == DBG_STRING) {
                    u64 l = str_len(col, i);
                    u8* s = arena->alloc(l ? l : 1, 1);
                    memcpy(s, str_ptr(col, i), l);
                    wr<u32>(dst, (u32)l);
                    wr<u64>(dst + 4, (u64)(uintptr_t)s);
                } else if (col.dt.type == DBG_BOOLEAN) {
                    dst[0] = bool_val(col, i) ? 1 : 0;
                } else {
                    size_t w = fixed_width(col.dt.type);
                    memcpy(dst, (const u8*)col.data + i * w, w);
                }
            }
            wr<u64>(row + L->hash_offset, hashes[idx]);
            if (!L->aggs.empty()) {
                u8* place = arena->alloc(L->state_size, L->state_align);
                wr<u64>(row + L->state_offset, (u64)(uintptr_t)place);
                for (size_t a = 0; a < L->aggs.size(); ++a) L->aggs[a]->init_state(place + L->state_addr_offsets[a]);
            }
        }
    }
    void combine(Payload& other) {
        total_rows += other.total_rows;
        for (auto& p : other.pages) pages.push_back(std::move(p));
        other.pages.clear();
        other.total_rows = 0;
        current_write_page = pages.size();  // appends go to a fresh page after the moved ones
    }
    // copy_rows (payload.rs:323-354)
    void copy_rows(const size_t* sel, size_t n, u8* const* address) {
        Page* page = writable_page();
        for (size_t k = 0; k < n; ++k) {
            memcpy(page->data.data() + page->rows * L->tuple_size, address[sel[k]], L->tuple_size);
            page->rows += 1;
            if (page->rows == page->capacity) page = writable_page();
        }
        total_rows += n;
    }
};

// PartitionedPayload (EAGG/partitioned_payload.rs:30-275): partition = (hash & mask) >> (48 - r).
struct PartitionedPayload {
    const Layout* L;
    std::vector<std::unique_ptr<Payload>> payloads;
    std::vector<std::shared_ptr<Bump>> arenas;
    u64 partition_count, mask_v, shift_v;
    PartitionedPayload(const Layout* l, u64 pc, std::vector<std::shared_ptr<Bump>> ar) : L(l), arenas(std::move(ar)), partition_count(pc) {
        u64 rb = __builtin_ctzll(pc);
        shift_v = 48 - rb;
        mask_v = ((1ULL << rb) - 1) << shift_v;
        for (u64 i = 0; i < pc; ++i) payloads.emplace_back(new Payload(l, arenas[0]));
    }
    size_t len() const {
        size_t s = 0;
        for (auto& p : payloads) s += p->total_rows;
        return s;
    }
    size_t memory_size() const {
        size_t s = 0;
        for (auto& p : payloads) s += p->memory_size();
        return s;
    }
    void append_rows(const size_t* sel, const u64* hashes, u8** address, size_t n, const dbg_column* cols, u64 start) {
        if (payloads.size() == 1) {
            payloads[0]->reserve_append_rows(sel, hashes, address, n, cols, start);
            return;
        }
        std::vector<std::vector<size_t>> parts(partition_count);
        for (size_t k = 0; k < n; ++k) {
            size_t idx = sel[k];
            parts[(hashes[idx] & mask_v) >> shift_v].push_back(idx);
        }
        for (u64 p = 0; p < partition_count; ++p)
            if (!parts[p].empty()) payloads[p]->reserve_append_rows(parts[p].data(), hashes, address, parts[p].size(), cols, start);
    }
    // combine / combine_single / gather_flush (partitioned_payload.rs:145-244)
    void combine(PartitionedPayload& other) {
        if (other.partition_count == partition_count) {
            for (u64 i = 0; i < partition_count; ++i) payloads[i]->combine(*other.payloads[i]);
        } else {
            for (auto& p : other.payloads) combine_single(*p);
        }
        for (auto& a : other.arenas) arenas.push_back(a);
    }
    void combine_single(Payload& other) {
        if (other.total_rows == 0) return;
        if (partition_count == 1) {
            payloads[0]->combine(other);
            return;
        }
        std::vector<u8*> address(BATCH_SIZE);
        std::vector<std::vector<size_t>> parts(partition_count);
        for (auto& pg : other.pages) {
            for (size_t r0 = 0; r0 < pg->rows; r0 += BATCH_SIZE) {
                size_t rows = std::min(BATCH_SIZE, pg->rows - r0);
                for (auto& v : parts) v.clear();
                for (size_t k = 0; k < rows; ++k) {
                    address[k] = pg->data.data() + (r0 + k) * L->tuple_size;
                    u64 h = rd<u64>(address[k] + L->hash_offset);
                    parts[(h & mask_v) >> shift_v].push_back(k);
                }
                for (u64 p = 0; p < partition_count; ++p)
                    if (!parts[p].empty()) payloads[p]->copy_rows(parts[p].data(), parts[p].size(), address.data());
            }
        }
    }
    std::unique_ptr<PartitionedPayload> repartition(u64 new_count) {
        auto np = std::make_unique<PartitionedPayload>(L, new_count, arenas);
        np->combine(*this);
        return np;
    }
};

// Key equality of row `i` of the input columns against a stored row (row_match_columns,
// payload_row.rs:169-528): nulls equal nulls; floats compare as OrderedFloat; strings by len + bytes.
static bool row_match(const Layout* L, const dbg_column* cols, u64 i, const u8* row) {
    for (size_t c = 0; c < L->group_types.size(); ++c) {
        const dbg_column& col = cols[c];
        bool v1 = is_valid(col, i);
        bool v2 = L->group_types[c].nullable ? row[L->validity_offsets[c]] != 0 : true;
        if (!(v1 && v2)) {
            if (v1 != v2) return false;
            continue;
        }
        const u8* p = row + L->group_offsets[c];
        switch (col.dt.type) {
            case DBG_STRING: {
                u64 l = rd<u32>(p);
                if (l != str_len(col, i)) return false;
                const u8* s = (const u8*)(uintptr_t)rd<u64>(p + 4);
                if (l && memcmp(s, str_ptr(col, i), l) != 0) return false;
                break;
            }
            case DBG_BOOLEAN:
                if ((p[0] != 0) != bool_val(col, i)) return false;
                break;
            case DBG_FLOAT32: {
                float a = rd<float>(p), b = val<float>(col, i);
                if (!((std::isnan(a) && std::isnan(b)) || a == b)) return false;
                break;
            }
            case DBG_FLOAT64: {
                double a = rd<double>(p), b = val<double>(col, i);
                if (!((std::isnan(a) && std::isnan(b)) || a == b)) return false;
                break;
            }
            default: {
                size_t w = fixed_width(col.dt.type);
                if (memcmp(p, (const u8*)col.data + i * w, w) != 0) return false;
            }
        }
    }
    return true;
}

// HashTableConfig (EAGG/mod.rs:59-132)
struct Config {
    std::shared_ptr<std::atomic<u64>> current_max_radix_bits;
    u64 initial_radix_bits = 3, max_radix_bits = 7, repartition_radix_bits_incr = 2;
    double block_fill_factor = 1.8;
    bool partial_agg = false;
    size_t max_partial_capacity = 131072;
    Config() : current_max_radix_bits(std::make_shared<std::atomic<u64>>(3)) {}
    Config with_initial_radix_bits(u64 r) const {
        Config c = *this;
        c.initial_radix_bits = r;
        c.current_max_radix_bits = std::make_shared<std::atomic<u64>>(r);
        return c;
    }
    Config with_partial(bool p, size_t active_threads) const {  // mod.rs:92-104
        Config c = *this;
        c.partial_agg = p;
        const size_t L1 = 32768 / 2, L2 = 1048576 / 2, L3 = 1572864 / 2;
        size_t total_shared = active_threads * L3;
        size_t per_thread = L1 + L2 + total_shared / active_threads;
        size_t per_entry = (size_t)(8.0 * LOAD_FACTOR);
        size_t cap = per_thread / per_entry;
        size_t p2 = 1;
        while (p2 < cap) p2 <<= 1;
        c.max_partial_capacity = p2;
        return c;
    }
};

static const u64 SALT_MASK = 0xFFFF000000000000ULL, POINTER_MASK = 0x0000FFFFFFFFFFFFULL;
static inline u64 get_salt(u64 e) { return e | POINTER_MASK; }  // aggregate_hashtable.rs:605-636

// AggregateHashTable (EAGG/aggregate_hashtable.rs:47-589).
struct AggregateHashTable {
    const Layout* L;
    Config config;
    u64 current_radix_bits;
    std::vector<u64> entries;
    size_t count = 0, capacity;
    std::unique_ptr<PartitionedPayload> payload;
    // ProbeState (EAGG/probe_state.rs)
    std::vector<u64> group_hashes = std::vector<u64>(BATCH_SIZE);
    std::vector<u8*> addresses = std::vector<u8*>(BATCH_SIZE);
    std::vector<u8*> state_places = std::vector<u8*>(BATCH_SIZE);
    std::vector<size_t> no_match = std::vector<size_t>(BATCH_SIZE), empty_v = std::vector<size_t>(BATCH_SIZE),
                        compare_v = std::vector<size_t>(BATCH_SIZE);

    AggregateHashTable(const Layout* l, Config c, size_t cap)
        : L(l), config(c), current_radix_bits(c.initial_radix_bits), entries(cap, 0), capacity(cap) {
        payload.reset(new PartitionedPayload(l, 1ULL << c.initial_radix_bits, {std::make_shared<Bump>()}));
    }
    static size_t initial_capacity() { return 8192 * 4; }
    static size_t get_capacity_for_count(size_t count) {
        size_t c = (size_t)((double)std::max(count, initial_capacity()) * LOAD_FACTOR);
        size_t p2 = 1;
        while (p2 < c) p2 <<= 1;
        return p2;
    }
    size_t resize_threshold() const { return (size_t)((double)capacity / LOAD_FACTOR); }

    // add_groups (:128-167): 2048-row chunks
    void add_groups(const dbg_column* groups, const dbg_column* const* args, u64 rows) {
        for (u64 s = 0; s < rows; s += BATCH_SIZE) add_groups_inner(groups, args, s, std::min<u64>(BATCH_SIZE, rows - s));
    }
    // add_groups with agg_states (AggregateMeta::Serialized: SerializedPayload::convert_to_aggregate_table,
    // AGG/aggregate_meta.rs:57-101): the same probe, then AggregateFunction::batch_merge of each
    // Binary state column (EAGG/aggregate_function.rs:96-103) instead of accumulate_keys.
    void add_groups_merge(const dbg_column* groups, const dbg_column* states, u64 rows) {
        for (u64 s = 0; s < rows; s += BATCH_SIZE) add_groups_inner(groups, nullptr, s, std::min<u64>(BATCH_SIZE, rows - s), states);
    }
    void add_groups_inner(const dbg_column* groups, const dbg_column* const* args, u64 start, u64 n,
                          const dbg_column* states = nullptr) {
        group_hash_columns(groups, (int)L->group_types.size(), start, n, group_hashes.data());
        probe_and_create(groups, start, n);
        if (!L->aggs.empty()) {
            for (u64 k = 0; k < n; ++k) state_places[k] = (u8*)(uintptr_t)rd<u64>(addresses[k] + L->state_offset);
            for (size_t a = 0; a < L->aggs.size(); ++a) {
                if (states) {
                    for (u64 k = 0; k < n; ++k)
                        L->aggs[a]->merge(state_places[k] + L->state_addr_offsets[a], str_ptr(states[a], start + k),
                                          str_len(states[a], start + k));
                } else {
                    L->aggs[a]->accumulate_keys(state_places.data(), L->state_addr_offsets[a], args[a], start, n);
                }
            }
        }
        if (config.partial_agg) {  // :225-239
            if (count + BATCH_SIZE > resize_threshold() && capacity >= config.max_partial_capacity) {
                clear_ht();
                count = 0;
            }
            if (maybe_repartition()) {
                clear_ht();
                count = 0;
            }
        }
    }
    // probe_and_create (:244-366)
    size_t probe_and_create(const dbg_column* groups, u64 start, u64 n) {
        if (n + count > resize_threshold()) resize(capacity * 2);
        size_t new_groups = 0, remaining = n;
        u64 mask = capacity - 1;
        std::vector<u64> offs(n), salts(n);
        for (u64 i = 0; i < n; ++i) {
            offs[i] = group_hashes[i] & mask;
            salts[i] = get_salt(group_hashes[i]);
            no_match[i] = i;
        }
        while (remaining > 0) {
            size_t new_count = 0, cmp_count = 0, nm_count = 0;
            for (size_t r = 0; r < remaining; ++r) {
                size_t idx = no_match[r];
                u64& off = offs[idx];
                for (;;) {
                    u64& e = entries[off];
                    if (e != 0) {
                        if (get_salt(e) == salts[idx]) {
                            compare_v[cmp_count++] = idx;
                            break;
                        }
                        off += 1;
                        if (off >= capacity) off = 0;
                    } else {
                        e = salts[idx];  // set_salt
                        empty_v[new_count++] = idx;
                        break;
                    }
                }
            }
            if (new_count) {
                new_groups += new_count;
                payload->append_rows(empty_v.data(), group_hashes.data(), addresses.data(), new_count, groups, start);
                for (size_t k = 0; k < new_count; ++k) {
                    size_t idx = empty_v[k];
                    entries[offs[idx]] &= ((u64)(uintptr_t)addresses[idx]) | SALT_MASK;  // set_pointer
                }
            }
            for (size_t k = 0; k < cmp_count; ++k) {
                size_t idx = compare_v[k];
                addresses[idx] = (u8*)(uintptr_t)(entries[offs[idx]] & POINTER_MASK);
                if (!row_match(L, groups, start + idx, addresses[idx])) no_match[nm_count++] = idx;
            }
            for (size_t k = 0; k < nm_count; ++k) {
                u64& off = offs[no_match[k]];
                off += 1;
                if (off >= capacity) off = 0;
            }
            remaining = nm_count;
        }
        count += new_groups;
        return new_groups;
    }
    // resize (:511-561)
    void resize(size_t new_cap) {
        if (config.partial_agg) {
            if (capacity == config.max_partial_capacity) return;
            entries.assign(new_cap, 0);
            count = 0;
            capacity = new_cap;
            return;
        }
        count = 0;
        u64 mask = new_cap - 1;
        std::vector<u64> ne(new_cap, 0);
        for (auto& p : payload->payloads)
            for (auto& pg : p->pages)
                for (size_t r = 0; r < pg->rows; ++r) {
                    u8* row = pg->data.data() + r * L->tuple_size;
                    u64 h = rd<u64>(row + L->hash_offset);
                    u64 s = h & mask;
                    while (ne[s] != 0) {
                        s += 1;
                        if (s >= new_cap) s = 0;
                    }
                    ne[s] = get_salt(h);
                    ne[s] &= ((u64)(uintptr_t)row) | SALT_MASK;
                    count += 1;
                }
        entries.swap(ne);
        capacity = new_cap;
    }
    void clear_ht() { std::fill(entries.begin(), entries.end(), 0); }
    // maybe_repartition (:453-503)
    bool maybe_repartition() {
        if (!config.partial_agg || current_radix_bits == config.max_radix_bits) return false;
        size_t bpp = payload->memory_size() / payload->partition_count;
        u64 nrb = current_radix_bits;
        if (bpp > MAX_PAGE_SIZE * (size_t)config.block_fill_factor) nrb += config.repartition_radix_bits_incr;
        for (;;) {
            u64 cur = config.current_max_radix_bits->load();
            if (cur < nrb && !config.current_max_radix_bits->compare_exchange_strong(cur, nrb)) continue;
            break;
        }
        u64 cmax = config.current_max_radix_bits->load();
        if (cmax > current_radix_bits) {
            current_radix_bits = cmax;
            payload = payload->repartition(1ULL << cmax);
            return true;
        }
        return false;
    }
    // combine_payload (:383-425): flush 2048 rows at a time -> probe -> merge_states
    void combine_payload(Payload& p) {
        std::vector<OwnedColumn> fc(L->group_types.size());
        std::vector<dbg_column> views(L->group_types.size());
        std::vector<u8*> rhs(BATCH_SIZE);
        for (auto& pg : p.pages) {
            for (size_t r0 = 0; r0 < pg->rows; r0 += BATCH_SIZE) {
                size_t rows = std::min(BATCH_SIZE, pg->rows - r0);
                // Payload::flush + flush_column (payload_flush.rs:182-351)
                for (size_t c = 0; c < fc.size(); ++c) {
                    fc[c].clear();
                    fc[c].dt = L->group_types[c];
                }
                for (size_t k = 0; k < rows; ++k) {
                    const u8* row = pg->data.data() + (r0 + k) * L->tuple_size;
                    group_hashes[k] = rd<u64>(row + L->hash_offset);
                    if (!L->aggs.empty()) rhs[k] = (u8*)(uintptr_t)rd<u64>(row + L->state_offset);
                    for (size_t c = 0; c < fc.size(); ++c) {
                        const u8* src = row + L->group_offsets[c];
                        OwnedColumn& o = fc[c];
                        if (o.dt.type == DBG_STRING) {
                            u64 l = rd<u32>(src);
                            const u8* s = (const u8*)(uintptr_t)rd<u64>(src + 4);
                            o.data.insert(o.data.end(), s, s + l);
                            o.offsets.push_back(o.data.size());
                        } else {
                            size_t w = o.dt.type == DBG_BOOLEAN ? 1 : fixed_width(o.dt.type);
                            o.data.insert(o.data.end(), src, src + w);
                        }
                        o.valid.push_back(o.dt.nullable ? row[L->validity_offsets[c]] : 1);
                        o.rows++;
                    }
                }
                for (size_t c = 0; c < fc.size(); ++c) views[c] = fc[c].view();
                probe_and_create(views.data(), 0, rows);
                if (!L->aggs.empty()) {
                    for (size_t k = 0; k < rows; ++k) state_places[k] = (u8*)(uintptr_t)rd<u64>(addresses[k] + L->state_offset);
                    for (size_t a = 0; a < L->aggs.size(); ++a) {
                        size_t off = L->state_addr_offsets[a];
                        for (size_t k = 0; k < rows; ++k) L->aggs[a]->merge_states(state_places[k] + off, rhs[k] + off);
                    }
                }
            }
        }
    }
    // merge_result (:427-451) + flush of group columns: append every group to the outputs.
    // ser: the states as Binary columns (payload_flush.rs:129-164 aggregate_flush) instead of results
    void merge_result(std::vector<OwnedColumn>& keys, std::vector<OwnedColumn>& results, bool ser = false) {
        for (auto& p : payload->payloads)
            for (auto& pg : p->pages)
                for (size_t r = 0; r < pg->rows; ++r) {
                    const u8* row = pg->data.data() + r * L->tuple_size;
                    for (size_t c = 0; c < keys.size(); ++c) {
                        OwnedColumn& o = keys[c];
                        const u8* src = row + L->group_offsets[c];
                        if (o.dt.type == DBG_STRING) {
                            u64 l = rd<u32>(src);
                            const u8* s = (const u8*)(uintptr_t)rd<u64>(src + 4);
                            o.data.insert(o.data.end(), s, s + l);
                            o.offsets.push_back(o.data.size());
                        } else {
                            size_t w = o.dt.type == DBG_BOOLEAN ? 1 : fixed_width(o.dt.type);
                            o.data.insert(o.data.end(), src, src + w);
                        }
                        o.valid.push_back(o.dt.nullable ? row[L->validity_offsets[c]] : 1);
                        o.rows++;
                    }
                    if (!L->aggs.empty()) {
                        u8* place = (u8*)(uintptr_t)rd<u64>(row + L->state_offset);
                        for (size_t a = 0; a < L->aggs.size(); ++a) {
                            if (ser) {
                                OwnedColumn& o = results[a];
                                L->aggs[a]->serialize(place + L->state_addr_offsets[a], o.data);
                                o.offsets.push_back(o.data.size());
                                o.valid.push_back(1);
                                o.rows++;
                                continue;
                            }
                            Builder b{&results[a]};
                            L->aggs[a]->merge_result(place + L->state_addr_offsets[a], b);
                        }
                    }
                }
    }
};

// ------------------------------------------------------------------------------------------
// Filter (EXP/filter/*): predicate program -> selection vector -> take
// ------------------------------------------------------------------------------------------
enum Tri : int8_t { T_FALSE = 0, T_TRUE = 1, T_NULL = 2 };

static int cmp_bytes(const u8* a, u64 la, const u8* b, u64 lb) {
    int r = memcmp(a, b, std::min(la, lb));
    if (r != 0) return r < 0 ? -1 : 1;
    return la < lb ? -1 : (la > lb ? 1 : 0);
}
template <class T>
static int cmp3(T a, T b) { return a < b ? -1 : (a > b ? 1 : 0); }
static int cmp_f64(double a, double b) {  // OrderedFloat total order
    bool an = std::isnan(a), bn = std::isnan(b);
    if (an || bn) return an == bn ? 0 : (an ? 1 : -1);
    return cmp3(a, b);
}
static bool apply_cmp(int c, int o) {
    switch (c) {
        case DBG_CMP_EQ: return o == 0;
        case DBG_CMP_NE: return o != 0;
        case DBG_CMP_LT: return o < 0;
        case DBG_CMP_LE: return o <= 0;
        case DBG_CMP_GT: return o > 0;
        case DBG_CMP_GE: return o >= 0;
    }
    return false;
}
static int cmp_const(const dbg_column& c, u64 i, const dbg_pred_node& n) {
    int t = c.dt.type;
    if (is_signed_int(t) || t == DBG_DATE || t == DBG_TIMESTAMP) return cmp3<i64>(arg_as<i64>(c, i), n.i64);
    if (is_unsigned_int(t)) return cmp3<u64>(arg_as<u64>(c, i), (u64)n.i64);
    if (is_float(t)) return cmp_f64(arg_as<double>(c, i), n.f64);
    if (t == DBG_DECIMAL128) return cmp3<i128>(val<i128>(c, i), (i128)(((u128)(u64)n.i128_hi << 64) | n.i128_lo));
    if (t == DBG_BOOLEAN) return cmp3<i64>(bool_val(c, i) ? 1 : 0, n.i64);
    if (t == DBG_STRING) return cmp_bytes(str_ptr(c, i), str_len(c, i), n.str, n.str_len);
    throw UnsupportedError("filter: type");
}
static int cmp_cols(const dbg_column& a, const dbg_column& b, u64 i) {
    int t = a.dt.type;
    if (is_signed_int(t) || t == DBG_DATE || t == DBG_TIMESTAMP) return cmp3<i64>(arg_as<i64>(a, i), arg_as<i64>(b, i));
    if (is_unsigned_int(t)) return cmp3<u64>(arg_as<u64>(a, i), arg_as<u64>(b, i));
    if (is_float(t)) return cmp_f64(arg_as<double>(a, i), arg_as<double>(b, i));
    if (t == DBG_DECIMAL128) return cmp3<i128>(val<i128>(a, i), val<i128>(b, i));
    if (t == DBG_BOOLEAN) return cmp3<int>(bool_val(a, i), bool_val(b, i));
    if (t == DBG_STRING) return cmp_bytes(str_ptr(a, i), str_len(a, i), str_ptr(b, i), str_len(b, i));
    throw UnsupportedError("filter: type");
}
static bool eval_pred(const dbg_filter& f, u64 i) {
    Tri st[64];
    int sp = 0;
    for (int k = 0; k < f.n_nodes; ++k) {
        const dbg_pred_node& n = f.nodes[k];
        switch (n.op) {
            case DBG_PRED_TRUE: st[sp++] = T_TRUE; break;
            case DBG_PRED_CMP_CONST: {
                const dbg_column& c = f.cols[n.col];
                st[sp++] = !is_valid(c, i) ? T_NULL : (apply_cmp(n.cmp, cmp_const(c, i, n)) ? T_TRUE : T_FALSE);
                break;
            }
            case DBG_PRED_CMP_COLS: {
                const dbg_column& a = f.cols[n.col];
                const dbg_column& b = f.cols[n.col2];
                st[sp++] = (!is_valid(a, i) || !is_valid(b, i)) ? T_NULL : (apply_cmp(n.cmp, cmp_cols(a, b, i)) ? T_TRUE : T_FALSE);
                break;
            }
            case DBG_PRED_IS_NULL: st[sp++] = is_valid(f.cols[n.col], i) ? T_FALSE : T_TRUE; break;
            case DBG_PRED_IS_NOT_NULL: st[sp++] = is_valid(f.cols[n.col], i) ? T_TRUE : T_FALSE; break;
            case DBG_PRED_NOT: st[sp - 1] = st[sp - 1] == T_NULL ? T_NULL : (st[sp - 1] == T_TRUE ? T_FALSE : T_TRUE); break;
            case DBG_PRED_AND: {
                Tri b = st[--sp], a = st[--sp];
                st[sp++] = (a == T_FALSE || b == T_FALSE) ? T_FALSE : ((a == T_TRUE && b == T_TRUE) ? T_TRUE : T_NULL);
                break;
            }
            case DBG_PRED_OR: {
                Tri b = st[--sp], a = st[--sp];
                st[sp++] = (a == T_TRUE || b == T_TRUE) ? T_TRUE : ((a == T_FALSE && b == T_FALSE) ? T_FALSE : T_NULL);
                break;
            }
        }
    }
    return sp > 0 && st[sp - 1] == T_TRUE;
}

// ------------------------------------------------------------------------------------------
// Pipeline: TransformFilter -> TransformPartialAggregate x T -> NewTransformPartitionBucket ->
// TransformFinalAggregate x T (builder_aggregate.rs:96-284)
// ------------------------------------------------------------------------------------------
struct Result {
    std::vector<OwnedColumn> keys, aggs;
    u64 rows = 0;
};

struct PipelineSpec {
    std::vector<dbg_column> keys;
    std::vector<dbg_column> args;  // one per agg
    std::vector<dbg_agg_spec> specs;
    const dbg_filter* filter = nullptr;
    u64 rows = 0;
    int threads = 1;
    size_t block_size = 65536;  // max_block_size (settings_default.rs:131)
    bool serialize = false;     // emit the final states as Binary columns (AggregateMeta::Serialized)
};

static void run_pipeline(const PipelineSpec& ps, Result& out) {
    std::vector<std::unique_ptr<AggFn>> owned;
    std::vector<AggFn*> fns;
    for (auto& s : ps.specs) {
        owned.emplace_back(make_fn(s));
        fns.push_back(owned.back().get());
    }
    std::vector<dbg_datatype> gtypes;
    for (auto& k : ps.keys) gtypes.push_back(k.dt);
    Layout L;
    L.init(gtypes, fns);
    int T = std::max(1, ps.threads);
    Config base = Config().with_partial(true, T);
    std::vector<std::unique_ptr<AggregateHashTable>> tables(T);
    std::vector<std::string> errs(T);
    std::vector<int> err_code(T, 0);

    // ---- partial stage (AGG/transform_aggregate_partial.rs:235-327), one table per thread
    auto partial = [&](int t) {
        try {
            tables[t].reset(new AggregateHashTable(&L, base, AggregateHashTable::initial_capacity()));
            u64 r0 = ps.rows * t / T, r1 = ps.rows * (t + 1) / T;
            std::vector<OwnedColumn> fk(ps.keys.size()), fa(ps.args.size());
            std::vector<dbg_column> vk(ps.keys.size()), va(ps.args.size());
            std::vector<const dbg_column*> argp(ps.args.size());
            std::vector<u64> sel;
            for (u64 b = r0; b < r1; b += ps.block_size) {
                u64 n = std::min<u64>(ps.block_size, r1 - b);
                if (ps.filter) {  // FilterExecutor::filter -> take (filter_executor.rs:73-128)
                    sel.clear();
                    for (u64 i = b; i < b + n; ++i)
                        if (eval_pred(*ps.filter, i)) sel.push_back(i);
                    if (sel.empty()) continue;
                    for (size_t c = 0; c < ps.keys.size(); ++c) {
                        fk[c].clear();
                        fk[c].dt = ps.keys[c].dt;
                        for (u64 i : sel) append_cell(fk[c], ps.keys[c], i);
                        vk[c] = fk[c].view();
                    }
                    for (size_t c = 0; c < ps.args.size(); ++c) {
                        if (ps.args[c].dt.type < 0) { va[c] = ps.args[c]; argp[c] = &va[c]; continue; }
                        fa[c].clear();
                        fa[c].dt = ps.args[c].dt;
                        for (u64 i : sel) append_cell(fa[c], ps.args[c], i);
                        va[c] = fa[c].view();
                        argp[c] = &va[c];
                    }
                    tables[t]->add_groups(vk.data(), argp.data(), sel.size());
                } else {
                    // zero-copy slices: rows [b, b+n) addressed through start offsets
                    for (size_t c = 0; c < ps.keys.size(); ++c) {
                        vk[c] = ps.keys[c];
                        const dbg_column& k = ps.keys[c];
                        size_t w = k.dt.type == DBG_STRING ? 0 : fixed_width(k.dt.type);
                        if (k.dt.type == DBG_STRING) vk[c].offsets = k.offsets + b;
                        else if (k.dt.type == DBG_BOOLEAN) vk[c].data_offset = k.data_offset + b;
                        else vk[c].data = (const u8*)k.data + b * w;
                        vk[c].validity_offset = k.validity_offset + b;
                    }
                    for (size_t c = 0; c < ps.args.size(); ++c) {
                        va[c] = ps.args[c];
                        const dbg_column& k = ps.args[c];
                        if (k.dt.type >= 0) {
                            if (k.dt.type == DBG_STRING) va[c].offsets = k.offsets + b;
                            else if (k.dt.type == DBG_BOOLEAN) va[c].data_offset = k.data_offset + b;
                            else va[c].data = (const u8*)k.data + b * fixed_width(k.dt.type);
                            va[c].validity_offset = k.validity_offset + b;
                        }
                        argp[c] = &va[c];
                    }
                    tables[t]->add_groups(vk.data(), argp.data(), n);
                }
            }
        } catch (OverflowError& e) {
            errs[t] = e.what();
            err_code[t] = DBG_ERR_OVERFLOW;
        } catch (std::exception& e) {
            errs[t] = e.what();
            err_code[t] = DBG_ERR_UNSUPPORTED;
        }
    };
    {
        std::vector<std::thread> th;
        for (int t = 1; t < T; ++t) th.emplace_back(partial, t);
        partial(0);
        for (auto& x : th) x.join();
    }
    for (int t = 0; t < T; ++t)
        if (err_code[t]) {
            if (err_code[t] == DBG_ERR_OVERFLOW) throw OverflowError(errs[t]);
            throw UnsupportedError(errs[t]);
        }

    // ---- partition bucket (AGG/new_transform_partition_bucket.rs:389-576): align to max partitions
    u64 maxp = 1;
    for (auto& t : tables) maxp = std::max<u64>(maxp, t->payload->partition_count);
    for (auto& t : tables)
        if (t->payload->partition_count != maxp) t->payload = t->payload->repartition(maxp);

    // ---- final stage per bucket (AGG/transform_aggregate_final.rs:71-156)
    std::vector<Result> per_bucket(maxp);
    std::atomic<u64> next{0};
    std::vector<std::string> ferrs(T);
    std::vector<int> fcode(T, 0);
    auto final_stage = [&](int t) {
        try {
            for (;;) {
                u64 b = next.fetch_add(1);
                if (b >= maxp) break;
                std::unique_ptr<AggregateHashTable> ht;
                for (auto& tb : tables) {
                    Payload& p = *tb->payload->payloads[b];
                    if (!ht) {
                        size_t cap = AggregateHashTable::get_capacity_for_count(p.total_rows);
                        ht.reset(new AggregateHashTable(&L, Config().with_initial_radix_bits(0), cap));
                    }
                    ht->combine_payload(p);
                }
                Result& r = per_bucket[b];
                r.keys.resize(ps.keys.size());
                r.aggs.resize(fns.size());
                for (size_t c = 0; c < ps.keys.size(); ++c) { r.keys[c].clear(); r.keys[c].dt = ps.keys[c].dt; }
                for (size_t a = 0; a < fns.size(); ++a) {
                    r.aggs[a].clear();
                    r.aggs[a].dt = ps.serialize ? dbg_datatype{DBG_STRING, 0, 0, 0, 0} : fns[a]->return_type();
                }
                ht->merge_result(r.keys, r.aggs, ps.serialize);
            }
        } catch (OverflowError& e) {
            ferrs[t] = e.what();
            fcode[t] = DBG_ERR_OVERFLOW;
        } catch (std::exception& e) {
            ferrs[t] = e.what();
            fcode[t] = DBG_ERR_UNSUPPORTED;
        }
    };
    {
        std::vector<std::thread> th;
        for (int t = 1; t < T; ++t) th.emplace_back(final_stage, t);
        final_stage(0);
        for (auto& x : th) x.join();
    }
    for (int t = 0; t < T; ++t)
        if (fcode[t]) {
            if (fcode[t] == DBG_ERR_OVERFLOW) throw OverflowError(ferrs[t]);
            throw UnsupportedError(ferrs[t]);
        }
    // concat buckets in order
    out.keys.assign(ps.keys.size(), OwnedColumn());
    out.aggs.assign(fns.size(), OwnedColumn());
    for (size_t c = 0; c < ps.keys.size(); ++c) { out.keys[c].clear(); out.keys[c].dt = ps.keys[c].dt; }
    for (size_t a = 0; a < fns.size(); ++a) {
        out.aggs[a].clear();
        out.aggs[a].dt = ps.serialize ? dbg_datatype{DBG_STRING, 0, 0, 0, 0} : fns[a]->return_type();
    }
    auto cat = [](OwnedColumn& d, OwnedColumn& s) {
        if (d.dt.type == DBG_STRING) {
            u64 base = d.data.size();
            for (size_t i = 1; i < s.offsets.size(); ++i) d.offsets.push_back(base + s.offsets[i]);
        }
        d.data.insert(d.data.end(), s.data.begin(), s.data.end());
        d.valid.insert(d.valid.end(), s.valid.begin(), s.valid.end());
        d.rows += s.rows;
    };
    for (auto& r : per_bucket) {
        for (size_t c = 0; c < r.keys.size(); ++c) cat(out.keys[c], r.keys[c]);
        for (size_t a = 0; a < r.aggs.size(); ++a) cat(out.aggs[a], r.aggs[a]);
    }
    out.rows = out.keys.empty() ? (out.aggs.empty() ? 0 : out.aggs[0].rows) : out.keys[0].rows;
}

// TransformFinalAggregate over AggregateMeta::Serialized blocks [states..., groups...]
// (AGG/transform_aggregate_final.rs:71-156 -> SerializedPayload::convert_to_aggregate_table,
// AGG/aggregate_meta.rs:57-101): one final table re-inserts every block's groups, merging the
// Binary states (batch_merge), then merge_result (or serialize again).
static void run_merge_serialized(const std::vector<dbg_column>& keys, const std::vector<dbg_column>& states,
                                 const std::vector<dbg_agg_spec>& specs, u64 rows, bool ser, Result& out) {
    std::vector<std::unique_ptr<AggFn>> owned;
    std::vector<AggFn*> fns;
    for (auto& s : specs) {
        owned.emplace_back(make_fn(s));
        fns.push_back(owned.back().get());
    }
    std::vector<dbg_datatype> gtypes;
    for (auto& k : keys) gtypes.push_back(k.dt);
    Layout L;
    L.init(gtypes, fns);
    AggregateHashTable ht(&L, Config().with_initial_radix_bits(0), AggregateHashTable::get_capacity_for_count(rows));
    ht.add_groups_merge(keys.data(), states.data(), rows);
    out.keys.assign(keys.size(), OwnedColumn());
    out.aggs.assign(fns.size(), OwnedColumn());
    for (size_t c = 0; c < keys.size(); ++c) { out.keys[c].clear(); out.keys[c].dt = keys[c].dt; }
    for (size_t a = 0; a < fns.size(); ++a) {
        out.aggs[a].clear();
        out.aggs[a].dt = ser ? dbg_datatype{DBG_STRING, 0, 0, 0, 0} : fns[a]->return_type();
    }
    ht.merge_result(out.keys, out.aggs, ser);
    out.rows = out.keys.empty() ? 0 : out.keys[0].rows;
}

}  // namespace orc

// ============================================================================================
// C API used by tests / bench (ctypes)
// ============================================================================================
using namespace orc;

struct orc_result {
    Result r;
};

// ------------------------------------------------------------------------------------------
// Legacy HashMethod keys + FastHash (enable_experimental_aggregate_hashtable = 0)
// choose_hash_method_with_types (EXP/kernels/group_by.rs:48-97); FixedKeys packing build_keys_vec /
// build / fixed_hash (EXP/kernels/group_by_hash/method_fixed_keys.rs:74-100, 366-470); FastHash
// (HT/traits.rs:172-330, sse4.2 build: _mm_crc32_u64 chained from u64::MAX); [u8] hash with the
// 1..8-byte little-endian tail (read_le, HT/utils.rs:94-102), an empty slice -> u64::MAX.
// ------------------------------------------------------------------------------------------
// CRC32C bytewise (reflected Castagnoli 0x82F63B78), bit by bit: the SSE4.2 crc32 instruction
// consumes its 8 bytes in little-endian order, the same as eight single-byte steps.
static u32 crc32c_byte(u32 crc, u8 b) {
    crc ^= b;
    for (int k = 0; k < 8; ++k) crc = (crc >> 1) ^ (0x82F63B78u & (0u - (crc & 1u)));
    return crc;
}
static u32 crc32c_u64_ref(u32 crc, u64 v) {  // _mm_crc32_u64(crc, v) (low 32 bits)
    for (int b = 0; b < 8; ++b) crc = crc32c_byte(crc, (u8)(v >> (8 * b)));
    return crc;
}

static void legacy_group_hash(const dbg_column* cols, int n, u64 rows, u64* out) {
    if (n == 1 && cols[0].dt.type == DBG_STRING && !cols[0].dt.nullable) {  // HashMethodSingleBinary
        for (u64 i = 0; i < rows; ++i) {
            const u8* p = str_ptr(cols[0], i);
            const u64 len = str_len(cols[0], i);
            u64 value = ~0ULL;  // u64::MAX; each crc step leaves a 32-bit value
            for (u64 o = 0; o < len; o += 8) {
                u64 w = 0;
                const u64 k = std::min<u64>(8, len - o);
                for (u64 b = 0; b < k; ++b) w |= (u64)p[o + b] << (8 * b);
                value = crc32c_u64_ref((u32)value, w);
            }
            out[i] = value;
        }
        return;
    }
    u64 len = 0;
    bool serializer = false;
    for (int j = 0; j < n; ++j) {
        const int t = cols[j].dt.type;
        if (t == DBG_STRING || t == DBG_BOOLEAN) serializer = true;
        len += fixed_width(t) + (cols[j].dt.nullable ? 1 : 0);
    }
    if (serializer || len > 32) {
        // HashMethodSerializer (EXP/kernels/group_by_hash/method_serializer.rs:39-70): the key is
        // serialize_column_binary of every column in order (utils.rs:64-121) — a nullable column's
        // validity byte, then for a valid row the value (numbers / dates in their width, Decimal128
        // 16 bytes, Boolean one byte, String u64 length + bytes) — hashed as [u8]
        std::vector<u8> key;
        for (u64 i = 0; i < rows; ++i) {
            key.clear();
            for (int j = 0; j < n; ++j) {
                const dbg_column& c = cols[j];
                const bool v = is_valid(c, i);
                if (c.dt.nullable) key.push_back(v ? 1 : 0);
                if (!v) continue;
                if (c.dt.type == DBG_STRING) {
                    const u64 sl = str_len(c, i);
                    for (int b = 0; b < 8; ++b) key.push_back((u8)(sl >> (8 * b)));
                    const u8* p = str_ptr(c, i);
                    key.insert(key.end(), p, p + sl);
                } else if (c.dt.type == DBG_BOOLEAN) {
                    key.push_back(bool_val(c, i) ? 1 : 0);
                } else {
                    const u64 w = fixed_width(c.dt.type);
                    const u8* p = (const u8*)c.data + i * w;
                    key.insert(key.end(), p, p + w);
                }
            }
            u64 value = ~0ULL;
            for (u64 o = 0; o < key.size(); o += 8) {
                u64 w = 0;
                const u64 k = std::min<u64>(8, key.size() - o);
                for (u64 b = 0; b < k; ++b) w |= (u64)key[o + b] << (8 * b);
                value = crc32c_u64_ref((u32)value, w);
            }
            out[i] = value;
        }
        return;
    }
    const u64 step = len == 1 ? 1 : len == 2 ? 2 : len <= 4 ? 4 : len <= 8 ? 8 : len <= 16 ? 16 : 32;
    // build_keys_vec: sort_by (stable) widest first; null bytes start after every value byte
    std::vector<int> order(n);
    for (int j = 0; j < n; ++j) order[j] = j;
    std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return fixed_width(cols[a].dt.type) > fixed_width(cols[b].dt.type); });
    u64 values = 0;
    for (int j = 0; j < n; ++j) values += fixed_width(cols[j].dt.type);
    std::vector<u8> key(32);
    for (u64 i = 0; i < rows; ++i) {
        std::fill(key.begin(), key.end(), 0);
        u64 off = 0, noff = values;
        for (int j = 0; j < n; ++j) {
            const dbg_column& c = cols[order[j]];
            const u64 w = fixed_width(c.dt.type);
            const bool nul = c.dt.nullable;
            if (nul && !is_valid(c, i)) key[noff] = 1;
            else memcpy(&key[off], (const u8*)c.data + i * w, w);
            off += w;
            if (nul) noff++;
        }
        u32 crc = 0xFFFFFFFFu;
        for (u64 wd = 0; wd < (step <= 8 ? 1 : step / 8); ++wd) {
            u64 v;
            memcpy(&v, &key[wd * 8], 8);
            crc = crc32c_u64_ref(crc, v);
        }
        out[i] = crc;
    }
}

extern "C" {

const char* orc_last_error(void) { return g_err.c_str(); }

int orc_legacy_group_hash(const dbg_column* cols, int n, uint64_t rows, uint64_t* out) {
    try {
        legacy_group_hash(cols, n, rows, out);
        return DBG_OK;
    } catch (std::exception& e) {
        g_err = e.what();
        return DBG_ERR_UNSUPPORTED;
    }
}

uint32_t orc_crc32c_bytes(uint32_t crc, const uint8_t* p, uint64_t n) {
    for (uint64_t i = 0; i < n; ++i) crc = crc32c_byte(crc, p[i]);
    return crc;
}

int orc_group_hash(const dbg_column* cols, int ncols, uint64_t rows, uint64_t* out) {
    try {
        group_hash_columns(cols, ncols, 0, rows, out);
        return DBG_OK;
    } catch (std::exception& e) {
        g_err = e.what();
        return DBG_ERR_UNSUPPORTED;
    }
}

int orc_result_type(const dbg_agg_spec* s, dbg_datatype* out) {
    try {
        std::unique_ptr<AggFn> f(make_fn(*s));
        *out = f->return_type();
        return DBG_OK;
    } catch (std::exception& e) {
        g_err = e.what();
        return DBG_ERR_UNSUPPORTED;
    }
}

int orc_filter_select(const dbg_filter* f, uint64_t rows, uint32_t* sel, uint64_t* n_sel) {
    try {
        u64 n = 0;
        for (u64 i = 0; i < rows; ++i)
            if (eval_pred(*f, i)) sel[n++] = (u32)i;
        *n_sel = n;
        return DBG_OK;
    } catch (std::exception& e) {
        g_err = e.what();
        return DBG_ERR_UNSUPPORTED;
    }
}

// Full pipeline over host columns.  arg_cols: n_aggs entries (count(*) entries may have
// dt.type = -1).  filter may be NULL.
int orc_aggregate(const dbg_column* keys, int n_keys, const dbg_column* args, const dbg_agg_spec* specs, int n_aggs,
                  const dbg_filter* filter, uint64_t rows, int threads, orc_result** out) {
    try {
        PipelineSpec ps;
        ps.keys.assign(keys, keys + n_keys);
        ps.args.assign(args, args + n_aggs);
        ps.specs.assign(specs, specs + n_aggs);
        ps.filter = filter;
        ps.rows = rows;
        ps.threads = threads;
        auto* r = new orc_result();
        run_pipeline(ps, r->r);
        *out = r;
        return DBG_OK;
    } catch (OverflowError& e) {
        g_err = e.what();
        return DBG_ERR_OVERFLOW;
    } catch (std::exception& e) {
        g_err = e.what();
        return DBG_ERR_UNSUPPORTED;
    }
}

// The same pipeline, the final states serialized (AggregateMeta::Serialized's Binary columns).
int orc_aggregate_serialized(const dbg_column* keys, int n_keys, const dbg_column* args, const dbg_agg_spec* specs,
                             int n_aggs, const dbg_filter* filter, uint64_t rows, int threads, orc_result** out) {
    try {
        PipelineSpec ps;
        ps.keys.assign(keys, keys + n_keys);
        ps.args.assign(args, args + n_aggs);
        ps.specs.assign(specs, specs + n_aggs);
        ps.filter = filter;
        ps.rows = rows;
        ps.threads = threads;
        ps.serialize = true;
        auto* r = new orc_result();
        run_pipeline(ps, r->r);
        *out = r;
        return DBG_OK;
    } catch (OverflowError& e) {
        g_err = e.what();
        return DBG_ERR_OVERFLOW;
    } catch (std::exception& e) {
        g_err = e.what();
        return DBG_ERR_UNSUPPORTED;
    }
}

// Final aggregate of one Serialized block (states: n_aggs Binary columns); ser = 1 re-serializes.
int orc_merge_serialized(const dbg_column* keys, int n_keys, const dbg_column* states, const dbg_agg_spec* specs,
                         int n_aggs, uint64_t rows, int ser, orc_result** out) {
    try {
        auto* r = new orc_result();
        try {
            run_merge_serialized(std::vector<dbg_column>(keys, keys + n_keys), std::vector<dbg_column>(states, states + n_aggs),
                                 std::vector<dbg_agg_spec>(specs, specs + n_aggs), rows, ser != 0, r->r);
        } catch (...) {
            delete r;
            throw;
        }
        *out = r;
        return DBG_OK;
    } catch (OverflowError& e) {
        g_err = e.what();
        return DBG_ERR_OVERFLOW;
    } catch (std::exception& e) {
        g_err = e.what();
        return DBG_ERR_UNSUPPORTED;
    }
}

uint64_t orc_result_rows(orc_result* r) { return r->r.rows; }
// which: 0 = key column, 1 = aggregate column.  Returns pointers into the result.
int orc_result_column(orc_result* r, int which, int idx, dbg_datatype* dt, const uint8_t** data, uint64_t* data_bytes,
                      const uint64_t** offsets, const uint8_t** valid) {
    std::vector<OwnedColumn>& v = which == 0 ? r->r.keys : r->r.aggs;
    if (idx < 0 || (size_t)idx >= v.size()) return DBG_ERR_INVALID;
    OwnedColumn& c = v[idx];
    *dt = c.dt;
    *data = c.data.data();
    *data_bytes = c.data.size();
    *offsets = c.dt.type == DBG_STRING ? c.offsets.data() : nullptr;
    *valid = c.valid.data();
    return DBG_OK;
}
void orc_result_free(orc_result* r) { delete r; }

// ---- CPU workload generator (same formulas as the device generator, include/dbgpu_datagen.h) ----
void orc_c5_cdf(uint64_t* cdf) {
    u64 s = 0;
    for (u64 r = 1; r <= DG_C5_K; ++r) {
        s += dg_c5_weight(r);
        cdf[r - 1] = s;
    }
}

static void par_for(u64 n, int threads, const std::function<void(u64, u64)>& f) {
    int T = std::max(1, threads);
    std::vector<std::thread> th;
    for (int t = 1; t < T; ++t) th.emplace_back(f, n * t / T, n * (t + 1) / T);
    f(0, n / T);
    for (auto& x : th) x.join();
}

// cfg 2: out0 i16.  cfg 3: out0 i64.  cfg 4: out0 i64 WatchID, out1 i32 ClientIP, out2 i16 IsRefresh,
// out3 i16 ResolutionWidth.  cfg 1: out0 i32 shipdate, out1 u8 returnflag, out2 u8 linestatus,
// out3..out7 i64 quantity, extprice, discount, tax, disc_price, out8 i64 charge.
// cfg 5 (lengths pass): out0 u32 length per row (0 = ''), needs cdf.
int orc_datagen(int cfg, uint64_t seed, uint64_t start, uint64_t rows, void** outs, const uint64_t* cdf, int threads) {
    switch (cfg) {
        case 1:
            par_for(rows, threads, [&](u64 a, u64 b) {
                for (u64 k = a; k < b; ++k) {
                    dg_c1_row r = dg_c1(seed, start + k);
                    ((int32_t*)outs[0])[k] = r.shipdate;
                    ((uint8_t*)outs[1])[k] = r.returnflag;
                    ((uint8_t*)outs[2])[k] = r.linestatus;
                    ((int64_t*)outs[3])[k] = r.quantity;
                    ((int64_t*)outs[4])[k] = r.extprice;
                    ((int64_t*)outs[5])[k] = r.discount;
                    ((int64_t*)outs[6])[k] = r.tax;
                    ((int64_t*)outs[7])[k] = r.disc_price;
                    ((int64_t*)outs[8])[k] = r.charge_lo;
                }
            });
            return DBG_OK;
        case 2:
            par_for(rows, threads, [&](u64 a, u64 b) {
                for (u64 k = a; k < b; ++k) ((int16_t*)outs[0])[k] = dg_c2_adv_engine_id(seed, start + k);
            });
            return DBG_OK;
        case 3:
            par_for(rows, threads, [&](u64 a, u64 b) {
                for (u64 k = a; k < b; ++k) ((int64_t*)outs[0])[k] = dg_c3_user_id(seed, start + k);
            });
            return DBG_OK;
        case 4:
            par_for(rows, threads, [&](u64 a, u64 b) {
                for (u64 k = a; k < b; ++k) {
                    u64 i = start + k;
                    ((int64_t*)outs[0])[k] = dg_c4_watch_id(seed, i);
                    ((int32_t*)outs[1])[k] = dg_c4_client_ip(seed, i);
                    ((int16_t*)outs[2])[k] = dg_c4_is_refresh(seed, i);
                    ((int16_t*)outs[3])[k] = dg_c4_resolution_width(seed, i);
                }
            });
            return DBG_OK;
        case 5:
            par_for(rows, threads, [&](u64 a, u64 b) {
                for (u64 k = a; k < b; ++k) {
                    u64 i = start + k;
                    ((uint32_t*)outs[0])[k] = dg_c5_is_empty(seed, i) ? 0 : dg_c5_phrase_len(dg_c5_rank(seed, i, cdf));
                }
            });
            return DBG_OK;
    }
    return DBG_ERR_INVALID;
}

// cfg 5 bytes pass: offsets (rows+1, from the lengths pass) -> phrase bytes.
int orc_datagen_c5_bytes(uint64_t seed, uint64_t start, uint64_t rows, const uint64_t* offsets, uint8_t* data,
                         const uint64_t* cdf, int threads) {
    par_for(rows, threads, [&](u64 a, u64 b) {
        for (u64 k = a; k < b; ++k) {
            u64 i = start + k;
            u64 o = offsets[k], l = offsets[k + 1] - offsets[k];
            if (l == 0) continue;
            u32 r = dg_c5_rank(seed, i, cdf);
            for (u32 j = 0; j < l; ++j) data[o + j] = dg_c5_phrase_byte(r, j);
        }
    });
    return DBG_OK;
}

}  // extern "C"
