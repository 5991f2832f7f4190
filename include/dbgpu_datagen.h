/*
 * dbgpu_datagen.h — the synthetic workloads C1..C5 of SURVEY.md §8d as pure integer formulas.
 *
 * Counter-based splitmix64: row i of stream s under seed S draws dg_rand(S, s, i), so any row range
 * can be generated independently and the host (tests, CPU baseline) and the device generator
 * produce bit-identical columns.  Base seed 0xDA7ABE7D + cfg.  Shared by the HIP generator
 * (databend_amd/csrc/datagen.hip) and the CPU generator (oracle/); it defines the INPUT, not the
 * algorithm under test.
 */
#ifndef DBGPU_DATAGEN_H
#define DBGPU_DATAGEN_H

#include <stdint.h>

#if defined(__HIPCC__)
#define DG_HD __host__ __device__ __forceinline__
#else
#define DG_HD static inline
#endif

#define DG_BASE_SEED 0xDA7ABE7DULL

DG_HD uint64_t dg_mix(uint64_t z) {
    z ^= z >> 30;
    z *= 0xbf58476d1ce4e5b9ULL;
    z ^= z >> 27;
    z *= 0x94d049bb133111ebULL;
    z ^= z >> 31;
    return z;
}

DG_HD uint64_t dg_rand(uint64_t seed, uint32_t stream, uint64_t i) {
    return dg_mix(seed + (uint64_t)stream * 0xD1B54A32D192ED03ULL + (i + 1) * 0x9E3779B97F4A7C15ULL);
}

/* ---- C2: ClickBench Q8 AdvEngineID Int16: 0 with p = 0.9937, else uniform {1..32} ---- */
#define DG_C2_P0_U32 4267909002u /* round(0.9937 * 2^32) */
DG_HD int16_t dg_c2_adv_engine_id(uint64_t seed, uint64_t i) {
    uint64_t u = dg_rand(seed, 0, i);
    if ((uint32_t)(u >> 32) < DG_C2_P0_U32) return 0;
    return (int16_t)(1 + (uint32_t)(u & 0xffffffffu) % 32u);
}

/* ---- C3: ClickBench Q16/17 UserID Int64 = mix64(u), u uniform in [0, 2^27) ---- */
DG_HD int64_t dg_c3_user_id(uint64_t seed, uint64_t i) {
    return (int64_t)dg_mix(dg_rand(seed, 0, i) >> 37);
}

/* ---- C4: ClickBench Q33 (WatchID, ClientIP), IsRefresh, ResolutionWidth ---- */
DG_HD int64_t dg_c4_watch_id(uint64_t seed, uint64_t i) { return (int64_t)dg_mix(seed ^ (i * 0x9E3779B97F4A7C15ULL)); }
DG_HD int32_t dg_c4_client_ip(uint64_t seed, uint64_t i) { return (int32_t)(uint32_t)dg_rand(seed, 1, i); }
#define DG_C4_P_REFRESH_U32 429496730u /* round(0.1 * 2^32) */
DG_HD int16_t dg_c4_is_refresh(uint64_t seed, uint64_t i) {
    return (int16_t)((uint32_t)(dg_rand(seed, 2, i) >> 32) < DG_C4_P_REFRESH_U32 ? 1 : 0);
}
DG_HD int16_t dg_c4_resolution_width(uint64_t seed, uint64_t i) { return (int16_t)(dg_rand(seed, 3, i) % 2561u); }

/* ---- C5: ClickBench Q13 SearchPhrase String: '' with p = 0.87, else Zipf(1) over 2^23 phrases ----
 * Zipf by an exact integer CDF: weight(r) = floor(2^40 / r), r = 1..2^23; cdf[r-1] = sum of weights
 * up to r.  A draw t = dg_rand(seed,1,i) % cdf[K-1] picks the smallest r with t < cdf[r-1].
 * Phrase r: length 5 + mix(r ^ 0x5EED) % 28 (5..32 bytes); bytes 0..4 are the base-26 digits of r-1
 * ('a' + digit, least significant first, so phrases are distinct), the rest 'a' + mix((r<<6)|j) % 26. */
#define DG_C5_K (1u << 23)
#define DG_C5_P_EMPTY_U32 3736621548u /* round(0.87 * 2^32) */
DG_HD uint64_t dg_c5_weight(uint64_t r) { return (1ULL << 40) / r; }
DG_HD int dg_c5_is_empty(uint64_t seed, uint64_t i) {
    return (uint32_t)(dg_rand(seed, 0, i) >> 32) < DG_C5_P_EMPTY_U32;
}
DG_HD uint32_t dg_c5_rank(uint64_t seed, uint64_t i, const uint64_t* cdf) {
    uint64_t t = dg_rand(seed, 1, i) % cdf[DG_C5_K - 1];
    uint32_t lo = 0, hi = DG_C5_K - 1; /* smallest idx with t < cdf[idx] */
    while (lo < hi) {
        uint32_t mid = (lo + hi) >> 1;
        if (t < cdf[mid]) hi = mid; else lo = mid + 1;
    }
    return lo + 1;
}
DG_HD uint32_t dg_c5_phrase_len(uint32_t r) { return 5u + (uint32_t)(dg_mix((uint64_t)r ^ 0x5EEDULL) % 28u); }
DG_HD uint8_t dg_c5_phrase_byte(uint32_t r, uint32_t j) {
    if (j < 5) {
        uint32_t v = r - 1;
        for (uint32_t k = 0; k < j; ++k) v /= 26u;
        return (uint8_t)('a' + v % 26u);
    }
    return (uint8_t)('a' + dg_mix(((uint64_t)r << 6) | j) % 26u);
}

/* ---- C1: TPC-H lineitem, spec-distributed (SURVEY.md §8d source (b)), SF1 = 6,001,215 rows ----
 * Dates are days since 1970-01-01.  Decimal(15,2) columns are in hundredths. */
#define DG_C1_ROWS_SF1 6001215ULL
#define DG_DATE_1992_01_01 8035
#define DG_DATE_1995_06_17 9298
#define DG_DATE_1998_08_02 10440
#define DG_DATE_1998_09_02 10471 /* Q1: l_shipdate <= add_days('1998-12-01', -90) */
typedef struct dg_c1_row {
    int32_t shipdate;
    uint8_t returnflag; /* 'A' 'N' 'R' */
    uint8_t linestatus; /* 'F' 'O' */
    int64_t quantity;   /* Decimal(15,2) */
    int64_t extprice;   /* Decimal(15,2) */
    int64_t discount;   /* Decimal(15,2) */
    int64_t tax;        /* Decimal(15,2) */
    int64_t disc_price; /* extprice * (1 - discount): Decimal(31,4) */
    int64_t charge_lo;  /* disc_price * (1 + tax): Decimal(38,6), fits in i64 at SF1 */
} dg_c1_row;
DG_HD dg_c1_row dg_c1(uint64_t seed, uint64_t i) {
    dg_c1_row r;
    int32_t orderdate = DG_DATE_1992_01_01 + (int32_t)(dg_rand(seed, 0, i) % (uint64_t)(DG_DATE_1998_08_02 - DG_DATE_1992_01_01 + 1));
    r.shipdate = orderdate + 1 + (int32_t)(dg_rand(seed, 1, i) % 121u);
    int32_t receipt = r.shipdate + 1 + (int32_t)(dg_rand(seed, 2, i) % 30u);
    uint64_t f = dg_rand(seed, 3, i);
    r.returnflag = receipt <= DG_DATE_1995_06_17 ? ((f & 1) ? 'R' : 'A') : 'N';
    r.linestatus = r.shipdate > DG_DATE_1995_06_17 ? 'O' : 'F';
    int64_t qty = 1 + (int64_t)(dg_rand(seed, 4, i) % 50u);
    int64_t partkey = 1 + (int64_t)(dg_rand(seed, 5, i) % 200000u);
    int64_t retail = 90000 + ((partkey / 10) % 20001) + 100 * (partkey % 1000); /* cents */
    r.quantity = qty * 100;
    r.extprice = qty * retail;
    r.discount = (int64_t)(dg_rand(seed, 6, i) % 11u);
    r.tax = (int64_t)(dg_rand(seed, 7, i) % 9u);
    r.disc_price = r.extprice * (100 - r.discount);
    r.charge_lo = r.disc_price * (100 + r.tax);
    return r;
}

#endif /* DBGPU_DATAGEN_H */
