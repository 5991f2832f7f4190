// legacy.hip — group keys and FastHash of the legacy HashMethod path
// (enable_experimental_aggregate_hashtable = 0).
//
// HashMethodKind::choose_hash_method_with_types (EXP/kernels/group_by.rs:48-97) picks
//   SingleBinary for one String/Binary key, FixedKeys<T> when every key is a number, date,
//   timestamp or decimal (T = u8 / u16 / u32 / u64 / u128 / U256 by the packed width: value bytes
//   plus one null byte per nullable key), Serializer otherwise (the serialized key bytes, SerCrc).
// FixedKeys packs a row (build_keys_vec / fixed_hash, EXP/kernels/group_by_hash/
// method_fixed_keys.rs:74-100, 366-470): columns stably sorted by byte width, widest first, values
// little-endian from offset 0, each nullable column's null byte after all the values (1 = NULL, the
// value bytes then stay 0).  FastHash (HT/traits.rs:172-330, the sse4.2 build): CRC32C of the key's
// little-endian u64 words, `_mm_crc32_u64(u64::MAX, w)` chained (no final inversion; the result is
// the 32-bit CRC zero-extended); [u8] hashes 8-byte words, the last one (1..8 bytes) read
// little-endian and zero-padded, and an empty slice hashes to u64::MAX.  The partitioned table's
// bucket is hash2bucket<BITS, true> = (hash >> (32 - BITS)) & (2^BITS - 1)
// (HT/partitioned_hashtable.rs:77-83).
#include "device.hpp"
#include "legacy.hpp"

__global__ void __launch_bounds__(256) legacy_fixed_hash_kernel(LegacyKeyDesc d, u64 rows, u64* __restrict__ hash,
                                                               u32* __restrict__ bucket, u32 bits) {
    __shared__ u32 tab[256];
    crc_table_init(tab);
    for (u64 i = blockIdx.x * (u64)blockDim.x + threadIdx.x; i < rows; i += (u64)gridDim.x * blockDim.x) {
        u64 k[4] = {0, 0, 0, 0};
        for (int j = 0; j < d.n; ++j) {
            const DCol& c = d.cols[j];
            if (c.nullable && !dcol_valid(c, i)) {
                const u32 o = d.null_off[j];
                k[o >> 3] |= 1ULL << (8 * (o & 7));
                continue;
            }
            const u32 w = c.width, o = d.off[j];
            const u64 lo = dcol_bits(c, i), hi = w == 16 ? dcol_hi(c, i) : 0;
            legacy_put(k, o, lo, hi, w);
        }
        const u64 crc = legacy_fixed_crc(tab, k, d.words);
        hash[i] = crc;
        if (bucket) bucket[i] = legacy_bucket(crc, bits);
    }
}

__global__ void __launch_bounds__(256) legacy_binary_hash_kernel(DCol c, u64 rows, u64* __restrict__ hash,
                                                                u32* __restrict__ bucket, u32 bits) {
    __shared__ u32 tab[256];
    crc_table_init(tab);
    for (u64 i = blockIdx.x * (u64)blockDim.x + threadIdx.x; i < rows; i += (u64)gridDim.x * blockDim.x) {
        // a NULL of a nullable String key hashes as its (empty) value bytes — NullableColumn keeps
        // the inner column's bytes; the reference hashes what the column holds at the row
        const StrRef s = dcol_str(c, i);
        const u64 v = legacy_bytes_hash(tab, s.p, s.len);
        hash[i] = v;
        if (bucket) bucket[i] = legacy_bucket(v, bits);
    }
}

// HashMethodSerializer: d.cols in key order (d.n columns), hashed as their serialized bytes
__global__ void __launch_bounds__(256) legacy_serializer_hash_kernel(LegacyKeyDesc d, u64 rows, u64* __restrict__ hash,
                                                                    u32* __restrict__ bucket, u32 bits) {
    __shared__ u32 tab[256];
    crc_table_init(tab);
    for (u64 i = blockIdx.x * (u64)blockDim.x + threadIdx.x; i < rows; i += (u64)gridDim.x * blockDim.x) {
        SerCrc sc;
        for (int j = 0; j < d.n; ++j) {
            const DCol& c = d.cols[j];
            const bool v = dcol_valid(c, i);
            if (c.type == DBG_STRING) {
                const StrRef sr = v ? dcol_str(c, i) : StrRef{nullptr, 0};
                sc.column(tab, c.type, c.nullable, v, 0, 0, sr.p, sr.len);
            } else {
                const u64 lo = v ? dcol_bits(c, i) : 0, hi = (v && c.type == DBG_DECIMAL128) ? dcol_hi(c, i) : 0;
                sc.column(tab, c.type, c.nullable, v, lo, hi, nullptr, 0);
            }
        }
        const u64 h = sc.finish(tab);
        hash[i] = h;
        if (bucket) bucket[i] = legacy_bucket(h, bits);
    }
}

static u32 grid_of(u64 rows) {
    u64 b = (rows + 255) / 256;
    return (u32)(b > 8192 ? 8192 : (b ? b : 1));
}

void launch_legacy_fixed_hash(hipStream_t s, const LegacyKeyDesc& d, u64 rows, u64* hash, u32* bucket, u32 bits) {
    if (!rows) return;
    hipLaunchKernelGGL(legacy_fixed_hash_kernel, dim3(grid_of(rows)), dim3(256), 0, s, d, rows, hash, bucket, bits);
}

void launch_legacy_binary_hash(hipStream_t s, const DCol& c, u64 rows, u64* hash, u32* bucket, u32 bits) {
    if (!rows) return;
    hipLaunchKernelGGL(legacy_binary_hash_kernel, dim3(grid_of(rows)), dim3(256), 0, s, c, rows, hash, bucket, bits);
}

void launch_legacy_serializer_hash(hipStream_t s, const LegacyKeyDesc& d, u64 rows, u64* hash, u32* bucket, u32 bits) {
    if (!rows) return;
    hipLaunchKernelGGL(legacy_serializer_hash_kernel, dim3(grid_of(rows)), dim3(256), 0, s, d, rows, hash, bucket, bits);
}
