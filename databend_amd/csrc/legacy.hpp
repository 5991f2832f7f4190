// legacy.hpp — descriptors of the legacy HashMethod FastHash kernels (legacy.hip).
#pragma once
#include "device.hpp"

// FixedKeys packing of up to 8 key columns: cols in packing order (widest first, stable), each
// value at off[j], each nullable column's null byte at null_off[j]; `words` little-endian u64
// words of the packed key T are hashed (1 for u8..u64, 2 for u128, 4 for U256).
struct LegacyKeyDesc {
    int32_t n;
    u32 words;
    DCol cols[DBG_MAX_KEYS];
    u32 off[DBG_MAX_KEYS];
    u32 null_off[DBG_MAX_KEYS];
};

// Layout of a table's group key under the legacy method, indexed by key column (abi.hip
// legacy_layout): FixedKeys value offset off[c] and null byte null_off[c] (-1: not nullable), or
// SingleBinary (binary = 1).  Buckets are hash2bucket<bits, true>.
struct LegacyLayout {
    int32_t binary;
    int32_t serializer;  // HashMethodSerializer: FastHash of the serialized key bytes
    u32 words;
    u32 bits;
    u32 off[DBG_MAX_KEYS];
    int32_t null_off[DBG_MAX_KEYS];
};

// CRC32C (Castagnoli, reflected 0x82F63B78) of 8 little-endian bytes, table-driven from LDS
__device__ __forceinline__ u32 crc32c_u64(const u32* tab, u32 crc, u64 v) {
#pragma unroll
    for (int b = 0; b < 8; ++b) crc = tab[(crc ^ (u32)(v >> (8 * b))) & 0xffu] ^ (crc >> 8);
    return crc;
}

__device__ __forceinline__ void crc_table_init(u32* tab) {
    for (u32 i = threadIdx.x; i < 256; i += blockDim.x) {
        u32 c = i;
        for (int k = 0; k < 8; ++k) c = (c >> 1) ^ (0x82F63B78u & (0u - (c & 1u)));
        tab[i] = c;
    }
    __syncthreads();
}

// value bytes (w <= 16, little-endian lo/hi) at byte offset o of the packed key k[4]
__device__ __forceinline__ void legacy_put(u64* k, u32 o, u64 lo, u64 hi, u32 w) {
    const u32 wi = o >> 3, sh = 8 * (o & 7);
    k[wi] |= lo << sh;
    if (sh && wi + 1 < 4) k[wi + 1] |= lo >> (64 - sh);
    if (w == 16) {
        k[wi + 1] |= hi << sh;
        if (sh && wi + 2 < 4) k[wi + 2] |= hi >> (64 - sh);
    }
}

__device__ __forceinline__ u64 legacy_fixed_crc(const u32* tab, const u64* k, u32 words) {
    u32 crc = 0xFFFFFFFFu;
    for (u32 w = 0; w < words; ++w) crc = crc32c_u64(tab, crc, k[w]);
    return crc;
}

// [u8] FastHash: 8-byte little-endian words, the last one zero-padded; empty -> u64::MAX
__device__ __forceinline__ u64 legacy_bytes_hash(const u32* tab, const u8* p, u64 len) {
    if (!len) return ~0ULL;
    u32 crc = 0xFFFFFFFFu;
    for (u64 o = 0; o < len; o += 8) {
        const u64 n = len - o < 8 ? len - o : 8;
        u64 w = 0;
        for (u64 b = 0; b < n; ++b) w |= (u64)p[o + b] << (8 * b);
        crc = crc32c_u64(tab, crc, w);
    }
    return crc;
}

// HashMethodSerializer (EXP/kernels/group_by_hash/method_serializer.rs:39-70): the key is the
// serialize_column_binary bytes of every group column in order (utils.rs:64-121): a nullable
// column's validity byte, then — valid rows only — the value: numbers / Date / Timestamp
// little-endian in their width, Decimal128 16 bytes, Boolean one byte, String its length as u64
// then its bytes.  The [u8] FastHash of that byte string, fed incrementally (8-byte words, the last
// one zero-padded, empty -> u64::MAX), equals legacy_bytes_hash of the concatenation.
struct SerCrc {
    u32 crc = 0xFFFFFFFFu;
    u64 w = 0;
    u32 n = 0;  // bytes in w (< 8)
    u64 total = 0;
    __device__ __forceinline__ void push(const u32* tab, u64 v, u32 nb) {  // nb in 1..8: v's low bytes
        total += nb;
        if (nb < 8) v &= (1ULL << (8 * nb)) - 1;
        w |= n ? (v << (8 * n)) : v;
        const u32 room = 8 - n;
        if (nb < room) {
            n += nb;
            return;
        }
        crc = crc32c_u64(tab, crc, w);
        const u32 rest = nb - room;
        w = rest ? (v >> (8 * room)) : 0;
        n = rest;
    }
    __device__ __forceinline__ void bytes(const u32* tab, const u8* p, u64 len) {
        u64 o = 0;
        for (; o + 8 <= len; o += 8) {
            u64 x = 0;
            for (int b = 0; b < 8; ++b) x |= (u64)gld<u8>(p + o + b) << (8 * b);
            push(tab, x, 8);
        }
        if (o < len) {
            u64 x = 0;
            for (u64 b = 0; b < len - o; ++b) x |= (u64)gld<u8>(p + o + b) << (8 * b);
            push(tab, x, (u32)(len - o));
        }
    }
    // one key column: validity byte (nullable), then the value of a valid row
    __device__ __forceinline__ void column(const u32* tab, int type, bool nullable, bool valid, u64 lo, u64 hi, const u8* sp,
                                           u64 slen) {
        if (nullable) push(tab, valid ? 1 : 0, 1);
        if (!valid) return;
        if (type == DBG_STRING) {
            push(tab, slen, 8);
            bytes(tab, sp, slen);
        } else if (type == DBG_BOOLEAN) {
            push(tab, lo & 1, 1);
        } else if (type == DBG_DECIMAL128) {
            push(tab, lo, 8);
            push(tab, hi, 8);
        } else {
            push(tab, lo, type_width(type));
        }
    }
    __device__ __forceinline__ u64 finish(const u32* tab) {
        if (!total) return ~0ULL;
        if (n) crc = crc32c_u64(tab, crc, w);
        return crc;
    }
};

__device__ __forceinline__ u32 legacy_bucket(u64 h, u32 bits) { return (u32)((h >> (32 - bits)) & ((1ULL << bits) - 1)); }

void launch_legacy_fixed_hash(hipStream_t s, const LegacyKeyDesc& d, u64 rows, u64* hash, u32* bucket, u32 bits);
void launch_legacy_binary_hash(hipStream_t s, const DCol& c, u64 rows, u64* hash, u32* bucket, u32 bits);
void launch_legacy_serializer_hash(hipStream_t s, const LegacyKeyDesc& d, u64 rows, u64* hash, u32* bucket, u32 bits);
