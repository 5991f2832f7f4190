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

void launch_legacy_fixed_hash(hipStream_t s, const LegacyKeyDesc& d, u64 rows, u64* hash, u32* bucket, u32 bits);
void launch_legacy_binary_hash(hipStream_t s, const DCol& c, u64 rows, u64* hash, u32* bucket, u32 bits);
