// serde.hpp — serialized-state ingest (serde.hip), shared with abi.hip.
#pragma once
#include "agg.hpp"

// The key columns (arrow layout, device) and the Binary state columns of one Serialized block.
struct SerIngest {
    DCol keys[DBG_MAX_KEYS];
    const u8* st_data[DBG_MAX_AGGS];
    const u64* st_offs[DBG_MAX_AGGS];  // rows + 1
};
enum { ERR_SER_MALFORMED = 1, ERR_SER_UNREP = 2 };
void launch_ser_ingest(hipStream_t s, const Spec* dspec, const SerIngest& in, u64 n, u8* rec_out, u64* err);
