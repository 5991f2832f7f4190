// filter.hpp — descriptors of the standalone filter (filter.hip) and the workload generator.
#pragma once
#include "device.hpp"

struct FilterDesc {
    u64 rows;
    int32_t n_cols, n_nodes;
    DCol cols[DBG_MAX_FCOLS];
    DNode nodes[DBG_MAX_NODES];
};

u64 filter_blocks(u64 rows);
void launch_filter_select(hipStream_t s, const FilterDesc* f, u64 rows, u64* scratch, u64* total, u32* sel);
void launch_take_fixed(hipStream_t s, const DCol& c, const u32* sel, u64 n, u8* out, u8* vbytes);
void launch_take_string_offsets(hipStream_t s, const u64* offs, const u32* sel, u64 n, u64* out_offs);
void launch_take_string_bytes(hipStream_t s, const DCol& c, const u32* sel, u64 n, const u64* out_offs, u8* out, u8* vbytes);

// datagen.hip
int launch_datagen(hipStream_t s, int cfg, u64 seed, u64 start, u64 rows, void** outs, int n_outs, const u64* aux);
