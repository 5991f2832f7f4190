// datagen.hip — device generator for the synthetic workloads C1..C5.
// The numbers_mt analog: every row is an independent function of (seed, row index), with the
// formulas of include/dbgpu_datagen.h, so device columns equal the host generator's bit for bit.
#include "device.hpp"
#include "filter.hpp"
#include "../../include/dbgpu_datagen.h"

__global__ void gen_c1(u64 seed, u64 start, u64 rows, int32_t* ship, u8* rf, u8* ls, u64* rf_off, u64* ls_off, u8* qty,
                       u8* price, u8* disc, u8* tax, u8* dprice, u8* charge) {
    for (u64 k = blockIdx.x * (u64)blockDim.x + threadIdx.x; k < rows; k += (u64)gridDim.x * blockDim.x) {
        dg_c1_row r = dg_c1(seed, start + k);
        ship[k] = r.shipdate;
        rf[k] = r.returnflag;
        ls[k] = r.linestatus;
        rf_off[k] = k;
        ls_off[k] = k;
        if (k == rows - 1) {
            rf_off[rows] = rows;
            ls_off[rows] = rows;
        }
        int64_t v[6] = {r.quantity, r.extprice, r.discount, r.tax, r.disc_price, r.charge_lo};
        u8* o[6] = {qty, price, disc, tax, dprice, charge};
        for (int c = 0; c < 6; ++c) {  // Decimal128 = i128 LE (sign-extended)
            u64* d = (u64*)(o[c] + k * 16);
            d[0] = (u64)v[c];
            d[1] = v[c] < 0 ? ~0ULL : 0ULL;
        }
    }
}

__global__ void gen_c2(u64 seed, u64 start, u64 rows, int16_t* out) {
    // 8 rows per thread, one 16-byte store
    u64 n8 = rows / 8;
    for (u64 k = blockIdx.x * (u64)blockDim.x + threadIdx.x; k < n8; k += (u64)gridDim.x * blockDim.x) {
        int16_t v[8];
        for (int j = 0; j < 8; ++j) v[j] = dg_c2_adv_engine_id(seed, start + k * 8 + j);
        *(uint4*)(out + k * 8) = *(uint4*)v;
    }
    for (u64 k = n8 * 8 + blockIdx.x * (u64)blockDim.x + threadIdx.x; k < rows; k += (u64)gridDim.x * blockDim.x)
        out[k] = dg_c2_adv_engine_id(seed, start + k);
}

__global__ void gen_c3(u64 seed, u64 start, u64 rows, int64_t* out) {
    for (u64 k = blockIdx.x * (u64)blockDim.x + threadIdx.x; k < rows; k += (u64)gridDim.x * blockDim.x)
        out[k] = dg_c3_user_id(seed, start + k);
}

__global__ void gen_c4(u64 seed, u64 start, u64 rows, int64_t* w, int32_t* ip, int16_t* rf, int16_t* rw) {
    for (u64 k = blockIdx.x * (u64)blockDim.x + threadIdx.x; k < rows; k += (u64)gridDim.x * blockDim.x) {
        u64 i = start + k;
        w[k] = dg_c4_watch_id(seed, i);
        ip[k] = dg_c4_client_ip(seed, i);
        rf[k] = dg_c4_is_refresh(seed, i);
        rw[k] = dg_c4_resolution_width(seed, i);
    }
}

// C5 pass 1: phrase length per row (0 for '').
__global__ void gen_c5_len(u64 seed, u64 start, u64 rows, const u64* cdf, u64* lens) {
    for (u64 k = blockIdx.x * (u64)blockDim.x + threadIdx.x; k < rows; k += (u64)gridDim.x * blockDim.x) {
        u64 i = start + k;
        lens[k] = dg_c5_is_empty(seed, i) ? 0 : dg_c5_phrase_len(dg_c5_rank(seed, i, cdf));
    }
}

// C5 pass 2: bytes at the given offsets.
__global__ void gen_c5_bytes(u64 seed, u64 start, u64 rows, const u64* cdf, const u64* offs, u8* data) {
    for (u64 k = blockIdx.x * (u64)blockDim.x + threadIdx.x; k < rows; k += (u64)gridDim.x * blockDim.x) {
        u64 o = offs[k], l = offs[k + 1] - o;
        if (!l) continue;
        u32 r = dg_c5_rank(seed, start + k, cdf);
        for (u32 j = 0; j < l; ++j) data[o + j] = dg_c5_phrase_byte(r, j);
    }
}

static u32 grid_for(u64 rows) {
    u64 b = (rows + 255) / 256;
    if (b > 16384) b = 16384;
    return (u32)(b ? b : 1);
}

int launch_datagen(hipStream_t s, int cfg, u64 seed, u64 start, u64 rows, void** o, int n, const u64* aux) {
    if (rows == 0) return 0;
    switch (cfg) {
        case 1:
            if (n < 11) return -1;
            hipLaunchKernelGGL(gen_c1, dim3(grid_for(rows)), dim3(256), 0, s, seed, start, rows, (int32_t*)o[0], (u8*)o[1],
                               (u8*)o[2], (u64*)o[3], (u64*)o[4], (u8*)o[5], (u8*)o[6], (u8*)o[7], (u8*)o[8], (u8*)o[9],
                               (u8*)o[10]);
            return 0;
        case 2:
            hipLaunchKernelGGL(gen_c2, dim3(grid_for(rows / 8 + 1)), dim3(256), 0, s, seed, start, rows, (int16_t*)o[0]);
            return 0;
        case 3:
            hipLaunchKernelGGL(gen_c3, dim3(grid_for(rows)), dim3(256), 0, s, seed, start, rows, (int64_t*)o[0]);
            return 0;
        case 4:
            if (n < 4) return -1;
            hipLaunchKernelGGL(gen_c4, dim3(grid_for(rows)), dim3(256), 0, s, seed, start, rows, (int64_t*)o[0], (int32_t*)o[1],
                               (int16_t*)o[2], (int16_t*)o[3]);
            return 0;
        case 5:  // o[0] = lengths (u64, pass 1)
            hipLaunchKernelGGL(gen_c5_len, dim3(grid_for(rows)), dim3(256), 0, s, seed, start, rows, aux, (u64*)o[0]);
            return 0;
        case 6:  // C5 pass 2: o[0] = offsets (rows+1), o[1] = bytes
            hipLaunchKernelGGL(gen_c5_bytes, dim3(grid_for(rows)), dim3(256), 0, s, seed, start, rows, aux, (const u64*)o[0], (u8*)o[1]);
            return 0;
    }
    return -1;
}
