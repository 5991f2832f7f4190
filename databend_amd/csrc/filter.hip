// filter.hip — standalone predicate -> selection vector -> compaction (TransformFilter).
//
// FilterExecutor::select fills an ascending u32 selection (EXP/filter/filter_executor.rs:73-90,
// selector.rs:64-325); take / take_ranges gather the selected rows (filter_executor.rs:91-128,
// EXP/kernels/take.rs:56-91).  The GROUP BY path does not call these — it fuses the predicate
// into agg_insert — they serve the TransformFilter seam on its own.
//
// Two passes over contiguous row tiles (count, then write at scanned offsets) keep the selection
// ascending without a sort.
#include "device.hpp"
#include "filter.hpp"

#define FBLOCK 256
#define ROWS_PER_THREAD 16
#define ROWS_PER_BLOCK (FBLOCK * ROWS_PER_THREAD)

void launch_exclusive_scan(hipStream_t s, u64* data, u64 n, u64* total);

__global__ void __launch_bounds__(FBLOCK) filter_count_kernel(const FilterDesc* __restrict__ f, u64* counts) {
    u64 rows = f->rows;
    u64 base = (u64)blockIdx.x * ROWS_PER_BLOCK + (u64)threadIdx.x * ROWS_PER_THREAD;
    u32 c = 0;
    for (int k = 0; k < ROWS_PER_THREAD; ++k) {
        u64 i = base + k;
        if (i < rows && eval_pred(f->nodes, f->n_nodes, f->cols, i)) c++;
    }
    __shared__ u32 red[FBLOCK];
    red[threadIdx.x] = c;
    __syncthreads();
    for (int off = FBLOCK / 2; off > 0; off >>= 1) {
        if ((int)threadIdx.x < off) red[threadIdx.x] += red[threadIdx.x + off];
        __syncthreads();
    }
    if (threadIdx.x == 0) counts[blockIdx.x] = red[0];
}

__global__ void __launch_bounds__(FBLOCK) filter_write_kernel(const FilterDesc* __restrict__ f, const u64* pos, u32* sel) {
    u64 rows = f->rows;
    u64 base = (u64)blockIdx.x * ROWS_PER_BLOCK + (u64)threadIdx.x * ROWS_PER_THREAD;
    u32 bits = 0;
    for (int k = 0; k < ROWS_PER_THREAD; ++k) {
        u64 i = base + k;
        if (i < rows && eval_pred(f->nodes, f->n_nodes, f->cols, i)) bits |= 1u << k;
    }
    __shared__ u32 sc[FBLOCK];
    u32 c = __popc(bits);
    sc[threadIdx.x] = c;
    __syncthreads();
    for (int off = 1; off < FBLOCK; off <<= 1) {
        u32 v = threadIdx.x >= (u32)off ? sc[threadIdx.x - off] : 0;
        __syncthreads();
        sc[threadIdx.x] += v;
        __syncthreads();
    }
    u64 p = pos[blockIdx.x] + sc[threadIdx.x] - c;
    for (int k = 0; k < ROWS_PER_THREAD; ++k)
        if (bits & (1u << k)) sel[p++] = (u32)(base + k);
}

u64 filter_blocks(u64 rows) { return (rows + ROWS_PER_BLOCK - 1) / ROWS_PER_BLOCK; }

void launch_filter_select(hipStream_t s, const FilterDesc* f, u64 rows, u64* scratch, u64* total, u32* sel) {
    u64 nb = filter_blocks(rows);
    if (nb == 0) return;
    hipLaunchKernelGGL(filter_count_kernel, dim3((u32)nb), dim3(FBLOCK), 0, s, f, scratch);
    launch_exclusive_scan(s, scratch, nb, total);
    hipLaunchKernelGGL(filter_write_kernel, dim3((u32)nb), dim3(FBLOCK), 0, s, f, scratch, sel);
}

__global__ void take_fixed_kernel(DCol c, const u32* sel, u64 n, u8* out, u8* vbytes) {
    for (u64 k = blockIdx.x * (u64)blockDim.x + threadIdx.x; k < n; k += (u64)gridDim.x * blockDim.x) {
        u64 i = sel[k];
        if (c.type == DBG_BOOLEAN) {
            out[k] = (u8)dcol_bits(c, i);
        } else {
            const u8* src = c.data + i * (u64)c.width;
            u8* dst = out + k * (u64)c.width;
            for (u32 b = 0; b < c.width; ++b) dst[b] = src[b];
        }
        if (vbytes) vbytes[k] = dcol_valid(c, i) ? 1 : 0;
    }
}

// StringColumn take (EXP/kernels/take.rs:56-91): lengths of the selected rows, then (after an
// exclusive scan turns them into the output offsets) their bytes.  Rows are copied 8 bytes at a
// time where source and destination allow it.
__global__ void take_str_len_kernel(const u64* __restrict__ offs, const u32* __restrict__ sel, u64 n, u64* __restrict__ out_offs) {
    for (u64 k = blockIdx.x * (u64)blockDim.x + threadIdx.x; k < n; k += (u64)gridDim.x * blockDim.x) {
        const u64 i = sel[k];
        out_offs[k] = offs[i + 1] - offs[i];
    }
}

__global__ void take_str_bytes_kernel(DCol c, const u32* __restrict__ sel, u64 n, const u64* __restrict__ out_offs,
                                      u8* __restrict__ out, u8* __restrict__ vbytes) {
    for (u64 k = blockIdx.x * (u64)blockDim.x + threadIdx.x; k < n; k += (u64)gridDim.x * blockDim.x) {
        const u64 i = sel[k];
        const u64 so = c.offsets[i], len = c.offsets[i + 1] - so;
        const u8* src = c.data + so;
        u8* dst = out + out_offs[k];
        u64 b = 0;
        if ((((uintptr_t)src | (uintptr_t)dst) & 7) == 0)
            for (; b + 8 <= len; b += 8) *(u64*)(dst + b) = *(const u64*)(src + b);
        for (; b < len; ++b) dst[b] = src[b];
        if (vbytes) vbytes[k] = dcol_valid(c, i) ? 1 : 0;
    }
}

void launch_take_string_offsets(hipStream_t s, const u64* offs, const u32* sel, u64 n, u64* out_offs) {
    if (!n) return;
    u64 blocks = (n + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL(take_str_len_kernel, dim3((u32)blocks), dim3(256), 0, s, offs, sel, n, out_offs);
}

void launch_take_string_bytes(hipStream_t s, const DCol& c, const u32* sel, u64 n, const u64* out_offs, u8* out, u8* vbytes) {
    if (!n) return;
    u64 blocks = (n + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL(take_str_bytes_kernel, dim3((u32)blocks), dim3(256), 0, s, c, sel, n, out_offs, out, vbytes);
}

void launch_take_fixed(hipStream_t s, const DCol& c, const u32* sel, u64 n, u8* out, u8* vbytes) {
    if (!n) return;
    u64 blocks = (n + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL(take_fixed_kernel, dim3((u32)blocks), dim3(256), 0, s, c, sel, n, out, vbytes);
}
