// Streaming-read ceiling on MI355X: how fast can one launch read N bytes (16-B loads)?
// Used to calibrate what the C2 insert kernel can reach.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
typedef unsigned int v4u __attribute__((ext_vector_type(4)));

template <int UNROLL>
__global__ void __launch_bounds__(1024) rd(const v4u* __restrict__ p, size_t nvec, unsigned* out) {
    unsigned acc = 0;
    size_t stride = (size_t)gridDim.x * blockDim.x;
    size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x;
    for (; i + (UNROLL - 1) * stride < nvec; i += UNROLL * stride) {
        v4u y[UNROLL];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) y[u] = __builtin_nontemporal_load(p + i + u * stride);
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) acc ^= y[u].x ^ y[u].y ^ y[u].z ^ y[u].w;
    }
    for (; i < nvec; i += stride) { v4u y = p[i]; acc ^= y.x ^ y.y ^ y.z ^ y.w; }
    if (acc == 0x12345678) out[0] = acc;
}

// contiguous chunk per block
template <int UNROLL>
__global__ void __launch_bounds__(1024) rdc(const v4u* __restrict__ p, size_t nvec, size_t per_block, unsigned* out) {
    unsigned acc = 0;
    size_t b0 = blockIdx.x * per_block, b1 = b0 + per_block < nvec ? b0 + per_block : nvec;
    size_t i = b0 + threadIdx.x;
    for (; i + (UNROLL - 1) * blockDim.x < b1; i += UNROLL * blockDim.x) {
        v4u y[UNROLL];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) y[u] = __builtin_nontemporal_load(p + i + u * blockDim.x);
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) acc ^= y[u].x ^ y[u].y ^ y[u].z ^ y[u].w;
    }
    for (; i < b1; i += blockDim.x) { v4u y = p[i]; acc ^= y.x ^ y.y ^ y.z ^ y.w; }
    if (acc == 0x12345678) out[0] = acc;
}

int main(int argc, char** argv) {
    size_t bytes = argc > 1 ? strtoull(argv[1], 0, 10) : 200000000ull;
    int copies = 4;
    size_t nvec = bytes / 16;
    v4u* bufs[4];
    for (int c = 0; c < copies; ++c) { hipMalloc(&bufs[c], bytes); hipMemset(bufs[c], c + 1, bytes); }
    unsigned* out; hipMalloc(&out, 4);
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    int grids[] = {256, 512, 1024, 2048, 4096};
    int blocks[] = {256, 512, 1024};
    for (int mode = 0; mode < 2; ++mode)
    for (int bs : blocks) for (int g : grids) for (int un = 4; un <= 8; un += 4) {
        auto launch = [&](int c) {
            if (mode == 0) {
                if (un == 4) hipLaunchKernelGGL(rd<4>, dim3(g), dim3(bs), 0, 0, bufs[c], nvec, out);
                else hipLaunchKernelGGL(rd<8>, dim3(g), dim3(bs), 0, 0, bufs[c], nvec, out);
            } else {
                size_t per = (nvec + g - 1) / g;
                if (un == 4) hipLaunchKernelGGL(rdc<4>, dim3(g), dim3(bs), 0, 0, bufs[c], nvec, per, out);
                else hipLaunchKernelGGL(rdc<8>, dim3(g), dim3(bs), 0, 0, bufs[c], nvec, per, out);
            }
        };
        for (int w = 0; w < 8; ++w) launch(w % copies);
        hipDeviceSynchronize();
        int iters = 40;
        float tot = 0;
        for (int it = 0; it < iters; ++it) {
            hipEventRecord(e0); launch(it % copies); hipEventRecord(e1); hipEventSynchronize(e1);
            float ms; hipEventElapsedTime(&ms, e0, e1); tot += ms;
        }
        float us = tot / iters * 1000;
        printf("%s bs=%4d grid=%4d unroll=%d  %7.2f us  %6.0f GB/s\n", mode ? "chunk " : "stride", bs, g, un, us, bytes / (us * 1e3));
    }
    return 0;
}
