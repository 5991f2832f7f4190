// Read-bandwidth ceiling for the C2 insert's access pattern: a 200 MB int16 column streamed with
// 16-byte nontemporal loads, grid-strided, U loads in flight per lane, a trivial reduction so the
// loads are live.  Prints GB/s per configuration (hipEvent timing, median of 20 launches).
// Build: hipcc --offload-arch=gfx950 -O3 -o stream stream.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdio>
#include <vector>

typedef unsigned int v4u __attribute__((ext_vector_type(4)));
typedef const v4u __attribute__((address_space(1)))* gv4p;

template <int U>
__global__ void rd(const v4u* __restrict__ p, unsigned long long n, unsigned* out) {
    gv4p vp = (gv4p)p;
    const unsigned long long g = (unsigned long long)gridDim.x * blockDim.x;
    unsigned long long k = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
    unsigned acc = 0;
    for (; k + (U - 1) * g < n; k += U * g) {
        v4u y[U];
#pragma unroll
        for (int u = 0; u < U; ++u) y[u] = __builtin_nontemporal_load(vp + k + u * g);
#pragma unroll
        for (int u = 0; u < U; ++u) acc |= (y[u].x | y[u].y | y[u].z | y[u].w) == 0x12345 ? 1u : 0u;
    }
    for (; k < n; k += g) acc |= vp[k].x == 0x12345;
    if (acc) out[0] = acc;
}

template <int U>
float run(const v4u* p, unsigned long long n, unsigned* out, int blocks, int nt) {
    hipEvent_t a, b;
    hipEventCreate(&a);
    hipEventCreate(&b);
    std::vector<float> ts;
    for (int r = 0; r < 23; ++r) {
        hipEventRecord(a);
        hipLaunchKernelGGL(rd<U>, dim3(blocks), dim3(nt), 0, 0, p + (r & 3) * n, n, out);
        hipEventRecord(b);
        hipEventSynchronize(b);
        float ms;
        hipEventElapsedTime(&ms, a, b);
        if (r >= 3) ts.push_back(ms);
    }
    std::sort(ts.begin(), ts.end());
    return ts[ts.size() / 2];
}

int main() {
    const unsigned long long bytes = 200000000ull, n = bytes / 16;
    v4u* p;
    unsigned* out;
    hipMalloc(&p, 4 * bytes);  // 4 rotating copies: not served from the 256 MiB MALL
    hipMalloc(&out, 4);
    hipMemset(p, 1, 4 * bytes);
    hipDeviceSynchronize();
    struct C { int blocks, nt, u; } cs[] = {{256, 1024, 4}, {256, 1024, 8}, {512, 512, 4}, {512, 512, 8}, {1024, 256, 8},
                                          {2048, 256, 4}, {4096, 256, 4}, {512, 1024, 4}, {1024, 1024, 2}};
    for (auto c : cs) {
        float ms = c.u == 8 ? run<8>(p, n, out, c.blocks, c.nt) : (c.u == 4 ? run<4>(p, n, out, c.blocks, c.nt) : run<2>(p, n, out, c.blocks, c.nt));
        printf("blocks %5d nt %4d unroll %d: %.2f us  %.0f GB/s\n", c.blocks, c.nt, c.u, ms * 1e3, bytes / (ms * 1e-3) / 1e9);
    }
    return 0;
}
