// FETCH_SIZE / WRITE_SIZE calibration on gfx950 for the access shapes of this repo's kernels
// (MI355X_MICROARCH.md, HBM section: only 16 B/lane streaming reads are calibrated there).
// Each kernel below is one dispatch with a known byte count over a 4 GiB buffer (16x the
// Infinity Cache, so nothing is served on-die from an earlier kernel):
//   stream16 / stream8 : coalesced streaming reads, 16 or 8 bytes per lane, every byte once
//   rand8 / rand16     : one 8- or 16-byte load per lane at an independent random 64-B-aligned
//                        address (the probe of a hash-table slot) — N loads, N distinct lines
//   rand_atom8         : one 8-byte device atomic add per lane at a random address (slot count)
//   rand_store16       : one 16-byte store per lane at a random 64-B-aligned address
//   stream_store16     : coalesced 16-byte stores, every byte once
// rocprofv3 --pmc FETCH_SIZE (then WRITE_SIZE) over this program gives the counter per dispatch;
// scripts/pmc_calib.py divides by the known bytes / lines.  Prints the known quantities.
// Build: hipcc --offload-arch=gfx950 -O3 -o fetch_calib fetch_calib.hip
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <vector>

typedef unsigned long long u64;
typedef u64 v2u64 __attribute__((ext_vector_type(2)));

__host__ __device__ __forceinline__ u64 mix(u64 x) {
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdULL;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ULL;
    x ^= x >> 33;
    return x;
}

__global__ void stream16(const v2u64* p, u64 n, u64* out) {
    u64 acc = 0;
    for (u64 k = blockIdx.x * (u64)blockDim.x + threadIdx.x; k < n; k += (u64)gridDim.x * blockDim.x) {
        const v2u64 v = p[k];
        acc ^= v.x ^ v.y;
    }
    if (acc == 0x1234567) out[0] = acc;
}
__global__ void stream8(const u64* p, u64 n, u64* out) {
    u64 acc = 0;
    for (u64 k = blockIdx.x * (u64)blockDim.x + threadIdx.x; k < n; k += (u64)gridDim.x * blockDim.x) acc ^= p[k];
    if (acc == 0x1234567) out[0] = acc;
}
// n_lines: 64-B lines of the buffer; loads: random loads to issue
template <int B>
__global__ void rand_load(const u64* p, u64 n_lines, u64 loads, u64 seed, u64* out) {
    u64 acc = 0;
    for (u64 k = blockIdx.x * (u64)blockDim.x + threadIdx.x; k < loads; k += (u64)gridDim.x * blockDim.x) {
        const u64 line = mix(k ^ seed) % n_lines;
        if (B == 8) acc ^= p[line * 8];
        else {
            const v2u64 v = *(const v2u64*)(p + line * 8);
            acc ^= v.x ^ v.y;
        }
    }
    if (acc == 0x1234567) out[0] = acc;
}
__global__ void rand_atom8(u64* p, u64 n_lines, u64 ops, u64 seed) {
    for (u64 k = blockIdx.x * (u64)blockDim.x + threadIdx.x; k < ops; k += (u64)gridDim.x * blockDim.x) {
        const u64 line = mix(k ^ seed) % n_lines;
        atomicAdd(p + line * 8 + 1, 1ULL);
    }
}
__global__ void rand_store16(u64* p, u64 n_lines, u64 ops, u64 seed) {
    for (u64 k = blockIdx.x * (u64)blockDim.x + threadIdx.x; k < ops; k += (u64)gridDim.x * blockDim.x) {
        const u64 line = mix(k ^ seed) % n_lines;
        *(v2u64*)(p + line * 8) = v2u64{k, k};
    }
}
__global__ void stream_store16(v2u64* p, u64 n) {
    for (u64 k = blockIdx.x * (u64)blockDim.x + threadIdx.x; k < n; k += (u64)gridDim.x * blockDim.x) p[k] = v2u64{k, ~k};
}

int main() {
    const u64 bytes = 4ULL << 30;
    u64* buf = nullptr;
    u64* out = nullptr;
    if (hipMalloc(&buf, bytes) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) {
        fprintf(stderr, "hipMalloc failed\n");
        return 1;
    }
    hipMemset(buf, 1, bytes);
    hipDeviceSynchronize();
    const dim3 g(4096), b(256);
    const u64 n_lines = bytes / 64;
    const u64 ops = 8ULL << 20;  // 8,388,608 random accesses over 67M lines (~6 % repeats: counted below)
    // each kernel twice: the second dispatch is the measured one (the first warms the TLB)
    for (int rep = 0; rep < 2; ++rep) {
        hipLaunchKernelGGL(stream16, g, b, 0, 0, (const v2u64*)buf, bytes / 16, out);
        hipLaunchKernelGGL(stream8, g, b, 0, 0, (const u64*)buf, bytes / 8, out);
        hipLaunchKernelGGL(rand_load<8>, g, b, 0, 0, (const u64*)buf, n_lines, ops, 11 + rep, out);
        hipLaunchKernelGGL(rand_load<16>, g, b, 0, 0, (const u64*)buf, n_lines, ops, 23 + rep, out);
        hipLaunchKernelGGL(rand_atom8, g, b, 0, 0, buf, n_lines, ops, 37 + rep);
        hipLaunchKernelGGL(rand_store16, g, b, 0, 0, buf, n_lines, ops, 41 + rep);
        hipLaunchKernelGGL(stream_store16, g, b, 0, 0, (v2u64*)buf, bytes / 16);
    }
    if (hipDeviceSynchronize() != hipSuccess) {
        fprintf(stderr, "kernel failed\n");
        return 1;
    }
    // distinct lines each measured (rep 1) random kernel touched
    auto distinct = [&](u64 seed) {
        std::vector<u64> v(ops);
        for (u64 k = 0; k < ops; ++k) v[k] = mix(k ^ seed) % n_lines;
        std::sort(v.begin(), v.end());
        return (u64)(std::unique(v.begin(), v.end()) - v.begin());
    };
    printf("{\"buffer_bytes\": %llu, \"random_ops\": %llu, \"line_bytes\": 64, \"distinct_lines\": "
           "{\"rand_load8\": %llu, \"rand_load16\": %llu, \"rand_atom8\": %llu, \"rand_store16\": %llu}}\n",
           bytes, ops, distinct(12), distinct(24), distinct(38), distinct(42));
    hipFree(buf);
    hipFree(out);
    return 0;
}
