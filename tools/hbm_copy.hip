// Achievable HBM rate of hand-written streaming kernels (read+write copy, read-only sum, write-only fill) for the
// roofline context in DESIGN §9. Not part of the product library: tools/hbm_calib.py builds and loads it.
//   hipcc --offload-arch=gfx950 -O3 -shared -fPIC tools/hbm_copy.hip -o tools/_hbm_copy.so
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

template <int U>
__global__ __launch_bounds__(256) void k_copy(const uint4* __restrict__ src, uint4* __restrict__ dst, long long n) {
    const long long stride = (long long)gridDim.x * 256 * U;
    for (long long i = (long long)blockIdx.x * 256 * U + threadIdx.x; i < n; i += stride) {
        uint4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = i + u * 256 < n ? src[i + u * 256] : make_uint4(0, 0, 0, 0);
#pragma unroll
        for (int u = 0; u < U; ++u)
            if (i + u * 256 < n) dst[i + u * 256] = v[u];
    }
}

template <int U>
__global__ __launch_bounds__(256) void k_read(const uint4* __restrict__ src, long long n, unsigned* out) {
    const long long stride = (long long)gridDim.x * 256 * U;
    unsigned acc = 0;
    for (long long i = (long long)blockIdx.x * 256 * U + threadIdx.x; i < n; i += stride) {
        uint4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = i + u * 256 < n ? src[i + u * 256] : make_uint4(0, 0, 0, 0);
#pragma unroll
        for (int u = 0; u < U; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
    }
    if (acc == 0x9e3779b9u) out[0] = acc;  // keeps the loads live; practically never stores
}

__global__ __launch_bounds__(256) void k_fill(uint4* __restrict__ dst, long long n) {
    const long long stride = (long long)gridDim.x * 256;
    for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) dst[i] = make_uint4(1, 2, 3, 4);
}

}  // namespace

// kind 0 copy, 1 read, 2 fill; n16 = 16-byte elements; returns the hipError_t of the launch
extern "C" int hbm_run(int kind, const void* src, void* dst, long long n16, int blocks, unsigned* out, void* stream) {
    hipStream_t s = (hipStream_t)stream;
    if (kind == 0)
        hipLaunchKernelGGL(k_copy<4>, dim3(blocks), dim3(256), 0, s, (const uint4*)src, (uint4*)dst, n16);
    else if (kind == 1)
        hipLaunchKernelGGL(k_read<4>, dim3(blocks), dim3(256), 0, s, (const uint4*)src, n16, out);
    else
        hipLaunchKernelGGL(k_fill, dim3(blocks), dim3(256), 0, s, (uint4*)dst, n16);
    return (int)hipGetLastError();
}
