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

// no per-element bounds checks (n16 a multiple of the grid's pass), nontemporal loads/stores on request: the
// guide's float4 copy (MI355X_MICROARCH.md: 6.29 TB/s) is this shape
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

template <int U, bool NT>
__global__ __launch_bounds__(256) void k_copy_nb(const u32x4* __restrict__ src, u32x4* __restrict__ dst, long long n) {
    const long long stride = (long long)gridDim.x * 256 * U;
    for (long long i = (long long)blockIdx.x * 256 * U + threadIdx.x; i < n; i += stride) {
        u32x4 v[U];
#pragma unroll
        for (int u = 0; u < U; ++u) v[u] = NT ? __builtin_nontemporal_load(src + i + u * 256) : src[i + u * 256];
#pragma unroll
        for (int u = 0; u < U; ++u) {
            if (NT) __builtin_nontemporal_store(v[u], dst + i + u * 256);
            else dst[i + u * 256] = v[u];
        }
    }
}

template <bool NT>
__global__ __launch_bounds__(256) void k_fill_nb(u32x4* __restrict__ dst, long long n) {
    const long long stride = (long long)gridDim.x * 256 * 4;
    const u32x4 v = {1u, 2u, 3u, 4u};
    for (long long i = (long long)blockIdx.x * 256 * 4 + threadIdx.x; i < n; i += stride)
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            if (NT) __builtin_nontemporal_store(v, dst + i + u * 256);
            else dst[i + u * 256] = v;
        }
}

}  // namespace

// kind 0 copy, 1 read, 2 fill; n16 = 16-byte elements; returns the hipError_t of the launch
extern "C" int hbm_run(int kind, const void* src, void* dst, long long n16, int blocks, unsigned* out, void* stream) {
    hipStream_t s = (hipStream_t)stream;
    if (kind == 0)
        hipLaunchKernelGGL(k_copy<4>, dim3(blocks), dim3(256), 0, s, (const uint4*)src, (uint4*)dst, n16);
    else if (kind == 1)
        hipLaunchKernelGGL(k_read<4>, dim3(blocks), dim3(256), 0, s, (const uint4*)src, n16, out);
    else if (kind == 2)
        hipLaunchKernelGGL(k_fill, dim3(blocks), dim3(256), 0, s, (uint4*)dst, n16);
    else if (kind == 3)  // 3-6: n16 must be a multiple of blocks * 256 * U (hbm_calib.py sizes it)
        hipLaunchKernelGGL((k_copy_nb<4, false>), dim3(blocks), dim3(256), 0, s, (const u32x4*)src, (u32x4*)dst, n16);
    else if (kind == 4)
        hipLaunchKernelGGL((k_copy_nb<4, true>), dim3(blocks), dim3(256), 0, s, (const u32x4*)src, (u32x4*)dst, n16);
    else if (kind == 5)
        hipLaunchKernelGGL((k_copy_nb<8, true>), dim3(blocks), dim3(256), 0, s, (const u32x4*)src, (u32x4*)dst, n16);
    else if (kind == 6)
        hipLaunchKernelGGL((k_fill_nb<true>), dim3(blocks), dim3(256), 0, s, (u32x4*)dst, n16);
    else if (kind == 7)
        hipLaunchKernelGGL((k_fill_nb<false>), dim3(blocks), dim3(256), 0, s, (u32x4*)dst, n16);
    return (int)hipGetLastError();
}
