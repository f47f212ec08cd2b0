// Shared device-side building blocks for libstereo_hip (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_bf16.h>
#include <stdint.h>

#include "../../include/stereo_hip.h"

typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef unsigned short u16x8 __attribute__((ext_vector_type(8)));
typedef float f32x8 __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) bf16x4 lds_bf16x4;

// ------------------------------------------------------------------ error plumbing (host)
void sd_set_error(const char* fmt, ...);
int sd_check_launch(const char* what);

#define SD_REQUIRE(cond, ...)          \
    do {                               \
        if (!(cond)) {                 \
            sd_set_error(__VA_ARGS__); \
            return SD_EINVAL;          \
        }                              \
    } while (0)

static inline hipStream_t to_stream(sd_stream s) { return reinterpret_cast<hipStream_t>(s); }

// BatchNorm layer whose backward sums a dgrad epilogue accumulates (sd_conv_gemm_bnsum -> conv_halo.hip)
struct HaloBnSum {
    const void* y;
    const float *scale, *shift, *mean, *invstd;
};

// BatchNorm-backward operands of the fused weight gradient (sd_wgrad_gemm_bnbwd -> conv_halo.hip)
struct HaloBnBwd {
    const void* da;
    const void* y;
    const float *scale, *shift, *mean, *invstd, *coef;
};

// ------------------------------------------------------------------ bilinear source index
// F.interpolate(mode="bilinear", align_corners=False) as ATen computes it (UpSample.h:
// area_pixel_compute_source_index + guard_index_and_lambda): s = (in/out)*(o+0.5)-0.5 clamped at
// 0, i0 = floor(s), i1 = i0+1 unless at the edge, lam = s - i0.
__device__ __forceinline__ void src_index(int o, int out_size, int in_size, int& i0, int& i1, float& lam) {
    const float scale = (float)in_size / (float)out_size;
    // one rounding, as torch's CPU kernel computes it (the compiler contracts it to an FMA there;
    // measured: identical to F.interpolate where two roundings differ by an ulp of s)
    float s = fmaf(scale, (float)o + 0.5f, -0.5f);
    if (s < 0.f) s = 0.f;
    i0 = (int)s;
    if (i0 > in_size - 1) i0 = in_size - 1;
    i1 = i0 + (i0 < in_size - 1 ? 1 : 0);
    lam = fminf(fmaxf(s - (float)i0, 0.f), 1.f);
}

// ------------------------------------------------------------------ division by a runtime constant
// n / d for n < 2^31 as a 64-bit multiply-high (d fixed per launch, m = ceil(2^(32+s) / d))
struct FastDiv {
    uint32_t d, s;
    uint64_t m;
};
static inline FastDiv make_fdiv(uint32_t d) {
    uint32_t s = 0;
    while ((1ull << s) < d) ++s;
    FastDiv f;
    f.d = d;
    f.s = s;
    f.m = ((1ull << (32 + s)) + d - 1) / d;
    return f;
}
__device__ __forceinline__ uint32_t fdiv(uint32_t n, const FastDiv& f) {
    return (uint32_t)(((uint64_t)n * f.m) >> (32 + f.s));
}

// ------------------------------------------------------------------ element conversion
__device__ __forceinline__ float to_f32(float x) { return x; }
__device__ __forceinline__ float to_f32(__bf16 x) { return (float)x; }
template <typename T> __device__ __forceinline__ T from_f32(float x);
template <> __device__ __forceinline__ float from_f32<float>(float x) { return x; }
template <> __device__ __forceinline__ __bf16 from_f32<__bf16>(float x) { return (__bf16)x; }

// 8 contiguous elements <-> 8 floats
__device__ __forceinline__ void load8(const float* p, float (&v)[8]) {
    const float4 a = *reinterpret_cast<const float4*>(p);
    const float4 b = *reinterpret_cast<const float4*>(p + 4);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}
__device__ __forceinline__ void load8(const __bf16* p, float (&v)[8]) {
    const uint4 r = *reinterpret_cast<const uint4*>(p);
    const unsigned w[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        v[2 * i] = __uint_as_float(w[i] << 16);
        v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
    }
}
__device__ __forceinline__ void store8(float* p, const float (&v)[8]) {
    *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
    *reinterpret_cast<float4*>(p + 4) = make_float4(v[4], v[5], v[6], v[7]);
}
__device__ __forceinline__ void store8(__bf16* p, const float (&v)[8]) {
    bf16x8 b;
#pragma unroll
    for (int i = 0; i < 8; ++i) b[i] = (__bf16)v[i];
    *reinterpret_cast<bf16x8*>(p) = b;
}
// Streaming output stores of the elementwise kernels (pool backward, BN-backward apply, heads' da, pooled
// activations, ConvTranspose outputs). Nontemporal (SD_NT_STORES=1) measured 0.6 % slower on the step (same-box A/B,
// 3 rounds: 6945 vs 6987 pairs/s), unlike the halo conv's epilogue (conv_halo.hip HC_ST_AUX), whose L2 holds re-read
// weight and halo rows: these kernels re-read nothing, and their outputs are read by the next kernel soon enough to
// hit in the 256 MB Infinity Cache. Default: plain stores.
#ifndef SD_NT_STORES
#define SD_NT_STORES 0
#endif
typedef unsigned u32x4_nt __attribute__((ext_vector_type(4)));
__device__ __forceinline__ void store16_nt(void* p, uint4 v) {
    if (SD_NT_STORES)
        __builtin_nontemporal_store(u32x4_nt{v.x, v.y, v.z, v.w}, reinterpret_cast<u32x4_nt*>(p));
    else
        *reinterpret_cast<uint4*>(p) = v;
}
__device__ __forceinline__ void store8_nt(float* p, const float (&v)[8]) { store8(p, v); }
__device__ __forceinline__ void store8_nt(__bf16* p, const float (&v)[8]) {
    bf16x8 b;
#pragma unroll
    for (int i = 0; i < 8; ++i) b[i] = (__bf16)v[i];
    store16_nt(p, *reinterpret_cast<uint4*>(&b));
}
__device__ __forceinline__ void zero8(float (&v)[8]) {
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = 0.f;
}

// ------------------------------------------------------------------ MFMA per element type
// fp32 parity mode : v_mfma_f32_16x16x4_f32  (exact f32 fma chain), lane holds A[l&15][l>>4]
// bf16 mode        : v_mfma_f32_16x16x32_bf16, lane holds A[l&15][8*(l>>4) + j], j < 8
// C/D (both)       : row = 4*(l>>4) + r, col = l&15
template <typename T> struct Mfma;
template <> struct Mfma<float> {
    static constexpr int KPL = 1;    // k elements per lane per MFMA
    static constexpr int KSTEP = 4;  // k per MFMA
    using frag = float;
    __device__ __forceinline__ static f32x4 mma(frag a, frag b, f32x4 c) {
        return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
    }
};
template <> struct Mfma<__bf16> {
    static constexpr int KPL = 8;
    static constexpr int KSTEP = 32;
    using frag = bf16x8;
    __device__ __forceinline__ static f32x4 mma(frag a, frag b, f32x4 c) {
        return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
    }
};

// fragment read from an LDS tile stored k-contiguous: tile[row][k], row stride `ld` elements
__device__ __forceinline__ float frag_row(const float* lds, int ld, int row, int k) { return lds[row * ld + k]; }
__device__ __forceinline__ bf16x8 frag_row(const __bf16* lds, int ld, int row, int k) {
    return *reinterpret_cast<const bf16x8*>(lds + row * ld + k);
}
// fragment read from an LDS tile stored [k][col] (k = pixel rows): operand[col][k0 + KPL*(l>>4) + j]
__device__ __forceinline__ float frag_tr(const float* lds, int ld, int col, int k0, int lane) {
    return lds[(k0 + (lane >> 4)) * ld + col];
}
// bf16: two ds_read_b64_tr_b16; within a 16-lane group, lane 4q+p supplies row q, columns 4p..4p+3
__device__ __forceinline__ bf16x8 frag_tr(const __bf16* lds, int ld, int col0, int k0, int lane) {
    const int i = lane & 15, g = lane >> 4;
    const int q = i >> 2, p = i & 3;
    const __bf16* a0 = lds + (k0 + 8 * g + q) * ld + col0 + 4 * p;
    const __bf16* a1 = a0 + 4 * ld;
    bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(a0));
    bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(a1));
    bf16x8 r;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        r[j] = lo[j];
        r[j + 4] = hi[j];
    }
    return r;
}

// ------------------------------------------------------------------ implicit-GEMM gather
// Device copy of sd_src with derived fields.
struct GatherSrc {
    const void* ptr0;
    const void* ptr1;
    const float* sc0;
    const float* sh0;
    const float* sc1;
    const float* sh1;
    int c0, c1;      // channels of each source
    int x0, x1;      // transforms
    int H, W;        // stored dims of the sources
    int Hl, Wl;      // logical grid of the tap addressing (pooled dims when pool)
    int taps, pool;
    int cpt;         // chunks (of 8 channels) per tap
    int kchunks;     // taps * cpt
};

static inline GatherSrc make_gather(const sd_src& s) {
    GatherSrc g;
    g.ptr0 = s.ptr[0];
    g.ptr1 = s.ptr[1];
    g.sc0 = s.scale[0];
    g.sh0 = s.shift[0];
    g.sc1 = s.scale[1];
    g.sh1 = s.shift[1];
    g.c0 = s.chans[0];
    g.c1 = s.chans[1];
    g.x0 = s.xform[0];
    g.x1 = s.xform[1];
    g.H = s.H;
    g.W = s.W;
    g.pool = s.pool;
    g.taps = s.taps;
    g.Hl = s.pool ? s.H / 2 : s.H;
    g.Wl = s.pool ? s.W / 2 : s.W;
    g.cpt = (s.chans[0] + s.chans[1]) / 8;
    g.kchunks = g.taps * g.cpt;
    return g;
}

__device__ __forceinline__ void xform8(float (&v)[8], const float* sc, const float* sh, int c) {
    const float4 s0 = *reinterpret_cast<const float4*>(sc + c);
    const float4 s1 = *reinterpret_cast<const float4*>(sc + c + 4);
    const float4 h0 = *reinterpret_cast<const float4*>(sh + c);
    const float4 h1 = *reinterpret_cast<const float4*>(sh + c + 4);
    const float s[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
    const float h[8] = {h0.x, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, h1.w};
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = fmaxf(__builtin_fmaf(v[i], s[i], h[i]), 0.f);
}

// 8 channels [c, c+8) of one source pixel (stored coords), with transform
template <typename T>
__device__ __forceinline__ void fetch8(const T* base, int C, int xf, const float* sc, const float* sh, int b, int H,
                                       int W, int h, int w, int c, float (&v)[8]) {
    load8(base + ((size_t)((size_t)b * H + h) * W + w) * C + c, v);
    if (xf == SD_BNRELU) xform8(v, sc, sh, c);
}

// Gather chunk `q` (8 consecutive K elements) for GEMM-grid pixel (b, h, w).
template <typename T>
__device__ __forceinline__ void gather_chunk(const GatherSrc& g, int b, int h, int w, int q, float (&v)[8]) {
    if (q >= g.kchunks) {
        zero8(v);
        return;
    }
    const int tap = q / g.cpt;
    int c = (q - tap * g.cpt) * 8;
    int gh, gw;
    if (g.taps == 9) {
        gh = h + tap / 3 - 1;
        gw = w + tap % 3 - 1;
    } else if (g.taps == 4) {
        gh = 2 * h + (tap >> 1);
        gw = 2 * w + (tap & 1);
    } else {
        gh = h;
        gw = w;
    }
    if (gh < 0 || gw < 0 || gh >= g.Hl || gw >= g.Wl) {
        zero8(v);
        return;
    }
    const T* base;
    int C, xf;
    const float *sc, *sh;
    if (c < g.c0) {
        base = (const T*)g.ptr0; C = g.c0; xf = g.x0; sc = g.sc0; sh = g.sh0;
    } else {
        c -= g.c0;
        base = (const T*)g.ptr1; C = g.c1; xf = g.x1; sc = g.sc1; sh = g.sh1;
    }
    if (!g.pool) {
        fetch8<T>(base, C, xf, sc, sh, b, g.H, g.W, gh, gw, c, v);
    } else {
        float t[8];
        fetch8<T>(base, C, xf, sc, sh, b, g.H, g.W, 2 * gh, 2 * gw, c, v);
        fetch8<T>(base, C, xf, sc, sh, b, g.H, g.W, 2 * gh, 2 * gw + 1, c, t);
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = fmaxf(v[i], t[i]);
        fetch8<T>(base, C, xf, sc, sh, b, g.H, g.W, 2 * gh + 1, 2 * gw, c, t);
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = fmaxf(v[i], t[i]);
        fetch8<T>(base, C, xf, sc, sh, b, g.H, g.W, 2 * gh + 1, 2 * gw + 1, c, t);
#pragma unroll
        for (int i = 0; i < 8; ++i) v[i] = fmaxf(v[i], t[i]);
    }
}

static inline int cdiv(long long a, long long b) { return (int)((a + b - 1) / b); }

// fp64 block sum of (a, b) over NT threads, the result in every thread (BatchNorm finalizes, the row sums of
// sd_wgrad_reduce_batch); one fixed summation order
template <int NT>
__device__ __forceinline__ void block_sum2(double& a, double& b) {
    static_assert(NT >= 64 && (NT & (NT - 1)) == 0, "whole waves, a power of two");
    // the tree t += t + s for s = NT/2 .. 1: the steps across waves through LDS, the last six (s < 64) as shuffles in
    // wave 0 with the same pairs and order (bit-identical sums; 8 -> 3 barriers: these launches are latency-bound)
    __shared__ double red[2][NT];
    red[0][threadIdx.x] = a;
    red[1][threadIdx.x] = b;
    __syncthreads();
    for (int s = NT / 2; s >= 64; s >>= 1) {
        if (threadIdx.x < s) {
            red[0][threadIdx.x] += red[0][threadIdx.x + s];
            red[1][threadIdx.x] += red[1][threadIdx.x + s];
        }
        __syncthreads();
    }
    if (threadIdx.x < 64) {
        double x = red[0][threadIdx.x], y = red[1][threadIdx.x];
#pragma unroll
        for (int s = 32; s > 0; s >>= 1) {
            x += __shfl_down(x, s);
            y += __shfl_down(y, s);
        }
        if (threadIdx.x == 0) {
            red[0][0] = x;
            red[1][0] = y;
        }
    }
    __syncthreads();
    a = red[0][0];
    b = red[1][0];
}
