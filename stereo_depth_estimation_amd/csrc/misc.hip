// Library plumbing, weight/input packing, fused AdamW and the bilinear resize of the data path.
#include <math.h>
#include <stdarg.h>
#include <stdio.h>

#include "common.h"

static thread_local char g_err[512] = "";

void sd_set_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}

int sd_check_launch(const char* what) {
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) {
        sd_set_error("%s: %s", what, hipGetErrorString(e));
        return SD_EHIP;
    }
    return SD_OK;
}

extern "C" int sd_version(void) { return 100; }
extern "C" const char* sd_last_error(void) { return g_err; }
extern "C" int sd_device_init(int device) {
    if (hipSetDevice(device) != hipSuccess) return sd_check_launch("sd_device_init");
    return SD_OK;
}

// Effective shader clock under MFMA load (bench.py "clock"): every block runs 4 waves of back-to-back
// v_mfma_f32_32x32x16_bf16 (4 independent accumulator chains per wave) and wave 0 stamps the shader-clock counter
// (s_memtime) and the 100 MHz constant clock (s_memrealtime) around its loop: clock = d(memtime) / d(realtime) * 100
// MHz. One block per CU loads the whole chip the way the persistent conv kernels do. out[4 * block + {0..3}] = (memtime
// start, memtime end, realtime start, realtime end).
typedef float f32x16_t __attribute__((ext_vector_type(16)));
__global__ __launch_bounds__(256) void k_clock_probe(int iters, unsigned long long* __restrict__ out,
                                                     float* __restrict__ sink) {
    const int lane = threadIdx.x & 63;
    bf16x8 a, b;
#pragma unroll
    for (int i = 0; i < 8; ++i) {  // random-looking operands (the power draw of real data, not of zeros)
        a[i] = (__bf16)(((lane * 37 + i * 11) % 17) * 0.0625f - 0.5f);
        b[i] = (__bf16)(((lane * 13 + i * 7) % 19) * 0.0625f - 0.55f);
    }
    f32x16_t acc[4] = {};
    __syncthreads();
    const unsigned long long t0 = __builtin_amdgcn_s_memtime(), r0 = __builtin_amdgcn_s_memrealtime();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int c = 0; c < 4; ++c) acc[c] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc[c], 0, 0, 0);
    }
    float s = 0.f;
#pragma unroll
    for (int c = 0; c < 4; ++c) s += acc[c][0] + acc[c][15];
    const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
    if (s == 12345.f) sink[threadIdx.x] = s;  // keeps the chains live
    if (threadIdx.x == 0) {
        out[4 * blockIdx.x] = t0;
        out[4 * blockIdx.x + 1] = t1;
        out[4 * blockIdx.x + 2] = r0;
        out[4 * blockIdx.x + 3] = r1;
    }
}

extern "C" int sd_clock_probe(int blocks, int iters, unsigned long long* out, float* sink, sd_stream s) {
    SD_REQUIRE(blocks > 0 && iters > 0 && out && sink, "sd_clock_probe: bad args");
    hipLaunchKernelGGL(k_clock_probe, dim3(blocks), dim3(256), 0, to_stream(s), iters, out, sink);
    return sd_check_launch("sd_clock_probe");
}

namespace {

// ------------------------------------------------------------------ packing
// one pixel per thread: coalesced plane reads (consecutive threads, consecutive pixels), one 8-channel
// vector store per 8 output channels
template <typename T>
__device__ __forceinline__ void pack_input_blocks(const float* __restrict__ x, int batch, int cin, int H, int W, int cpad,
                                                  T* out, int bid, int nblk) {
    const long long P = (long long)batch * H * W;
    const long long hw = (long long)H * W;
    for (long long px = bid * 256LL + threadIdx.x; px < P; px += (long long)nblk * 256) {
        const long long b = px / hw, r = px - b * hw;
        const float* src = x + b * cin * hw + r;
        for (int c0 = 0; c0 < cpad; c0 += 8) {
            float v[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) v[i] = c0 + i < cin ? src[(c0 + i) * hw] : 0.f;
            store8(out + px * cpad + c0, v);
        }
    }
}
// The same for H*W % 4 == 0 and a 16-B aligned x: four consecutive pixels per thread, one 16-B load per channel plane
// (the scalar form kept only 4 B per lane and plane in flight and ran the B = 64 320x240 pack at ~4 TB/s)
template <typename T>
__device__ __forceinline__ void pack_input_blocks4(const float* __restrict__ x, int batch, int cin, int H, int W,
                                                   int cpad, T* out, int bid, int nblk) {
    const long long hw = (long long)H * W, Q = (long long)batch * hw / 4;
    for (long long q = bid * 256LL + threadIdx.x; q < Q; q += (long long)nblk * 256) {
        const long long px = 4 * q, b = px / hw, r = px - b * hw;
        const float* src = x + b * cin * hw + r;
        for (int c0 = 0; c0 < cpad; c0 += 8) {
            float4 v[8];
#pragma unroll
            for (int i = 0; i < 8; ++i)
                v[i] = c0 + i < cin ? *reinterpret_cast<const float4*>(src + (c0 + i) * hw) : make_float4(0, 0, 0, 0);
            const float p0[8] = {v[0].x, v[1].x, v[2].x, v[3].x, v[4].x, v[5].x, v[6].x, v[7].x};
            const float p1[8] = {v[0].y, v[1].y, v[2].y, v[3].y, v[4].y, v[5].y, v[6].y, v[7].y};
            const float p2[8] = {v[0].z, v[1].z, v[2].z, v[3].z, v[4].z, v[5].z, v[6].z, v[7].z};
            const float p3[8] = {v[0].w, v[1].w, v[2].w, v[3].w, v[4].w, v[5].w, v[6].w, v[7].w};
            store8(out + px * cpad + c0, p0);
            store8(out + (px + 1) * cpad + c0, p1);
            store8(out + (px + 2) * cpad + c0, p2);
            store8(out + (px + 3) * cpad + c0, p3);
        }
    }
}
template <typename T>
__global__ void k_pack_input(const float* __restrict__ x, int batch, int cin, int H, int W, int cpad, T* out) {
    pack_input_blocks(x, batch, cin, H, W, cpad, out, blockIdx.x, gridDim.x);
}
template <typename T>
__global__ void k_pack_input4(const float* __restrict__ x, int batch, int cin, int H, int W, int cpad, T* out) {
    pack_input_blocks4(x, batch, cin, H, W, cpad, out, blockIdx.x, gridDim.x);
}

// k_pack_input that also takes max |x| over the batch (the fp8 path's input-range check, engine._fp8_policy): per-block
// reduce, one atomicMax of the float bits (|x| >= 0 orders like its bits) into amax[slot]; block 0 clears amax[clear]
// for a later frame (the caller orders this kernel after the host's read-back of that slot)
template <typename T>
__global__ __launch_bounds__(256) void k_pack_input_amax(const float* __restrict__ x, int batch, int cin, int H, int W,
                                                         int cpad, T* out, unsigned* amax, int slot, int clear) {
    const long long P = (long long)batch * H * W;
    const long long hw = (long long)H * W;
    float m = 0.f;
    for (long long px = blockIdx.x * 256LL + threadIdx.x; px < P; px += (long long)gridDim.x * 256) {
        const long long b = px / hw, r = px - b * hw;
        const float* src = x + b * cin * hw + r;
        for (int c0 = 0; c0 < cpad; c0 += 8) {
            float v[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                v[i] = c0 + i < cin ? src[(c0 + i) * hw] : 0.f;
                m = fmaxf(m, fabsf(v[i]));
            }
            store8(out + px * cpad + c0, v);
        }
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) m = fmaxf(m, __shfl_xor(m, o));
    __shared__ float wm[4];
    if ((threadIdx.x & 63) == 0) wm[threadIdx.x >> 6] = m;
    __syncthreads();
    if (threadIdx.x == 0) {  // skip the atomic unless this block raises the max (few blocks do: no contention)
        const unsigned mb = __float_as_uint(fmaxf(fmaxf(wm[0], wm[1]), fmaxf(wm[2], wm[3])));
        if (mb > __hip_atomic_load(amax + slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) atomicMax(amax + slot, mb);
    }
    if (blockIdx.x == 0 && threadIdx.x == 64 && clear >= 0) amax[clear] = 0u;
}

// fwd : out[o][tap*ci_pad + i] = w[o][i][tap]
// dgrad: out[i][tap*co + o]    = w[o][i][8 - tap]
template <typename T>
__global__ void k_pack_conv3(const float* __restrict__ w, int co, int ci, int ci_pad, int dgrad, int kpad, T* out) {
    const int rows = dgrad ? ci : co;
    const long long total = (long long)rows * kpad;
    for (long long e = blockIdx.x * 256LL + threadIdx.x; e < total; e += (long long)gridDim.x * 256) {
        const int r = (int)(e / kpad), k = (int)(e % kpad);
        float v = 0.f;
        if (!dgrad) {
            const int tap = k / ci_pad, i = k % ci_pad;
            if (tap < 9 && i < ci) v = w[((size_t)r * ci + i) * 9 + tap];
        } else {
            const int tap = k / co, o = k % co;
            if (tap < 9) v = w[((size_t)o * ci + r) * 9 + (8 - tap)];
        }
        out[e] = from_f32<T>(v);
    }
}

// fwd : out[t*co + o][i] = w[i][o][t];   dgrad: out[i][t*co + o] = w[i][o][t]
template <typename T>
__global__ void k_pack_convT(const float* __restrict__ w, int ci, int co, int dgrad, int kpad, T* out) {
    const int rows = dgrad ? ci : 4 * co;
    const long long total = (long long)rows * kpad;
    for (long long e = blockIdx.x * 256LL + threadIdx.x; e < total; e += (long long)gridDim.x * 256) {
        const int r = (int)(e / kpad), k = (int)(e % kpad);
        float v = 0.f;
        if (!dgrad) {
            const int t = r / co, o = r % co;
            if (k < ci) v = w[((size_t)k * co + o) * 4 + t];
        } else {
            const int t = k / co, o = k % co;
            if (t < 4) v = w[((size_t)r * co + o) * 4 + t];
        }
        out[e] = from_f32<T>(v);
    }
}

// all weight packs of a step in one launch: jobs in the kernel arguments, each job a contiguous
// range of blocks (first[j] = its first block; a block finds its job by binary search). A block
// owns one output row group: it stages the fp32 source weights that row needs into LDS with
// contiguous loads, then writes the packed row(s) contiguously (a direct per-element gather read
// each 4-B weight through its own cache line: 20x the source bytes, measured with FETCH_SIZE).
//   conv3 fwd   : out row o      <- w[o][0:ci][0:9]            (contiguous ci*9 floats)
//   conv3 dgrad : out row i      <- w[0:co][i][0:9]            (co pieces of 9 floats)
//   convT fwd   : out rows (t,o), t = 0..3 <- w[0:ci][o][0:4]  (ci pieces of 4 floats)
//   convT dgrad : out row i      <- w[i][0:co][0:4]            (contiguous co*4 floats)
constexpr int PACK_MAX_JOBS = 64;
constexpr int PACK_LDS_FLOATS = 512 * 9;  // the largest staged source (ci or co <= 512)
struct PackJobs {
    sd_pack_job j[PACK_MAX_JOBS];
    int first[PACK_MAX_JOBS + 1];
    int n;
};
// the hi (lo = 0) or lo (lo = 1) bf16 half of v: hi = bf16(v), lo = bf16(v - hi) (v - hi is exact in fp32), so
// hi + lo carries ~16 significant bits of v (the split packs; bf16 only)
template <typename T>
__device__ __forceinline__ T split_half(float v, int lo) {
    const float hi = (float)from_f32<T>(v);
    return from_f32<T>(lo ? v - hi : v);
}
template <typename T>
__device__ __forceinline__ void pack_multi_block(const PackJobs& P, T* __restrict__ out, int bid, float* sw) {
    int lo = 0, hi = P.n - 1;  // largest j with first[j] <= bid
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (P.first[mid] <= bid) lo = mid; else hi = mid - 1;
    }
    const sd_pack_job& jb = P.j[lo];
    const int r = bid - P.first[lo];  // row (group) of this block
    const int tid = threadIdx.x;
    T* o = out + jb.out_off;
    const int co = jb.co, ci = jb.ci;
    switch (jb.kind) {
        case SD_PACK_CONV3_FWD: {  // out[r][tap*ci_pad + i] = w[r][i][tap]
            const float* src = jb.w + (size_t)r * ci * 9;
            for (int e = tid; e < ci * 9; e += 256) sw[e] = src[e];
            __syncthreads();
            for (int k = tid; k < jb.kpad; k += 256) {
                const int tap = k / jb.ci_pad, i = k - tap * jb.ci_pad;
                o[(size_t)r * jb.kpad + k] = from_f32<T>(tap < 9 && i < ci ? sw[i * 9 + tap] : 0.f);
            }
            break;
        }
        case SD_PACK_CONV3_DGRAD: {  // out[r][tap*co + oo] = w[oo][r][8 - tap]
            for (int e = tid; e < co * 9; e += 256) {
                const int oo = e / 9, t = e - oo * 9;
                sw[e] = jb.w[((size_t)oo * ci + r) * 9 + t];
            }
            __syncthreads();
            for (int k = tid; k < jb.kpad; k += 256) {
                const int tap = k / co, oo = k - tap * co;
                o[(size_t)r * jb.kpad + k] = from_f32<T>(tap < 9 ? sw[oo * 9 + (8 - tap)] : 0.f);
            }
            break;
        }
        case SD_PACK_CONVT_FWD: {  // out[t*co + r][i] = w[i][r][t], t = 0..3
            for (int e = tid; e < ci * 4; e += 256) {
                const int i = e >> 2, t = e & 3;
                sw[e] = jb.w[((size_t)i * co + r) * 4 + t];
            }
            __syncthreads();
            for (int q = tid; q < 4 * jb.kpad; q += 256) {
                const int t = q / jb.kpad, k = q - t * jb.kpad;
                o[(size_t)(t * co + r) * jb.kpad + k] = from_f32<T>(k < ci ? sw[k * 4 + t] : 0.f);
            }
            break;
        }
        case SD_PACK_CONV3_FWD_SPLIT: {  // out[r][tap*2ci_pad + {i | ci_pad + i}] = {hi | lo}(w[r][i][tap])
            const float* src = jb.w + (size_t)r * ci * 9;
            for (int e = tid; e < ci * 9; e += 256) sw[e] = src[e];
            __syncthreads();
            const int wct = 2 * jb.ci_pad;
            for (int k = tid; k < jb.kpad; k += 256) {
                const int tap = k / wct, rem = k - tap * wct, lo = rem >= jb.ci_pad, i = rem - lo * jb.ci_pad;
                o[(size_t)r * jb.kpad + k] = split_half<T>(tap < 9 && i < ci ? sw[i * 9 + tap] : 0.f, lo);
            }
            break;
        }
        case SD_PACK_CONVT_FWD_SPLIT: {  // out[t*co + r][{i | ci + i}] = {hi | lo}(w[i][r][t]), t = 0..3
            for (int e = tid; e < ci * 4; e += 256) {
                const int i = e >> 2, t = e & 3;
                sw[e] = jb.w[((size_t)i * co + r) * 4 + t];
            }
            __syncthreads();
            for (int q = tid; q < 4 * jb.kpad; q += 256) {
                const int t = q / jb.kpad, k = q - t * jb.kpad, lo = k >= ci, i = k - lo * ci;
                o[(size_t)(t * co + r) * jb.kpad + k] = split_half<T>(i < ci ? sw[i * 4 + t] : 0.f, lo);
            }
            break;
        }
        default: {  // SD_PACK_CONVT_DGRAD: out[r][t*co + oo] = w[r][oo][t]
            const float* src = jb.w + (size_t)r * co * 4;
            for (int e = tid; e < co * 4; e += 256) sw[e] = src[e];
            __syncthreads();
            for (int k = tid; k < jb.kpad; k += 256) {
                const int t = k / co, oo = k - t * co;
                o[(size_t)r * jb.kpad + k] = from_f32<T>(t < 4 ? sw[oo * 4 + t] : 0.f);
            }
        }
    }
}
template <typename T>
__global__ __launch_bounds__(256) void k_pack_multi(const PackJobs P, T* __restrict__ out) {
    __shared__ float sw[PACK_LDS_FLOATS];
    pack_multi_block(P, out, blockIdx.x, sw);
}

// ------------------------------------------------------------------ valid-pixel count (train.py:329-330)
// 4 pixels per thread per iteration (one 32-bit mask word, one float4 of targets), block reduction, one atomic per
// block and counter
__device__ __forceinline__ void count_valid_blocks(const float* __restrict__ t, const uint8_t* __restrict__ m,
                                                   long long P, int* count, int ncount, int* clear, int bid, int nblk) {
    // clear: the other slot of the caller's double-buffered counters, zeroed for its next call (no memset launch)
    if (clear && bid == 0 && threadIdx.x < ncount) clear[threadIdx.x] = 0;
    int c = 0;
    const long long P4 = P / 4;
    auto cnt = [](unsigned mw, float4 tv) {
        return ((mw & 0xffu) != 0 && isfinite(tv.x)) + (((mw >> 8) & 0xffu) != 0 && isfinite(tv.y)) +
               (((mw >> 16) & 0xffu) != 0 && isfinite(tv.z)) + ((mw >> 24) != 0 && isfinite(tv.w));
    };
    // four passes' loads issued together: each pass was a dependent HBM round trip (the 4.9 M pixels of a 320x240
    // B = 64 step took 5 of them at 1024 blocks, 29 us for 25 MB)
    const long long stride = (long long)nblk * 256;
    long long i = bid * 256LL + threadIdx.x;
    for (; i + 3 * stride < P4; i += 4 * stride) {
        unsigned mw[4];
        float4 tv[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            mw[k] = reinterpret_cast<const unsigned*>(m)[i + k * stride];
            tv[k] = reinterpret_cast<const float4*>(t)[i + k * stride];
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) c += cnt(mw[k], tv[k]);
    }
    for (; i < P4; i += stride) c += cnt(reinterpret_cast<const unsigned*>(m)[i], reinterpret_cast<const float4*>(t)[i]);
    for (long long i = P4 * 4 + bid * 256LL + threadIdx.x; i < P; i += (long long)nblk * 256)
        c += (m[i] != 0 && isfinite(t[i])) ? 1 : 0;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o);
    __shared__ int red[4];
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = c;
    __syncthreads();
    // the counters' atomics from different lanes (they serialize per address, not across addresses)
    if (threadIdx.x < ncount) {
        const int s = red[0] + red[1] + red[2] + red[3];
        if (s) atomicAdd(count + threadIdx.x, s);
    }
}
__global__ __launch_bounds__(256) void k_count_valid(const float* __restrict__ t, const uint8_t* __restrict__ m,
                                                     long long P, int* count, int ncount, int* clear) {
    count_valid_blocks(t, m, P, count, ncount, clear, blockIdx.x, gridDim.x);
}
__global__ __launch_bounds__(256) void k_count_valid_scalar(const float* __restrict__ t, const uint8_t* __restrict__ m,
                                                            long long P, int* count, int ncount) {
    int c = 0;
    for (long long i = blockIdx.x * 256LL + threadIdx.x; i < P; i += (long long)gridDim.x * 256)
        c += (m[i] != 0 && isfinite(t[i])) ? 1 : 0;
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o);
    if ((threadIdx.x & 63) == 0 && c)
        for (int k = 0; k < ncount; ++k) atomicAdd(count + k, c);
}

// ------------------------------------------------------------------ the train step's prologue in one launch
// blocks [0, nb_cnt): the valid count (latency-bound: dispatched first); the rest the weight packs (one LDS-staged
// row per block: latency-bound) and the input pack (HBM-bound, vec4: four pixels per thread) interleaved evenly in
// dispatch order, so every CU runs both kinds side by side (r05 dispatched all pack blocks before the input pack:
// 91.7 us for ~0.3 GB, about the sum of the three former launches); three independent jobs whose launches were three
// kernel boundaries
template <typename T>
__global__ __launch_bounds__(256) void k_step_prologue(const PackJobs P, T* __restrict__ wout, int nb_pack,
                                                       const float* __restrict__ x, int batch, int cin, int H, int W,
                                                       int cpad, T* __restrict__ xout, int nb_in, int vec4,
                                                       const float* __restrict__ t, const uint8_t* __restrict__ m,
                                                       long long pixels, int* count, int ncount, int* clear,
                                                       int nb_cnt) {
    __shared__ float sw[PACK_LDS_FLOATS];
    const int b = blockIdx.x;
    if (b < nb_cnt) {
        count_valid_blocks(t, m, pixels, count, ncount, clear, b, nb_cnt);
        return;
    }
    // Bresenham interleave: among the first j + 1 of the remaining blocks, np(j) = (j + 1) * nb_pack / tot are packs
    const long long j = b - nb_cnt, tot = (long long)nb_pack + nb_in;
    const long long np = (j + 1) * nb_pack / tot, np0 = j * nb_pack / tot;
    if (np > np0) {
        pack_multi_block(P, wout, (int)np0, sw);
        return;
    }
    if (vec4) pack_input_blocks4(x, batch, cin, H, W, cpad, xout, (int)(j - np0), nb_in);
    else pack_input_blocks(x, batch, cin, H, W, cpad, xout, (int)(j - np0), nb_in);
}

// ------------------------------------------------------------------ AdamW
struct AdamScalars {
    float decay;      // 1 - lr*wd
    float step_size;  // lr / (1 - b1^t)
    float bc2_sqrt;   // sqrt(1 - b2^t)
};

// the step's scalars from step t in fp64 (outside the contract(off) region below: the same code the former one-thread
// prep launch ran, so the updates are unchanged)
__device__ __forceinline__ AdamScalars adam_scalars(int t, double lr, double wd, double b1, double b2) {
    const double bc1 = 1.0 - pow(b1, (double)t);
    const double bc2 = 1.0 - pow(b2, (double)t);
    return AdamScalars{(float)(1.0 - lr * wd), (float)(lr / bc1), (float)sqrt(bc2)};
}

// One launch per step: every block derives the scalars from *step itself, and the step counter advances once every
// block has read it: each block counts itself out on `done` (an agent-scope relaxed add after a barrier, so all of
// its waves have read *step), and the block that counts last writes step + 1 and re-arms the counter. Skipped
// steps (*count == 0, train.py:331-332) touch neither. The per-block cost of this hand-off (the counter add and the
// scalar evaluation: 8192 blocks took 103 us against 41 us at 1024, tools/adamw_micro.py; three group counters
// measured the same) caps the grid at 1024 blocks, grid-stride (SD_ADAM_BLOCKS overrides).
#pragma clang fp contract(off)
__global__ __launch_bounds__(256) void k_adamw(float* __restrict__ p, const float* __restrict__ g,
                                               float* __restrict__ m, float* __restrict__ v, long long n, float w1,
                                               float b2, float w2, float eps, int* step, const int* count, double lr,
                                               double wd, double b1d, double b2d, unsigned* done) {
    if (count != nullptr && *count == 0) return;
    const int t = *step + 1;
    __shared__ AdamScalars scs;  // one thread per block evaluates the fp64 pows
    if (threadIdx.x == 0) scs = adam_scalars(t, lr, wd, b1d, b2d);
    __syncthreads();
    const float decay = scs.decay, step_size = scs.step_size, bc2s = scs.bc2_sqrt;
    for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
        const float gi = g[i];
        float pi = p[i] * decay;                  // param.mul_(1 - lr*wd)
        float mi = m[i];
        mi = mi + w1 * (gi - mi);                 // exp_avg.lerp_(grad, 1-b1)
        float vi = v[i] * b2;                     // exp_avg_sq.mul_(b2)
        vi = vi + w2 * gi * gi;                   //   .addcmul_(grad, grad, 1-b2)
        const float denom = sqrtf(vi) / bc2s + eps;
        pi = pi + (-step_size) * (mi / denom);    // param.addcdiv_(exp_avg, denom, -step_size)
        p[i] = pi;
        m[i] = mi;
        v[i] = vi;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned prev = __hip_atomic_fetch_add(done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (prev == gridDim.x - 1) {
            *step = t;
            __hip_atomic_store(done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

#pragma clang fp contract(on)

// ------------------------------------------------------------------ bilinear resize (align_corners=False)
__global__ void k_resize_bilinear(const float* __restrict__ in, int planes, int Hi, int Wi, float* __restrict__ out,
                                  int Ho, int Wo, float mul) {
    const long long total = (long long)planes * Ho * Wo;
    for (long long e = blockIdx.x * 256LL + threadIdx.x; e < total; e += (long long)gridDim.x * 256) {
        const int x = (int)(e % Wo);
        const long long t = e / Wo;
        const int y = (int)(t % Ho), pl = (int)(t / Ho);
        int y0, y1, x0, x1;
        float ly, lx;
        src_index(y, Ho, Hi, y0, y1, ly);
        src_index(x, Wo, Wi, x0, x1, lx);
        const float* src = in + (size_t)pl * Hi * Wi;
        const float v = (1.f - ly) * ((1.f - lx) * src[y0 * Wi + x0] + lx * src[y0 * Wi + x1]) +
                        ly * ((1.f - lx) * src[y1 * Wi + x0] + lx * src[y1 * Wi + x1]);
        out[e] = v * mul;
    }
}

int grid_for(long long work) {
    long long g = (work + 255) / 256;
    if (g > 8192) g = 8192;
    return (int)(g < 1 ? 1 : g);
}

}  // namespace

extern "C" int sd_pack_input(int dtype, const float* x, int batch, int cin, int H, int W, int cpad, void* out,
                             sd_stream s) {
    SD_REQUIRE(x && out && batch > 0 && cin > 0 && H > 0 && W > 0, "sd_pack_input: bad args");
    SD_REQUIRE(cpad >= cin && cpad % 8 == 0, "sd_pack_input: cpad %d", cpad);
    const bool vec4 = ((long long)H * W) % 4 == 0 && (uintptr_t)x % 16 == 0;
    const int g = grid_for((long long)batch * H * W / (vec4 ? 4 : 1));
    if (dtype == SD_BF16)
        hipLaunchKernelGGL(vec4 ? k_pack_input4<__bf16> : k_pack_input<__bf16>, dim3(g), dim3(256), 0, to_stream(s), x,
                           batch, cin, H, W, cpad, (__bf16*)out);
    else
        hipLaunchKernelGGL(vec4 ? k_pack_input4<float> : k_pack_input<float>, dim3(g), dim3(256), 0, to_stream(s), x,
                           batch, cin, H, W, cpad, (float*)out);
    return sd_check_launch("sd_pack_input");
}

extern "C" int sd_pack_input_amax(int dtype, const float* x, int batch, int cin, int H, int W, int cpad, void* out,
                                  unsigned* amax, int slot, int clear, sd_stream s) {
    SD_REQUIRE(x && out && amax && batch > 0 && cin > 0 && H > 0 && W > 0 && slot >= 0 && clear != slot,
               "sd_pack_input_amax: bad args");
    SD_REQUIRE(cpad >= cin && cpad % 8 == 0, "sd_pack_input_amax: cpad %d", cpad);
    int g = grid_for((long long)batch * H * W);
    if (g > 512) g = 512;  // grid-stride: at most 512 block maxima compete for the atomic
    if (dtype == SD_BF16)
        hipLaunchKernelGGL(k_pack_input_amax<__bf16>, dim3(g), dim3(256), 0, to_stream(s), x, batch, cin, H, W, cpad,
                           (__bf16*)out, amax, slot, clear);
    else
        hipLaunchKernelGGL(k_pack_input_amax<float>, dim3(g), dim3(256), 0, to_stream(s), x, batch, cin, H, W, cpad,
                           (float*)out, amax, slot, clear);
    return sd_check_launch("sd_pack_input_amax");
}

extern "C" int sd_pack_conv3_w(int dtype, const float* w, int co, int ci, int ci_pad, int dgrad, int kpad, void* out,
                               sd_stream s) {
    SD_REQUIRE(w && out && co > 0 && ci > 0 && ci_pad >= ci && ci_pad % 8 == 0, "sd_pack_conv3_w: bad args");
    SD_REQUIRE(kpad % 64 == 0 && kpad >= 9 * (dgrad ? co : ci_pad), "sd_pack_conv3_w: kpad %d too small", kpad);
    SD_REQUIRE(!dgrad || (ci == ci_pad && co % 8 == 0), "sd_pack_conv3_w: dgrad needs unpadded ci, co%%8==0");
    const int rows = dgrad ? ci : co;
    const int g = grid_for((long long)rows * kpad);
    if (dtype == SD_BF16)
        hipLaunchKernelGGL(k_pack_conv3<__bf16>, dim3(g), dim3(256), 0, to_stream(s), w, co, ci, ci_pad, dgrad, kpad,
                           (__bf16*)out);
    else
        hipLaunchKernelGGL(k_pack_conv3<float>, dim3(g), dim3(256), 0, to_stream(s), w, co, ci, ci_pad, dgrad, kpad,
                           (float*)out);
    return sd_check_launch("sd_pack_conv3_w");
}

extern "C" int sd_pack_convT_w(int dtype, const float* w, int ci, int co, int dgrad, int kpad, void* out,
                               sd_stream s) {
    SD_REQUIRE(w && out && ci > 0 && co > 0 && ci % 8 == 0 && co % 8 == 0, "sd_pack_convT_w: bad args");
    SD_REQUIRE(kpad % 64 == 0 && kpad >= (dgrad ? 4 * co : ci), "sd_pack_convT_w: kpad %d too small", kpad);
    const int rows = dgrad ? ci : 4 * co;
    const int g = grid_for((long long)rows * kpad);
    if (dtype == SD_BF16)
        hipLaunchKernelGGL(k_pack_convT<__bf16>, dim3(g), dim3(256), 0, to_stream(s), w, ci, co, dgrad, kpad,
                           (__bf16*)out);
    else
        hipLaunchKernelGGL(k_pack_convT<float>, dim3(g), dim3(256), 0, to_stream(s), w, ci, co, dgrad, kpad,
                           (float*)out);
    return sd_check_launch("sd_pack_convT_w");
}

// validation and block ranges of a pack job table (sd_pack_weights, sd_step_prologue)
static int pack_plan(int dtype, const sd_pack_job* jobs, int njobs, PackJobs& P, long long& blocks) {
    SD_REQUIRE(jobs && njobs > 0 && njobs <= PACK_MAX_JOBS, "sd_pack_weights: njobs=%d (max %d)", njobs,
               PACK_MAX_JOBS);
    P.n = njobs;
    blocks = 0;
    for (int j = 0; j < njobs; ++j) {
        const sd_pack_job& q = jobs[j];
        SD_REQUIRE(q.w && q.kind >= SD_PACK_CONV3_FWD && q.kind <= SD_PACK_CONVT_FWD_SPLIT && q.co > 0 && q.ci > 0 &&
                       q.out_off >= 0 && q.kpad % 64 == 0,
                   "sd_pack_weights: job %d bad args", j);
        SD_REQUIRE(dtype == SD_BF16 || q.kind < SD_PACK_CONV3_FWD_SPLIT, "sd_pack_weights: job %d: split packs are bf16",
                   j);
        int groups;  // blocks of this job: one per output row (convT fwd: per o, its 4 rows)
        switch (q.kind) {
            case SD_PACK_CONV3_FWD:
                SD_REQUIRE(q.ci_pad >= q.ci && q.ci_pad % 8 == 0 && q.kpad >= 9 * q.ci_pad && q.ci * 9 <= PACK_LDS_FLOATS,
                           "sd_pack_weights: job %d", j);
                groups = q.co;
                break;
            case SD_PACK_CONV3_DGRAD:
                SD_REQUIRE(q.co % 8 == 0 && q.kpad >= 9 * q.co && q.co * 9 <= PACK_LDS_FLOATS, "sd_pack_weights: job %d", j);
                groups = q.ci;
                break;
            case SD_PACK_CONVT_FWD:
                SD_REQUIRE(q.ci % 8 == 0 && q.co % 8 == 0 && q.kpad >= q.ci && q.ci * 4 <= PACK_LDS_FLOATS,
                           "sd_pack_weights: job %d", j);
                groups = q.co;
                break;
            case SD_PACK_CONV3_FWD_SPLIT:
                SD_REQUIRE(q.ci_pad >= q.ci && q.ci_pad % 8 == 0 && q.kpad >= 18 * q.ci_pad && q.ci * 9 <= PACK_LDS_FLOATS,
                           "sd_pack_weights: job %d", j);
                groups = q.co;
                break;
            case SD_PACK_CONVT_FWD_SPLIT:
                SD_REQUIRE(q.ci % 8 == 0 && q.co % 8 == 0 && q.kpad >= 2 * q.ci && q.ci * 4 <= PACK_LDS_FLOATS,
                           "sd_pack_weights: job %d", j);
                groups = q.co;
                break;
            default:
                SD_REQUIRE(q.ci % 8 == 0 && q.co % 8 == 0 && q.kpad >= 4 * q.co && q.co * 4 <= PACK_LDS_FLOATS,
                           "sd_pack_weights: job %d", j);
                groups = q.ci;
        }
        P.j[j] = q;
        P.first[j] = (int)blocks;
        blocks += groups;
        SD_REQUIRE(blocks < (1LL << 30), "sd_pack_weights: too large");
    }
    P.first[njobs] = (int)blocks;
    return 0;
}

extern "C" int sd_pack_weights(int dtype, const sd_pack_job* jobs, int njobs, void* out, sd_stream s) {
    SD_REQUIRE(out, "sd_pack_weights: null output");
    PackJobs P;
    long long blocks = 0;
    if (int e = pack_plan(dtype, jobs, njobs, P, blocks)) return e;
    if (dtype == SD_BF16)
        hipLaunchKernelGGL(k_pack_multi<__bf16>, dim3((unsigned)blocks), dim3(256), 0, to_stream(s), P, (__bf16*)out);
    else
        hipLaunchKernelGGL(k_pack_multi<float>, dim3((unsigned)blocks), dim3(256), 0, to_stream(s), P, (float*)out);
    return sd_check_launch("sd_pack_weights");
}

static int count_grid(long long pixels) {
    // one atomic per block and counter, and the same-address atomics serialize (1024 blocks x 2 counters took ~28 us
    // at 320x240 B=64): 256 blocks, each thread with ~18 16-B target loads in passes of four
    long long g = (pixels / 4 + 255) / 256;
    if (g > 256) g = 256;
    return (int)(g < 1 ? 1 : g);
}

extern "C" int sd_count_valid(const float* target, const uint8_t* mask, int64_t pixels, int* count, int ncount,
                              int* clear, sd_stream s) {
    SD_REQUIRE(target && mask && count && pixels > 0 && ncount >= 1 && ncount <= 4, "sd_count_valid: bad args");
    SD_REQUIRE(!clear || clear + ncount <= count || count + ncount <= clear, "sd_count_valid: clear overlaps count");
    if (!clear && hipMemsetAsync(count, 0, sizeof(int) * ncount, to_stream(s)) != hipSuccess)
        return sd_check_launch("sd_count_valid");
    const int g = count_grid(pixels);
    // the vector path needs a 4-B aligned mask and 16-B aligned targets; otherwise scalar-only
    const bool vec = ((uintptr_t)mask % 4 == 0) && ((uintptr_t)target % 16 == 0);
    hipLaunchKernelGGL(k_count_valid, dim3(g), dim3(256), 0, to_stream(s), target, mask, vec ? (long long)pixels : 0LL,
                       count, ncount, clear);
    if (!vec)
        hipLaunchKernelGGL(k_count_valid_scalar, dim3(g), dim3(256), 0, to_stream(s), target, mask, (long long)pixels,
                           count, ncount);
    return sd_check_launch("sd_count_valid");
}

extern "C" int sd_step_prologue(int dtype, const sd_pack_job* jobs, int njobs, void* wpack, const float* x, int batch,
                                int cin, int H, int W, int cpad, void* xout, const float* target, const uint8_t* mask,
                                int64_t pixels, int* count, int ncount, int* clear, sd_stream s) {
    SD_REQUIRE(dtype == SD_BF16 || dtype == SD_F32, "sd_step_prologue: dtype %d", dtype);
    SD_REQUIRE(wpack, "sd_step_prologue: null weight pack");
    SD_REQUIRE(x && xout && batch > 0 && cin > 0 && H > 0 && W > 0 && cpad >= cin && cpad % 8 == 0,
               "sd_step_prologue: bad input pack args");
    SD_REQUIRE(target && mask && count && clear && pixels > 0 && ncount >= 1 && ncount <= 4 &&
                   (clear + ncount <= count || count + ncount <= clear),
               "sd_step_prologue: bad count args");
    SD_REQUIRE((uintptr_t)mask % 4 == 0 && (uintptr_t)target % 16 == 0,
               "sd_step_prologue: the count needs a 4-B aligned mask and 16-B aligned targets (use sd_count_valid)");
    PackJobs P;
    long long nb_pack = 0;
    if (int e = pack_plan(dtype, jobs, njobs, P, nb_pack)) return e;
    // the vectorised input pack: 4 | H*W (whole quads of pixels inside one image plane) and a 16-B aligned x
    const bool vec4 = ((long long)H * W) % 4 == 0 && (uintptr_t)x % 16 == 0;
    const int nb_cnt = count_grid(pixels), nb_in = grid_for((long long)batch * H * W / (vec4 ? 4 : 1));
    const long long blocks = nb_pack + nb_cnt + nb_in;
    SD_REQUIRE(blocks < (1LL << 30), "sd_step_prologue: too large");
    if (dtype == SD_BF16)
        hipLaunchKernelGGL(k_step_prologue<__bf16>, dim3((unsigned)blocks), dim3(256), 0, to_stream(s), P,
                           (__bf16*)wpack, (int)nb_pack, x, batch, cin, H, W, cpad, (__bf16*)xout, nb_in, (int)vec4,
                           target, mask, (long long)pixels, count, ncount, clear, nb_cnt);
    else
        hipLaunchKernelGGL(k_step_prologue<float>, dim3((unsigned)blocks), dim3(256), 0, to_stream(s), P,
                           (float*)wpack, (int)nb_pack, x, batch, cin, H, W, cpad, (float*)xout, nb_in, (int)vec4,
                           target, mask, (long long)pixels, count, ncount, clear, nb_cnt);
    return sd_check_launch("sd_step_prologue");
}

extern "C" int sd_adamw(float* p, const float* g, float* m, float* v, int64_t n, double lr, double weight_decay,
                          double beta1, double beta2, double eps, int* step, const int* count, float* scratch,
                          sd_stream s) {
    SD_REQUIRE(p && g && m && v && n > 0 && step && scratch, "sd_adamw: bad args");
    const float w1 = (float)(1.0 - beta1), w2 = (float)(1.0 - beta2);
    static const int cap = [] {
        const char* e = getenv("SD_ADAM_BLOCKS");
        return e && atoi(e) > 0 ? atoi(e) : 1024;
    }();
    const int grid = std::min(grid_for(n), cap);
    hipLaunchKernelGGL(k_adamw, dim3(grid), dim3(256), 0, to_stream(s), p, g, m, v, (long long)n, w1, (float)beta2,
                       w2, (float)eps, step, count, lr, weight_decay, beta1, beta2, reinterpret_cast<unsigned*>(scratch));
    return sd_check_launch("sd_adamw");
}

extern "C" int sd_resize_bilinear(const float* in, int planes, int Hi, int Wi, float* out, int Ho, int Wo, float mul,
                                  sd_stream s) {
    SD_REQUIRE(in && out && planes > 0 && Hi > 0 && Wi > 0 && Ho > 0 && Wo > 0, "sd_resize_bilinear: bad args");
    const int g = grid_for((long long)planes * Ho * Wo);
    hipLaunchKernelGGL(k_resize_bilinear, dim3(g), dim3(256), 0, to_stream(s), in, planes, Hi, Wi, out, Ho, Wo, mul);
    return sd_check_launch("sd_resize_bilinear");
}
