// Fused output heads + masked heteroscedastic NLL + its gradient + metric sums.
// Replaces (one pass over the dec1 activation):
//   model.py:76-77,98,103  two 1x1 convs 32->1 (+bias), softplus(beta=1,threshold=20), clamp(-6,3)
//   train.py:329-340       mask = valid & isfinite(t); nll = |p-t|*exp(-lv) + lv; loss = mean
//   train.py:341           the loss/heads part of loss.backward()
//   train.py:345-352       sums of nll, |d|, d^2, exp(lv/2) and the valid count
#include <type_traits>

#include "common.h"

namespace {

constexpr int NMET = 5;  // nll, |d|, d^2, sigma, pad

__device__ __forceinline__ float softplus_f(float x) { return x > 20.f ? x : log1pf(expf(x)); }
// ATen softplus_backward: z = exp(x*beta); x*beta > threshold ? g : g*z/(z+1)
__device__ __forceinline__ float softplus_grad(float x, float g) {
    if (x > 20.f) return g;
    const float z = expf(x);
    return g * z / (z + 1.f);
}

// 8 consecutive elements from their raw 16-B pieces (bf16: one, fp32: two)
template <typename T>
__device__ __forceinline__ void raw_to_f32(const uint4* q, float* f) {
    if constexpr (sizeof(T) == 2) {
        const unsigned w[4] = {q[0].x, q[0].y, q[0].z, q[0].w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            f[2 * i] = __uint_as_float(w[i] << 16);
            f[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
        }
    } else {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            f[4 * h] = __uint_as_float(q[h].x);
            f[4 * h + 1] = __uint_as_float(q[h].y);
            f[4 * h + 2] = __uint_as_float(q[h].z);
            f[4 * h + 3] = __uint_as_float(q[h].w);
        }
    }
}

// Lanes of one pixel group: value of lane (l ^ o), and of group lane u. DPP quad permutes for groups of
// up to 4 lanes (VALU moves), ds_bpermute for 8.
template <int LPP>
__device__ __forceinline__ float grp_xor(float v, int o) {
    const int x = __float_as_int(v);
    if constexpr (LPP <= 4) {
        if (o == 1) return __int_as_float(__builtin_amdgcn_update_dpp(0, x, 0xB1, 0xF, 0xF, false));  // [1,0,3,2]
        return __int_as_float(__builtin_amdgcn_update_dpp(0, x, 0x4E, 0xF, 0xF, false));              // [2,3,0,1]
    }
    return __shfl_xor(v, o);
}
template <int LPP>
__device__ __forceinline__ float grp_bcast(float v, int u) {
    const int x = __float_as_int(v);
    if constexpr (LPP == 1) {
        return v;
    } else if constexpr (LPP == 2) {  // quad_perm [u, u, 2+u, 2+u]
        if (u == 0) return __int_as_float(__builtin_amdgcn_update_dpp(0, x, 0xA0, 0xF, 0xF, false));
        return __int_as_float(__builtin_amdgcn_update_dpp(0, x, 0xF5, 0xF, 0xF, false));
    } else if constexpr (LPP == 4) {  // quad_perm [u, u, u, u]
        switch (u) {
            case 0: return __int_as_float(__builtin_amdgcn_update_dpp(0, x, 0x00, 0xF, 0xF, false));
            case 1: return __int_as_float(__builtin_amdgcn_update_dpp(0, x, 0x55, 0xF, 0xF, false));
            case 2: return __int_as_float(__builtin_amdgcn_update_dpp(0, x, 0xAA, 0xF, 0xF, false));
            default: return __int_as_float(__builtin_amdgcn_update_dpp(0, x, 0xFF, 0xF, 0xF, false));
        }
    } else {
        return __shfl(v, (int)(threadIdx.x & 63 & ~(LPP - 1)) | u);
    }
}

// LPP = C/8 lanes per pixel, 8 channels per lane: the y / da traffic is whole 16-B pieces with
// consecutive lanes on consecutive pieces (fully coalesced), each lane keeps accumulators for its 8
// channels only. A lane group takes LPP pixels per iteration: the per-pixel dot products of the two
// 1x1 heads are reduce-scattered over the group so that lane `sub` finishes pixel `sub` alone
// (softplus, clamp, loss, its gradient and the metric sums: no lane repeats another's scalar math),
// and the two head gradients are broadcast back for the per-channel work.
// BNSUM: also the BatchNorm-backward partial sums of the dec1 layer whose output this reads (what
// sd_bn_bwd_reduce computes over da and y): dz = da (as stored) where y*scale+shift > 0,
// sums of dz and dz*(y-mean)*invstd, one float2 row per block.
// The kernel is VALU-bound: two waves per SIMD (launch bound) measured 205 us vs 231 us at one wave
// (256 VGPRs) and 310 us for the version that repeated the per-pixel math on every lane of a group.
template <typename T, int C, bool BNSUM, int MODE>
__global__ __launch_bounds__(256, 2) void k_heads(const T* __restrict__ y, const float* __restrict__ sc,
                                               const float* __restrict__ sh, long long P, const float* __restrict__ wd,
                                               const float* __restrict__ bd_, const float* __restrict__ wl,
                                               const float* __restrict__ bl_, float* disp, float* logvar,
                                               const float* __restrict__ target, const uint8_t* __restrict__ mask,
                                               const int* count, const float* gdisp, const float* glogvar, T* da,
                                               float* partials, const float* __restrict__ mean,
                                               const float* __restrict__ invstd, float2* bnpart) {
    constexpr int LPP = C / 8, PPB = 256 / LPP;  // lanes per pixel, pixels per block iteration
    constexpr int NV = 2 * C + 2 + NMET;
    static_assert(64 % LPP == 0, "a pixel's lanes sit in one wave");
    const int sub = threadIdx.x % LPP, c0 = sub * 8;
    float w_d[8], w_l[8], s_c[8], s_h[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        w_d[i] = wd[c0 + i];
        w_l[i] = wl[c0 + i];
        s_c[i] = sc[c0 + i];
        s_h[i] = sh[c0 + i];
    }
    float gw_d[8], gw_l[8], b1[8], b2[8], met[2 + NMET];  // met: bias grads, then the metric sums
#pragma unroll
    for (int i = 0; i < 8; ++i) gw_d[i] = gw_l[i] = b1[i] = b2[i] = 0.f;
#pragma unroll
    for (int i = 0; i < 2 + NMET; ++i) met[i] = 0.f;
    const float bd = bd_[0], bl = bl_[0];
    float inv_n = 0.f;
    if constexpr (MODE == SD_HEADS_LOSS) {
        const int n = *count;
        inv_n = n > 0 ? 1.0f / (float)n : 0.f;
    }
    // UNR = LPP pixels per lane group per iteration (their 16-B loads issued together); pixel u of the
    // group is px0 + u*stride, and lane `sub` owns pixel u = sub for the scalar work
    constexpr int UNR = LPP;
    const long long stride = (long long)gridDim.x * PPB;
    // Software-pipelined over two register sets: iteration k+1's loads are issued before iteration k's math, so
    // two iterations of loads are in flight per lane (one left the kernel at ~4 TB/s, bytes-in-flight bound).
    // Every iteration issues the same loads (past P: pixel 0, results dropped), none conditional.
    struct Ld {
        uint4 raw[UNR][sizeof(T) / 2];
        float tg, gdv, glv;
        bool mk;
    };
    auto load = [&](Ld& q, long long px0) __attribute__((always_inline)) {
#pragma unroll
        for (int u = 0; u < UNR; ++u) {
            const long long px = px0 + u * stride;
            const long long pq = px < P ? px : 0;  // tail: re-read pixel 0, results dropped below
#pragma unroll
            for (int h = 0; h < (int)(sizeof(T) / 2); ++h) q.raw[u][h] = reinterpret_cast<const uint4*>(y + pq * C + c0)[h];
        }
        const long long pme = px0 + sub * stride;  // this lane's own pixel
        const bool mine = pme < P;
        const long long pmq = mine ? pme : 0;
        q.tg = 0.f;
        q.gdv = 0.f;
        q.glv = 0.f;
        q.mk = false;
        if constexpr (MODE == SD_HEADS_LOSS) {
            q.tg = target[pmq];
            q.mk = mine & (mask[pmq] != 0);
        } else if constexpr (MODE == SD_HEADS_GRADS) {
            q.gdv = gdisp ? gdisp[pmq] : 0.f;
            q.glv = glogvar ? glogvar[pmq] : 0.f;
        }
    };
    auto compute = [&](const Ld& q, long long px0) __attribute__((always_inline)) {
        const long long pme = px0 + sub * stride;  // this lane's own pixel
        const bool mine = pme < P;
        const float tg = q.tg, gdv = q.gdv, glv_in = q.glv;
        const bool mk = q.mk;
        float a[UNR][8], vd[UNR], vl[UNR];
#pragma unroll
        for (int u = 0; u < UNR; ++u) {
            float yv[8];
            raw_to_f32<T>(q.raw[u], yv);
            float pd = 0.f, pl = 0.f;
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                a[u][i] = fmaxf(__builtin_fmaf(yv[i], s_c[i], s_h[i]), 0.f);
                pd = __builtin_fmaf(a[u][i], w_d[i], pd);
                pl = __builtin_fmaf(a[u][i], w_l[i], pl);
            }
            vd[u] = pd;
            vl[u] = pl;
        }
        // reduce-scatter over the group: at lane bit o the lane with the bit clear keeps the low half of
        // the pixel vector plus its partner's low half; lane `sub` ends with pixel sub's sums in [0]
#pragma unroll
        for (int o = LPP / 2, len = UNR; o >= 1; o >>= 1, len >>= 1) {
            const bool hi = (sub & o) != 0;
#pragma unroll
            for (int j = 0; j < len / 2; ++j) {
                const float kd = hi ? vd[j + len / 2] : vd[j], sd_ = hi ? vd[j] : vd[j + len / 2];
                const float kl = hi ? vl[j + len / 2] : vl[j], sl_ = hi ? vl[j] : vl[j + len / 2];
                vd[j] = kd + grp_xor<LPP>(sd_, o);
                vl[j] = kl + grp_xor<LPP>(sl_, o);
            }
        }
        const float xd = vd[0] + bd, xl = vl[0] + bl;
        const float p = softplus_f(xd);
        const float lv = fminf(fmaxf(xl, -6.f), 3.f);
        if (mine) {
            if (disp) disp[pme] = p;
            if (logvar) logvar[pme] = lv;
        }
        if constexpr (MODE == SD_HEADS_INFER) return;
        float gxd = 0.f, gxl = 0.f;
        if constexpr (MODE == SD_HEADS_LOSS) {
            if (mk && isfinite(tg)) {
                const float d = p - tg;
                const float ad = fabsf(d);
                const float e = expf(-lv);
                met[2] += ad * e + lv;
                met[3] += ad;
                met[4] += d * d;
                met[5] += expf(0.5f * lv);
                const float sgn = d > 0.f ? 1.f : (d < 0.f ? -1.f : 0.f);
                const float gp = sgn * (inv_n * e);
                const float glv = inv_n - (inv_n * ad) * e;
                gxd = softplus_grad(xd, gp);
                gxl = (xl >= -6.f && xl <= 3.f) ? glv : 0.f;
            }
        } else if (mine) {  // SD_HEADS_GRADS
            gxd = softplus_grad(xd, gdv);
            gxl = (xl >= -6.f && xl <= 3.f) ? glv_in : 0.f;
        }
        met[0] += gxd;
        met[1] += gxl;
#pragma unroll
        for (int u = 0; u < UNR; ++u) {
            const long long px = px0 + u * stride;
            const float gd = grp_bcast<LPP>(gxd, u), gl = grp_bcast<LPP>(gxl, u);
            if (px >= P) break;  // uniform across a pixel's lanes
            float o[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                o[i] = __builtin_fmaf(gl, w_l[i], gd * w_d[i]);
                gw_d[i] += gd * a[u][i];
                gw_l[i] += gl * a[u][i];
            }
            if (da) store8_nt(da + px * C + c0, o);
            if constexpr (BNSUM) {
                float yv[8];
                raw_to_f32<T>(q.raw[u], yv);
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    const float dz = a[u][i] > 0.f ? (float)(T)o[i] : 0.f;  // the stored da, through the ReLU mask
                    b1[i] += dz;
                    b2[i] += dz * yv[i];  // sum dz*y; sum dz*xhat = invstd*(sum dz*y - mean*sum dz)
                }
            }
        }
    };
    const long long step = UNR * stride;
    // the pipelined form where its second register set fits in 256 VGPRs without spilling (bf16, C <= 32 except two
    // C = 32 instances off the training path); one set otherwise
    constexpr bool PIPE = sizeof(T) == 2 && (C <= 16 || (C == 32 && (BNSUM || MODE == SD_HEADS_INFER)));
    Ld qa, qb;
    long long px0 = blockIdx.x * (long long)PPB + threadIdx.x / LPP;
    if constexpr (PIPE) {
        load(qa, px0);
        for (; px0 < P; px0 += 2 * step) {
            load(qb, px0 + step);
            compute(qa, px0);
            load(qa, px0 + 2 * step);
            compute(qb, px0 + step);
        }
    } else {
        for (; px0 < P; px0 += step) {
            load(qa, px0);
            compute(qa, px0);
        }
    }
    if constexpr (MODE == SD_HEADS_INFER) return;
    // block reduction: lanes of one channel group (equal lane % LPP) by shuffles, then the 4 waves via LDS
    __shared__ float red[4][NV + (BNSUM ? 2 * C : 0)];
    const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
    auto lane_sum = [&](float v) {
#pragma unroll
        for (int o = LPP; o < 64; o <<= 1) v += __shfl_xor(v, o);
        return v;
    };
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        const float vd = lane_sum(gw_d[i]), vl = lane_sum(gw_l[i]);
        if (lane < LPP) {
            red[wid][c0 + i] = vd;
            red[wid][C + c0 + i] = vl;
        }
        if constexpr (BNSUM) {
            const float v1 = lane_sum(b1[i]), v2 = lane_sum(b2[i]);
            if (lane < LPP) {
                red[wid][NV + 2 * (c0 + i)] = v1;
                red[wid][NV + 2 * (c0 + i) + 1] = v2;
            }
        }
    }
#pragma unroll
    for (int i = 0; i < 2 + NMET; ++i) {  // per-pixel values, each pixel held by one lane: full-wave sum
        float v = met[i];
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) v += __shfl_xor(v, o);
        if (lane == 0) red[wid][2 * C + i] = v;
    }
    __syncthreads();
    for (int i = threadIdx.x; i < NV; i += 256)
        partials[(size_t)blockIdx.x * NV + i] = red[0][i] + red[1][i] + red[2][i] + red[3][i];
    if constexpr (BNSUM) {
        for (int c = threadIdx.x; c < C; c += 256) {
            const int k = NV + 2 * c;
            const float s1 = red[0][k] + red[1][k] + red[2][k] + red[3][k];
            const float sy = red[0][k + 1] + red[1][k + 1] + red[2][k + 1] + red[3][k + 1];
            bnpart[(size_t)blockIdx.x * C + c] = make_float2(s1, invstd[c] * (sy - mean[c] * s1));
        }
    }
}

// one block per reduced value: 256 threads stride the partial rows, fp64 tree reduction
__global__ __launch_bounds__(256) void k_heads_finalize(const float* __restrict__ part, int rows, int C, float* dwd,
                                                        float* dbd, float* dwl, float* dbl, double* metrics,
                                                        const int* count) {
    const int NV = 2 * C + 2 + NMET;
    const int i = blockIdx.x;
    __shared__ double red[256];
    double acc = 0.0;
    for (int r = threadIdx.x; r < rows; r += 256) acc += part[(size_t)r * NV + i];
    red[threadIdx.x] = acc;
    __syncthreads();
    for (int st = 128; st > 0; st >>= 1) {
        if (threadIdx.x < st) red[threadIdx.x] += red[threadIdx.x + st];
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        const double s = red[0];
        if (i < C) {
            if (dwd) dwd[i] = (float)s;
        } else if (i < 2 * C) {
            if (dwl) dwl[i - C] = (float)s;
        } else if (i == 2 * C) {
            if (dbd) dbd[0] = (float)s;
        } else if (i == 2 * C + 1) {
            if (dbl) dbl[0] = (float)s;
        } else if (i < 2 * C + 6 && metrics) {
            metrics[i - (2 * C + 2)] += s;
        }
        if (i == 0 && metrics && count) metrics[4] += (double)(*count);
    }
}

int heads_rows(long long P) {
    long long r = (P + 255) / 256;
    return (int)(r > 1024 ? 1024 : (r < 1 ? 1 : r));
}

template <typename T>
int launch_heads(int C, int mode, const void* y, const float* sc, const float* sh, long long P, const float* wd,
                 const float* bd, const float* wl, const float* bl, float* disp, float* logvar, const float* target,
                 const uint8_t* mask, const int* count, const float* gdisp, const float* glogvar, void* da,
                 float* partials, const float* mean, const float* invstd, float* bnpart, hipStream_t st) {
    const dim3 g(heads_rows(P)), b(256);
    auto go = [&](auto cc, auto bnsum, auto md) {
        constexpr int CC = decltype(cc)::value, MD = decltype(md)::value;
        constexpr bool BNS = decltype(bnsum)::value;
        hipLaunchKernelGGL((k_heads<T, CC, BNS, MD>), g, b, 0, st, (const T*)y, sc, sh, P, wd, bd, wl, bl, disp,
                           logvar, target, mask, count, gdisp, glogvar, (T*)da, partials, BNS ? mean : nullptr,
                           BNS ? invstd : nullptr, BNS ? (float2*)bnpart : nullptr);
    };
    auto by_mode = [&](auto cc) {
        using std::integral_constant;
        if (mode == SD_HEADS_INFER) go(cc, std::false_type{}, integral_constant<int, SD_HEADS_INFER>{});
        else if (mode == SD_HEADS_LOSS && bnpart) go(cc, std::true_type{}, integral_constant<int, SD_HEADS_LOSS>{});
        else if (mode == SD_HEADS_LOSS) go(cc, std::false_type{}, integral_constant<int, SD_HEADS_LOSS>{});
        else if (bnpart) go(cc, std::true_type{}, integral_constant<int, SD_HEADS_GRADS>{});
        else go(cc, std::false_type{}, integral_constant<int, SD_HEADS_GRADS>{});
    };
    switch (C) {
        case 8: by_mode(std::integral_constant<int, 8>{}); break;
        case 16: by_mode(std::integral_constant<int, 16>{}); break;
        case 32: by_mode(std::integral_constant<int, 32>{}); break;
        case 64: by_mode(std::integral_constant<int, 64>{}); break;
        default:
            sd_set_error("sd_heads: C=%d not in {8,16,32,64}", C);
            return SD_EINVAL;
    }
    return sd_check_launch("sd_heads");
}

}  // namespace

extern "C" int sd_heads_rows(int64_t pixels) { return heads_rows(pixels); }

static int heads_entry(int dtype, int mode, const void* y, const float* scale, const float* shift, int64_t pixels,
                       int C, const float* wd, const float* bd, const float* wl, const float* bl, float* disp,
                       float* logvar, const float* target, const uint8_t* mask, const int* count, const float* gdisp,
                       const float* glogvar, void* da, float* partials, const float* mean, const float* invstd,
                       float* bnpart, sd_stream s) {
    SD_REQUIRE(y && scale && shift && wd && bd && wl && bl && pixels > 0, "sd_heads: null input");
    SD_REQUIRE(mode == SD_HEADS_INFER || mode == SD_HEADS_LOSS || mode == SD_HEADS_GRADS, "sd_heads: mode %d", mode);
    if (mode == SD_HEADS_LOSS) SD_REQUIRE(target && mask && count, "sd_heads: LOSS needs target/mask/count");
    if (mode != SD_HEADS_INFER) SD_REQUIRE(partials, "sd_heads: LOSS/GRADS need partials");
    if (mode == SD_HEADS_GRADS) SD_REQUIRE(da, "sd_heads: GRADS needs da");
    if (dtype == SD_BF16)
        return launch_heads<__bf16>(C, mode, y, scale, shift, pixels, wd, bd, wl, bl, disp, logvar, target, mask,
                                    count, gdisp, glogvar, da, partials, mean, invstd, bnpart, to_stream(s));
    return launch_heads<float>(C, mode, y, scale, shift, pixels, wd, bd, wl, bl, disp, logvar, target, mask, count,
                               gdisp, glogvar, da, partials, mean, invstd, bnpart, to_stream(s));
}

extern "C" int sd_heads(int dtype, int mode, const void* y, const float* scale, const float* shift, int64_t pixels,
                        int C, const float* wd, const float* bd, const float* wl, const float* bl, float* disp,
                        float* logvar, const float* target, const uint8_t* mask, const int* count, const float* gdisp,
                        const float* glogvar, void* da, float* partials, sd_stream s) {
    return heads_entry(dtype, mode, y, scale, shift, pixels, C, wd, bd, wl, bl, disp, logvar, target, mask, count,
                       gdisp, glogvar, da, partials, nullptr, nullptr, nullptr, s);
}

extern "C" int sd_heads_bnsum(int dtype, int mode, const void* y, const float* scale, const float* shift,
                              int64_t pixels, int C, const float* wd, const float* bd, const float* wl, const float* bl,
                              float* disp, float* logvar, const float* target, const uint8_t* mask, const int* count,
                              const float* gdisp, const float* glogvar, void* da, float* partials, const float* mean,
                              const float* invstd, float* bnpart, sd_stream s) {
    SD_REQUIRE(mode != SD_HEADS_INFER && da && mean && invstd && bnpart, "sd_heads_bnsum: needs da, mean, invstd, bnpart");
    return heads_entry(dtype, mode, y, scale, shift, pixels, C, wd, bd, wl, bl, disp, logvar, target, mask, count,
                       gdisp, glogvar, da, partials, mean, invstd, bnpart, s);
}

extern "C" int sd_heads_finalize(const float* partials, int rows, int C, float* dwd, float* dbd, float* dwl,
                                 float* dbl, double* metrics, const int* count, sd_stream s) {
    SD_REQUIRE(partials && rows > 0 && C > 0, "sd_heads_finalize: bad args");
    hipLaunchKernelGGL(k_heads_finalize, dim3(2 * C + 2 + NMET), dim3(256), 0, to_stream(s), partials, rows, C, dwd,
                       dbd, dwl, dbl, metrics, count);
    return sd_check_launch("sd_heads_finalize");
}
