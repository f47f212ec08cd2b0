// Device helpers shared by the halo kernels (conv_halo.hip) and the fused full-resolution backward (bwd_fused.hip):
// the packed BN+ReLU and BatchNorm-backward transforms of 8-channel pieces, the BatchNorm-backward sums of a stored
// piece, and the transposed LDS fragment read.
#pragma once
#include "common.h"

namespace {

typedef float f32x2 __attribute__((ext_vector_type(2)));

// halo_finish_pk's transform on an explicit per-channel affine (8 channels: s0|s1 scales, h0|h1 shifts). One
// v_fma_f32 per channel: packed v_pk_fma_f32 pairs measured 2.2 % slower over the bench step (these loaders run
// beside MFMA waves on the same SIMDs, where packed fp32 VALU issues slower than two scalar ops)
__device__ __forceinline__ uint4 bnrelu_pk(uint4 raw, float4 s0, float4 s1, float4 h0, float4 h1) {
    const unsigned w[4] = {raw.x, raw.y, raw.z, raw.w};
    const f32x2 s[4] = {{s0.x, s0.y}, {s0.z, s0.w}, {s1.x, s1.y}, {s1.z, s1.w}};
    const f32x2 h[4] = {{h0.x, h0.y}, {h0.z, h0.w}, {h1.x, h1.y}, {h1.z, h1.w}};
    unsigned o[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const f32x2 v = {__uint_as_float(w[i] << 16), __uint_as_float(w[i] & 0xffff0000u)};
        const float rx = __builtin_fmaf(v.x, s[i].x, h[i].x), ry = __builtin_fmaf(v.y, s[i].y, h[i].y);
        asm("v_cvt_pk_bf16_f32 %0, %1, %2\n\tv_pk_max_i16 %0, %0, 0" : "=v"(o[i]) : "v"(rx), "v"(ry));
    }
    return make_uint4(o[0], o[1], o[2], o[3]);
}

// BNS: the BatchNorm constants of a channel pair, -mean*invstd folded for xhat = y*invstd + nmi
struct BnsK {
    f32x2 sc, sh, is, nmi;
};
// BatchNorm-backward sums of one stored 16-B piece of da (8 bf16 channels) and the y piece of the same pixel:
// dz = da where y*scale+shift > 0 (a pixel outside the tile adds zeros), own[4q + {0,1}] += dz and
// own[4q + {2,3}] += dz*xhat for channel pair q, in packed fp32 pairs
__device__ __forceinline__ void bns_add(float* own, const uint4 v, const uint4 yv, const bool live, const BnsK* bk) {
    const unsigned wv[4] = {v.x, v.y, v.z, v.w}, yw[4] = {yv.x, yv.y, yv.z, yv.w};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const f32x2 d = {__uint_as_float(wv[q] << 16), __uint_as_float(wv[q] & 0xffff0000u)};
        const f32x2 yy = {__uint_as_float(yw[q] << 16), __uint_as_float(yw[q] & 0xffff0000u)};
        const f32x2 z = __builtin_elementwise_fma(yy, bk[q].sc, bk[q].sh);
        const f32x2 xh = __builtin_elementwise_fma(yy, bk[q].is, bk[q].nmi);
        const f32x2 dz = {(live & (z.x > 0.f)) ? d.x : 0.f, (live & (z.y > 0.f)) ? d.y : 0.f};
        f32x2 sm = {own[4 * q], own[4 * q + 1]}, sx = {own[4 * q + 2], own[4 * q + 3]};
        sm += dz;
        sx = __builtin_elementwise_fma(dz, xh, sx);
        own[4 * q] = sm.x;
        own[4 * q + 1] = sm.y;
        own[4 * q + 2] = sx.x;
        own[4 * q + 3] = sx.y;
    }
}

// ds_read_b64_tr_b16 pair: rows r and r+8 (per-lane row addresses), 4 columns at col0+4*(i&3)
__device__ __forceinline__ bf16x8 tr_pair(const __bf16* a0, const __bf16* a1) {
    bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(a0));
    bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(a1));
    bf16x8 r;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        r[t] = lo[t];
        r[t + 4] = hi[t];
    }
    return r;
}

// dy for 8 channels from the raw bf16 pieces (da, y): the BatchNorm-backward apply of k_bn_bwd_apply,
// dy = k0*(dz - k1 - xhat*k2), dz = da where z = y*scale+shift > 0 (the forward ReLU mask, recomputed as
// k_bn_bwd_apply does), xhat = (y-mean)*invstd, written in terms of z (which the mask needs anyway) with
// k0 = scale: dy = scale*dz + Bz*z + Cz, Bz = -invstd*k2, Cz = invstd*k2*shift + scale*(mean*invstd*k2 - k1);
// the mask applied to da (scalar fp32, as bnrelu_pk)
__device__ __forceinline__ uint4 bn_bwd_pk(uint4 da, uint4 y, const float* sc, const float* sh, const float* Bz,
                                           const float* Cz) {
    const unsigned dw[4] = {da.x, da.y, da.z, da.w}, yw[4] = {y.x, y.y, y.z, y.w};
    unsigned o[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const f32x2 s2 = {sc[2 * i], sc[2 * i + 1]}, h2 = {sh[2 * i], sh[2 * i + 1]};
        const f32x2 b2 = {Bz[2 * i], Bz[2 * i + 1]}, c2 = {Cz[2 * i], Cz[2 * i + 1]};
        const f32x2 yv = {__uint_as_float(yw[i] << 16), __uint_as_float(yw[i] & 0xffff0000u)};
        const f32x2 dv = {__uint_as_float(dw[i] << 16), __uint_as_float(dw[i] & 0xffff0000u)};
        f32x2 r;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const float z = __builtin_fmaf(yv[h], s2[h], h2[h]);
            const float t = __builtin_fmaf(b2[h], z, c2[h]);
            r[h] = __builtin_fmaf(s2[h], z > 0.f ? dv[h] : 0.f, t);
        }
        asm("v_cvt_pk_bf16_f32 %0, %1, %2" : "=v"(o[i]) : "v"(r.x), "v"(r.y));
    }
    return make_uint4(o[0], o[1], o[2], o[3]);
}

}  // namespace
