// On-device sample preparation: what FoundationStereoDataset.__getitem__ does with tensors
// (dataset.py:184-212, 305-311), moved off the DataLoader workers. The host only decodes image
// files to uint8 and copies uint8 (pinned, async) to HBM; one kernel then produces the batch dict.
//
// Arithmetic follows the reference in fp32 and in its order: RGB bytes / 255 before the
// interpolation; disparity (R*255*255 + G*255 + B) exact in fp32 (< 2^24), / 1000, interpolated,
// then times Wo/Ws. Bilinear weights and indices as ATen's upsample_bilinear2d (common.h).
// HBM-bound byte work: one thread per output pixel, 4 source taps x 9 bytes, 8 outputs.
#include <hip/hip_fp16.h>

#include "common.h"

namespace {

__device__ __forceinline__ float bilerp(float a, float b, float c, float d, float lx, float ly) {
    // ATen Interpolate<2>: (x00*w0x + x01*w1x)*w0y + (x10*w0x + x11*w1x)*w1y
    return (a * (1.f - lx) + b * lx) * (1.f - ly) + (c * (1.f - lx) + d * lx) * ly;
}

__device__ __forceinline__ float decode_rgb24(const uint8_t* px) {
    return (float)((int)px[0] * 65025 + (int)px[1] * 255 + (int)px[2]) / 1000.f;
}

__global__ void k_stereo_preprocess(const uint8_t* __restrict__ left, const uint8_t* __restrict__ right,
                                    const uint8_t* __restrict__ disp, int B, int Hs, int Ws, int Ho, int Wo,
                                    float wscale, float* __restrict__ input, float* __restrict__ target,
                                    uint8_t* __restrict__ valid) {
    const long long plane = (long long)Ho * Wo, total = (long long)B * plane;
    for (long long e = blockIdx.x * 256LL + threadIdx.x; e < total; e += (long long)gridDim.x * 256) {
        const int b = (int)(e / plane);
        const int rem = (int)(e - (long long)b * plane);
        const int y = rem / Wo, x = rem - y * Wo;
        int y0, y1, x0, x1;
        float ly, lx;
        src_index(y, Ho, Hs, y0, y1, ly);
        src_index(x, Wo, Ws, x0, x1, lx);
        const size_t img = (size_t)b * Hs * Ws * 3;
        const size_t o00 = img + ((size_t)y0 * Ws + x0) * 3, o01 = img + ((size_t)y0 * Ws + x1) * 3;
        const size_t o10 = img + ((size_t)y1 * Ws + x0) * 3, o11 = img + ((size_t)y1 * Ws + x1) * 3;
        float* in_b = input + (size_t)b * 6 * plane + rem;
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            in_b[c * plane] = bilerp((float)left[o00 + c] / 255.f, (float)left[o01 + c] / 255.f,
                                     (float)left[o10 + c] / 255.f, (float)left[o11 + c] / 255.f, lx, ly);
            in_b[(3 + c) * plane] = bilerp((float)right[o00 + c] / 255.f, (float)right[o01 + c] / 255.f,
                                           (float)right[o10 + c] / 255.f, (float)right[o11 + c] / 255.f, lx, ly);
        }
        const float t = bilerp(decode_rgb24(disp + o00), decode_rgb24(disp + o01), decode_rgb24(disp + o10),
                               decode_rgb24(disp + o11), lx, ly) * wscale;
        target[e] = t;
        valid[e] = t > 0.f;
    }
}

__global__ void k_stereo_from_cache(const uint8_t* __restrict__ left, const uint8_t* __restrict__ right,
                                    const __half* __restrict__ disp, int B, int Ho, int Wo, float* __restrict__ input,
                                    float* __restrict__ target, uint8_t* __restrict__ valid) {
    const long long plane = (long long)Ho * Wo, total = (long long)B * plane;
    for (long long e = blockIdx.x * 256LL + threadIdx.x; e < total; e += (long long)gridDim.x * 256) {
        const int b = (int)(e / plane);
        const int rem = (int)(e - (long long)b * plane);
        const size_t px = (size_t)e * 3;
        float* in_b = input + (size_t)b * 6 * plane + rem;
#pragma unroll
        for (int c = 0; c < 3; ++c) {
            in_b[c * plane] = (float)left[px + c] / 255.f;
            in_b[(3 + c) * plane] = (float)right[px + c] / 255.f;
        }
        const float t = __half2float(disp[e]);
        target[e] = t;
        valid[e] = t > 0.f;
    }
}

// 4 pixels per thread (plane % 4 == 0): three 4-B loads per image of the packed HWC bytes, one 8-B load of the f16
// disparities, 16-B stores per output plane (the per-pixel form issued 6 byte loads and 8 scalar stores per pixel)
__global__ void k_stereo_from_cache4(const uint8_t* __restrict__ left, const uint8_t* __restrict__ right,
                                     const __half* __restrict__ disp, int B, int Ho, int Wo, float* __restrict__ input,
                                     float* __restrict__ target, uint8_t* __restrict__ valid) {
    const long long plane = (long long)Ho * Wo, total4 = (long long)B * plane / 4;
    for (long long q = blockIdx.x * 256LL + threadIdx.x; q < total4; q += (long long)gridDim.x * 256) {
        const long long e = q * 4;
        const int b = (int)(e / plane);
        const int rem = (int)(e - (long long)b * plane);
        float* in_b = input + (size_t)b * 6 * plane + rem;
#pragma unroll
        for (int side = 0; side < 2; ++side) {
            const uint32_t* src = reinterpret_cast<const uint32_t*>((side ? right : left) + (size_t)e * 3);
            const uint32_t w0 = src[0], w1 = src[1], w2 = src[2];  // r0 g0 b0 r1 | g1 b1 r2 g2 | b2 r3 g3 b3
            const uint8_t v[12] = {(uint8_t)w0, (uint8_t)(w0 >> 8), (uint8_t)(w0 >> 16), (uint8_t)(w0 >> 24),
                                   (uint8_t)w1, (uint8_t)(w1 >> 8), (uint8_t)(w1 >> 16), (uint8_t)(w1 >> 24),
                                   (uint8_t)w2, (uint8_t)(w2 >> 8), (uint8_t)(w2 >> 16), (uint8_t)(w2 >> 24)};
#pragma unroll
            for (int c = 0; c < 3; ++c)
                *reinterpret_cast<float4*>(in_b + (3 * side + c) * plane) =
                    make_float4((float)v[c] / 255.f, (float)v[3 + c] / 255.f, (float)v[6 + c] / 255.f, (float)v[9 + c] / 255.f);
        }
        const uint2 dh = *reinterpret_cast<const uint2*>(disp + e);
        const __half* h = reinterpret_cast<const __half*>(&dh);
        const float t0 = __half2float(h[0]), t1 = __half2float(h[1]), t2 = __half2float(h[2]), t3 = __half2float(h[3]);
        *reinterpret_cast<float4*>(target + e) = make_float4(t0, t1, t2, t3);
        *reinterpret_cast<uint32_t*>(valid + e) =
            (uint32_t)(t0 > 0.f) | (uint32_t)(t1 > 0.f) << 8 | (uint32_t)(t2 > 0.f) << 16 | (uint32_t)(t3 > 0.f) << 24;
    }
}

int grid_for(long long work) {
    long long g = (work + 255) / 256;
    if (g > 16384) g = 16384;
    return (int)(g < 1 ? 1 : g);
}

}  // namespace

extern "C" int sd_stereo_preprocess(const uint8_t* left, const uint8_t* right, const uint8_t* disp_rgb, int batch,
                                    int Hs, int Ws, int Ho, int Wo, float* input, float* target, uint8_t* valid,
                                    sd_stream s) {
    SD_REQUIRE(left && right && disp_rgb && input && target && valid, "sd_stereo_preprocess: null pointer");
    SD_REQUIRE(batch > 0 && Hs > 0 && Ws > 0 && Ho > 0 && Wo > 0, "sd_stereo_preprocess: bad sizes");
    // width_scale = resized_width / float(original_width) in double, applied as a float32 scalar
    const float wscale = (float)((double)Wo / (double)Ws);
    hipLaunchKernelGGL(k_stereo_preprocess, dim3(grid_for((long long)batch * Ho * Wo)), dim3(256), 0, to_stream(s),
                       left, right, disp_rgb, batch, Hs, Ws, Ho, Wo, wscale, input, target, valid);
    return sd_check_launch("sd_stereo_preprocess");
}

extern "C" int sd_stereo_from_cache(const uint8_t* left, const uint8_t* right, const uint16_t* disp_f16, int batch,
                                    int Ho, int Wo, float* input, float* target, uint8_t* valid, sd_stream s) {
    SD_REQUIRE(left && right && disp_f16 && input && target && valid, "sd_stereo_from_cache: null pointer");
    SD_REQUIRE(batch > 0 && Ho > 0 && Wo > 0, "sd_stereo_from_cache: bad sizes");
    const bool vec = ((long long)Ho * Wo) % 4 == 0 && (uintptr_t)left % 4 == 0 && (uintptr_t)right % 4 == 0 &&
                     (uintptr_t)disp_f16 % 8 == 0 && (uintptr_t)input % 16 == 0 && (uintptr_t)target % 16 == 0 &&
                     (uintptr_t)valid % 4 == 0;
    if (vec)
        hipLaunchKernelGGL(k_stereo_from_cache4, dim3(grid_for((long long)batch * Ho * Wo / 4)), dim3(256), 0,
                           to_stream(s), left, right, reinterpret_cast<const __half*>(disp_f16), batch, Ho, Wo, input,
                           target, valid);
    else
        hipLaunchKernelGGL(k_stereo_from_cache, dim3(grid_for((long long)batch * Ho * Wo)), dim3(256), 0, to_stream(s),
                           left, right, reinterpret_cast<const __half*>(disp_f16), batch, Ho, Wo, input, target, valid);
    return sd_check_launch("sd_stereo_from_cache");
}

// =====================================================================================
// Asymmetric colour augmentation: FoundationStereoDataset._augment_rgb (dataset.py:248-270) on
// 2B independent RGB images (left and right of each pair), torchvision 0.25 functional ops:
//   brightness: blend(img, 0, f) ; contrast: blend(img, mean(gray(img)), f) ;
//   saturation: blend(img, gray(img), f) ; hue: HSV round trip with h += shift (mod 1) ;
//   gamma: img^g ; optional gaussian blur (k x k, reflect padding) ; + N(0, std) ; clamp [0, 1].
// blend(a, b, r) = clamp(r*a + (1-r)*b, 0, 1); gray = 0.2989 r + 0.587 g + 0.114 b.
// Parameters are sampled on the host in the reference's RNG order; the noise field comes from a
// counter-based generator (the reference draws it from torch's CPU generator, so it is not
// reproducible bit for bit, only in distribution).
// =====================================================================================
namespace {

constexpr int AUG_P = 7;  // brightness, contrast, saturation, hue, gamma, blur sigma, noise std

__device__ __forceinline__ float clamp01(float x) { return fminf(fmaxf(x, 0.f), 1.f); }
__device__ __forceinline__ float blend(float a, float b, float r) { return clamp01(r * a + (1.f - r) * b); }
__device__ __forceinline__ float gray(float r, float g, float b) { return 0.2989f * r + 0.587f * g + 0.114f * b; }

// per-image mean of gray(brightness-adjusted image) (adjust_contrast's mean), fp64 accumulation: MEAN_SPLIT blocks
// per image each write one partial sum (an image is 0.3 M pixels at 640x480: one block per image took ~60 us)
constexpr int MEAN_SPLIT = 32;
__global__ void k_aug_gray_mean(const float* __restrict__ input, int HW, const float* __restrict__ params,
                                double* __restrict__ partial) {
    const int im = blockIdx.y;  // image = 2*pair + side
    const float* x = input + ((size_t)(im >> 1) * 6 + (im & 1) * 3) * HW;
    const float fb = params[im * AUG_P + 0];
    double acc = 0.0;
    for (int i = blockIdx.x * 256 + threadIdx.x; i < HW; i += MEAN_SPLIT * 256)
        acc += gray(clamp01(fb * x[i]), clamp01(fb * x[HW + i]), clamp01(fb * x[2 * HW + i]));
    __shared__ double red[256];
    red[threadIdx.x] = acc;
    __syncthreads();
    for (int o = 128; o > 0; o >>= 1) {
        if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
        __syncthreads();
    }
    if (threadIdx.x == 0) partial[im * MEAN_SPLIT + blockIdx.x] = red[0];
}

__device__ __forceinline__ void hue_shift(float& r, float& g, float& b, float shift) {
    // _rgb2hsv
    const float maxc = fmaxf(fmaxf(r, g), b), minc = fminf(fminf(r, g), b);
    const bool eqc = maxc == minc;
    const float cr = maxc - minc;
    const float s = cr / (eqc ? 1.f : maxc);
    const float crd = eqc ? 1.f : cr;
    const float rc = (maxc - r) / crd, gc = (maxc - g) / crd, bc = (maxc - b) / crd;
    const float hr = (maxc == r) ? (bc - gc) : 0.f;
    const float hg = ((maxc == g) && (maxc != r)) ? (2.f + rc - bc) : 0.f;
    const float hb = ((maxc != g) && (maxc != r)) ? (4.f + gc - rc) : 0.f;
    float h = fmodf((hr + hg + hb) / 6.f + 1.f, 1.f);
    // adjust_hue: (h + shift) % 1.0 (python-style modulo, result in [0, 1))
    h = h + shift;
    h = h - floorf(h);
    if (h >= 1.f) h = 0.f;
    // _hsv2rgb
    const float v = maxc;
    const float i6 = floorf(h * 6.f);
    const float f = h * 6.f - i6;
    int i = (int)i6 % 6;
    if (i < 0) i += 6;
    const float p = clamp01(v * (1.f - s)), q = clamp01(v * (1.f - s * f)), t = clamp01(v * (1.f - s * (1.f - f)));
    switch (i) {
        case 0: r = v; g = t; b = p; break;
        case 1: r = q; g = v; b = p; break;
        case 2: r = p; g = v; b = t; break;
        case 3: r = p; g = q; b = v; break;
        case 4: r = t; g = p; b = v; break;
        default: r = v; g = p; b = q; break;
    }
}

__device__ __forceinline__ uint32_t mix32(uint64_t x) {
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdULL;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ULL;
    x ^= x >> 33;
    return (uint32_t)x;
}
// Box-Muller on two hashed uniforms: the pair of independent N(0,1) values (r cos, r sin) of counter idx
__device__ __forceinline__ float2 normal2_at(uint64_t seed, uint64_t idx) {
    const float u1 = ((mix32(seed ^ (idx * 2 + 1) * 0x9E3779B97F4A7C15ULL) >> 8) + 1) * (1.f / 16777217.f);
    const float u2 = (mix32(seed + (idx * 2 + 2) * 0xD1B54A32D192ED03ULL) >> 8) * (1.f / 16777216.f);
    const float r = sqrtf(-2.f * logf(u1));
    float sn, cs;
    sincospif(2.f * u2, &sn, &cs);
    return make_float2(r * cs, r * sn);
}
// x^g for x in [0, 1] (torchvision adjust_gamma, gain 1): exp2(g log2 x) on the hardware transcendentals (~1 ulp each;
// powf's exact-rounding path cost most of the pointwise kernel's time); 0^g = 0 for g > 0
__device__ __forceinline__ float pow01(float x, float g) {
    return x > 0.f ? __builtin_amdgcn_exp2f(g * __builtin_amdgcn_logf(x)) : (g == 0.f ? 1.f : 0.f);
}

// brightness, contrast, saturation, hue, gamma -> work (same layout as input); blockIdx.y = image, whose contrast mean
// the block sums from the partials once
__global__ void k_aug_pointwise(const float* __restrict__ input, int HW, const float* __restrict__ params,
                                const double* __restrict__ partial, float* __restrict__ work) {
    const int im = blockIdx.y;
    __shared__ float s_m;
    if (threadIdx.x == 0) {
        double t = 0.0;
        for (int k = 0; k < MEAN_SPLIT; ++k) t += partial[im * MEAN_SPLIT + k];
        s_m = (float)(t / HW);
    }
    __syncthreads();
    const float m = s_m;
    const float* pr = params + im * AUG_P;
    const float fb = pr[0], fc = pr[1], fs = pr[2], fh = pr[3], fg = pr[4];
    const size_t base0 = ((size_t)(im >> 1) * 6 + (im & 1) * 3) * HW;
    for (int px = blockIdx.x * 256 + threadIdx.x; px < HW; px += gridDim.x * 256) {
        const size_t base = base0 + px;
        float r = input[base], g = input[base + HW], b = input[base + 2 * HW];
        r = clamp01(fb * r);  // brightness: blend with zeros
        g = clamp01(fb * g);
        b = clamp01(fb * b);
        r = blend(r, m, fc);  // contrast
        g = blend(g, m, fc);
        b = blend(b, m, fc);
        const float l = gray(r, g, b);  // saturation
        r = blend(r, l, fs);
        g = blend(g, l, fs);
        b = blend(b, l, fs);
        hue_shift(r, g, b, fh);  // the reference calls adjust_hue even for a zero shift
        r = clamp01(pow01(r, fg));  // gamma (gain 1)
        g = clamp01(pow01(g, fg));
        b = clamp01(pow01(b, fg));
        work[base] = r;
        work[base + HW] = g;
        work[base + 2 * HW] = b;
    }
}

// optional gaussian blur (per-image sigma, 0 = off), + noise, clamp -> input; blockIdx.y = plane (image, channel), whose
// normalised 1-D kernel the block builds once in LDS (_get_gaussian_kernel1d: linspace(-(k-1)/2, (k-1)/2, k),
// exp(-0.5 (x/sigma)^2), normalised)
__global__ void k_aug_blur_noise(const float* __restrict__ work, int H, int W, const float* __restrict__ params, int ks,
                                 uint64_t seed, float* __restrict__ input) {
    const int HW = H * W;
    const int half = ks / 2;
    const int plane = blockIdx.y, im = plane / 3, c = plane - im * 3;
    const size_t base = ((size_t)(im >> 1) * 6 + (im & 1) * 3 + c) * HW;
    const float* pr = params + im * AUG_P;
    const float sigma = pr[5], std = pr[6];
    __shared__ float k1[31];
    if (threadIdx.x == 0 && sigma > 0.f) {
        float ksum = 0.f;
        for (int i = 0; i < ks; ++i) {
            const float x = (float)(i - half) / sigma;
            k1[i] = expf(-0.5f * x * x);
            ksum += k1[i];
        }
        for (int i = 0; i < ks; ++i) k1[i] /= ksum;
    }
    __syncthreads();
    // two adjacent pixels per thread, one Box-Muller draw for both
    for (int px = 2 * (blockIdx.x * 256 + threadIdx.x); px < HW; px += 2 * gridDim.x * 256) {
        float v[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int q = px + h < HW ? px + h : px;  // odd HW: the last thread's second pixel repeats its first
            if (sigma > 0.f) {
                const int y = q / W, x = q - y * W;
                float acc = 0.f;
                for (int i = 0; i < ks; ++i) {
                    int yy = y + i - half;
                    yy = yy < 0 ? -yy : (yy >= H ? 2 * H - 2 - yy : yy);  // reflect
                    const float* row = work + base + (size_t)yy * W;
                    for (int j = 0; j < ks; ++j) {
                        int xx = x + j - half;
                        xx = xx < 0 ? -xx : (xx >= W ? 2 * W - 2 - xx : xx);
                        acc += (k1[i] * k1[j]) * row[xx];
                    }
                }
                v[h] = acc;
            } else {
                v[h] = work[base + q];
            }
        }
        if (std > 0.f) {
            const float2 z = normal2_at(seed, ((uint64_t)plane * HW + px) >> 1);
            v[0] += z.x * std;
            v[1] += z.y * std;
        }
        input[base + px] = clamp01(v[0]);
        if (px + 1 < HW) input[base + px + 1] = clamp01(v[1]);
    }
}

}  // namespace

extern "C" int sd_augment_rgb(float* input, int batch, int H, int W, const float* params, int blur_ksize,
                              uint64_t seed, float* work, sd_stream s) {
    SD_REQUIRE(input && params && work && batch > 0 && H > 0 && W > 0 && ((uintptr_t)work % 8) == 0,
               "sd_augment_rgb: bad args");
    SD_REQUIRE(blur_ksize >= 3 && blur_ksize % 2 == 1 && blur_ksize <= 31, "sd_augment_rgb: blur_ksize %d", blur_ksize);
    SD_REQUIRE(blur_ksize / 2 < H && blur_ksize / 2 < W, "sd_augment_rgb: blur kernel larger than the image");
    const int HW = H * W;
    // the contrast partial sums (2*batch*MEAN_SPLIT doubles) follow the images in `work` (8-B aligned: 6*HW*batch is even)
    double* partial = reinterpret_cast<double*>(work + (size_t)batch * 6 * HW);
    hipStream_t st = to_stream(s);
    const int per = (HW + 255) / 256;
    const int gx = per < 64 ? per : 64;  // blocks per image / plane (2*batch or 6*batch rows of the grid)
    hipLaunchKernelGGL(k_aug_gray_mean, dim3(MEAN_SPLIT, 2 * batch), dim3(256), 0, st, input, HW, params, partial);
    hipLaunchKernelGGL(k_aug_pointwise, dim3(gx, 2 * batch), dim3(256), 0, st, input, HW, params, partial, work);
    hipLaunchKernelGGL(k_aug_blur_noise, dim3(gx, 6 * batch), dim3(256), 0, st, work, H, W, params, blur_ksize, seed, input);
    return sd_check_launch("sd_augment_rgb");
}
