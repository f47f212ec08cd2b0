// BatchNorm2d (train + eval), ReLU / MaxPool2d backward, per-channel sums.
// Replaces native_batch_norm{,_backward}, threshold_backward and max_pool2d_with_indices_backward
// for model.py:37-41 (BN+ReLU) and model.py:59,83-86 (MaxPool2d(2)).
// Forward BN statistics arrive as per-M-block (sum, sumsq) partials from the producing conv's
// epilogue (conv_gemm.hip); finalize reduces them in fp64 (ATen CPU accumulates BN moments in
// double) and emits the fused affine (scale, shift) consumed by the next GEMM's gather.
#include "common.h"

namespace {

// ------------------------------------------------------------------ finalize (one block per channel; block_sum2 in common.h)
// mean/invstd/scale/shift and the running-statistics update of channel c from its fp64 (sum, sumsq) over `count`
// pixels (every rank's, with SyncBatchNorm: the unbiased variance then uses the global count, as torch's)
__device__ __forceinline__ void bn_fwd_emit(int c, double s, double ss, double count, const float* gamma,
                                            const float* beta, float* running_mean, float* running_var, int64_t* nbt,
                                            float momentum, float eps, float* mean_o, float* invstd_o, float* scale_o,
                                            float* shift_o) {
    const double mean = s / count;
    double var = ss / count - mean * mean;
    if (var < 0.0) var = 0.0;
    const float invstd = (float)(1.0 / sqrt(var + (double)eps));
    const float sc = gamma[c] * invstd;
    mean_o[c] = (float)mean;
    invstd_o[c] = invstd;
    scale_o[c] = sc;
    shift_o[c] = beta[c] - (float)mean * sc;
    if (running_mean) {
        const double unbiased = count > 1.0 ? var * count / (count - 1.0) : var;
        running_mean[c] = (float)(momentum * mean + (1.0 - momentum) * (double)running_mean[c]);
        running_var[c] = (float)(momentum * unbiased + (1.0 - momentum) * (double)running_var[c]);
    }
    if (nbt && c == 0) nbt[0] += 1;
}

__global__ __launch_bounds__(256) void k_bn_fwd_finalize(const float2* __restrict__ stats, int rows, int C,
                                                         double count, const float* gamma, const float* beta,
                                                         float* running_mean, float* running_var, int64_t* nbt,
                                                         float momentum, float eps, float* mean_o, float* invstd_o,
                                                         float* scale_o, float* shift_o) {
    const int c = blockIdx.x;
    double s = 0.0, ss = 0.0;
    for (int r = threadIdx.x; r < rows; r += 256) {
        const float2 v = stats[(size_t)r * C + c];
        s += v.x;
        ss += v.y;
    }
    block_sum2<256>(s, ss);
    if (threadIdx.x == 0)
        bn_fwd_emit(c, s, ss, count, gamma, beta, running_mean, running_var, nbt, momentum, eps, mean_o, invstd_o,
                    scale_o, shift_o);
}

// SyncBatchNorm: the float2 partial rows of one rank -> fp64 per-channel sums[2c], sums[2c+1] (the same fixed-order
// reduction the finalizes run), which the host all-reduces across ranks before the *_finalize64 kernels
__global__ __launch_bounds__(256) void k_rows_sum64(const float2* __restrict__ rows_, int rows, int C, double pixels,
                                                    double* sums) {
    const int c = blockIdx.x;
    if (c == 0 && threadIdx.x == 0) sums[2 * C] = pixels;  // summed with the channel sums by the all-reduce
    double s = 0.0, ss = 0.0;
    for (int r = threadIdx.x; r < rows; r += 256) {
        const float2 v = rows_[(size_t)r * C + c];
        s += v.x;
        ss += v.y;
    }
    block_sum2<256>(s, ss);
    if (threadIdx.x == 0) {
        sums[2 * c] = s;
        sums[2 * c + 1] = ss;
    }
}

__global__ __launch_bounds__(256) void k_bn_fwd_finalize64(const double* __restrict__ sums, int C,
                                                           const float* gamma, const float* beta, float* running_mean,
                                                           float* running_var, int64_t* nbt, float momentum, float eps,
                                                           float* mean_o, float* invstd_o, float* scale_o,
                                                           float* shift_o) {
    const int c = blockIdx.x * 256 + threadIdx.x;
    const double count = sums[2 * C];  // global pixel count
    if (c < C)
        bn_fwd_emit(c, sums[2 * c], sums[2 * c + 1], count, gamma, beta, running_mean, running_var, nbt, momentum, eps,
                    mean_o, invstd_o, scale_o, shift_o);
}

__global__ void k_bn_eval_coeffs(const float* rm, const float* rv, const float* gamma, const float* beta, int C,
                                 float eps, float* mean_o, float* invstd_o, float* scale_o, float* shift_o) {
    const int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    const float invstd = 1.0f / sqrtf(rv[c] + eps);
    const float sc = gamma[c] * invstd;
    mean_o[c] = rm[c];
    invstd_o[c] = invstd;
    scale_o[c] = sc;
    shift_o[c] = beta[c] - rm[c] * sc;
}

// ------------------------------------------------------------------ channel reductions over NHWC
enum { OP_SUM = 0, OP_BNBWD = 1 };

struct ChanArgs {
    const void* x;   // da (BNBWD) or x (SUM)
    const void* y;   // pre-BN conv output (BNBWD)
    const float *sc, *sh, *mean, *invstd;
    long long P;
    int C;
    float2* partials;
};

int chan_rows(long long P, int C) {
    const int cpr = C / 8;
    const int ppi = 256 / cpr;
    long long r = (P + ppi - 1) / ppi;
    return (int)(r < 1024 ? r : 1024);
}

template <typename T, int OP>
__global__ __launch_bounds__(256) void k_chan_reduce(const ChanArgs a) {
    const int cpr = a.C / 8, ppi = 256 / cpr;
    const int chunk = threadIdx.x % cpr, prow = threadIdx.x / cpr;
    const int c = chunk * 8;
    float s1[8], s2[8];
    zero8(s1);
    zero8(s2);
    if (prow < ppi) {
        float sc[8], sh[8], mu[8], is[8];
        if (OP == OP_BNBWD) {
            load8(a.sc + c, sc);
            load8(a.sh + c, sh);
            load8(a.mean + c, mu);
            load8(a.invstd + c, is);
        }
        for (long long px = (long long)blockIdx.x * ppi + prow; px < a.P; px += (long long)gridDim.x * ppi) {
            float v[8];
            load8((const T*)a.x + px * a.C + c, v);
            if (OP == OP_BNBWD) {
                float y[8];
                load8((const T*)a.y + px * a.C + c, y);
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    const float z = __builtin_fmaf(y[i], sc[i], sh[i]);
                    const float dz = z > 0.f ? v[i] : 0.f;
                    s1[i] += dz;
                    s2[i] += dz * ((y[i] - mu[i]) * is[i]);
                }
            } else {
#pragma unroll
                for (int i = 0; i < 8; ++i) s1[i] += v[i];
            }
        }
    }
    __shared__ float red[256][17];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        red[threadIdx.x][i] = s1[i];
        red[threadIdx.x][8 + i] = s2[i];
    }
    __syncthreads();
    // thread t sums channels t, t+256, ... over the block's pixel rows
    for (int cc = threadIdx.x; cc < a.C; cc += 256) {
        const int ch = cc / 8, ci = cc % 8;
        float t1 = 0.f, t2 = 0.f;
        for (int r = 0; r < ppi; ++r) {
            t1 += red[r * cpr + ch][ci];
            t2 += red[r * cpr + ch][8 + ci];
        }
        a.partials[(size_t)blockIdx.x * a.C + cc] = make_float2(t1, t2);
    }
}

// dgamma/dbeta from this rank's sums (the gradient all-reduce adds the ranks' shares), coef from the sums over
// `count` pixels (with SyncBatchNorm every rank's: gs/gss and count are global)
__device__ __forceinline__ void bn_bwd_emit(int c, double s, double ss, double gs, double gss, double count,
                                            const float* gamma, const float* invstd, int batch_stats, float* dgamma,
                                            float* dbeta, float* coef) {
    dbeta[c] = (float)s;
    dgamma[c] = (float)ss;
    coef[3 * c + 0] = gamma[c] * invstd[c];
    coef[3 * c + 1] = batch_stats ? (float)(gs / count) : 0.f;
    coef[3 * c + 2] = batch_stats ? (float)(gss / count) : 0.f;
}

__global__ __launch_bounds__(256) void k_bn_bwd_finalize(const float2* __restrict__ part, int rows, int C,
                                                         double count, const float* gamma, const float* invstd,
                                                         int batch_stats, float* dgamma, float* dbeta, float* coef) {
    const int c = blockIdx.x;
    double s = 0.0, ss = 0.0;
    for (int r = threadIdx.x; r < rows; r += 256) {
        const float2 v = part[(size_t)r * C + c];
        s += v.x;
        ss += v.y;
    }
    block_sum2<256>(s, ss);
    if (threadIdx.x == 0) bn_bwd_emit(c, s, ss, s, ss, count, gamma, invstd, batch_stats, dgamma, dbeta, coef);
}

__global__ __launch_bounds__(256) void k_bn_bwd_finalize64(const double* __restrict__ local,
                                                           const double* __restrict__ global, int C,
                                                           const float* gamma, const float* invstd, int batch_stats,
                                                           float* dgamma, float* dbeta, float* coef) {
    const int c = blockIdx.x * 256 + threadIdx.x;
    const double count = global[2 * C];  // global pixel count
    if (c < C)
        bn_bwd_emit(c, local[2 * c], local[2 * c + 1], global[2 * c], global[2 * c + 1], count, gamma, invstd,
                    batch_stats, dgamma, dbeta, coef);
}

__global__ __launch_bounds__(256) void k_sum_finalize(const float2* __restrict__ part, int rows, int ld, float* out) {
    const int c = blockIdx.x;
    double s = 0.0, ss = 0.0;
    for (int r = threadIdx.x; r < rows; r += 256) s += part[(size_t)r * ld + c].x;
    block_sum2<256>(s, ss);
    if (threadIdx.x == 0) out[c] = (float)s;
}

// ------------------------------------------------------------------ elementwise backward passes
template <typename T>
__global__ __launch_bounds__(256) void k_bn_bwd_apply(const T* __restrict__ da, const T* __restrict__ y,
                                                      const float* sc_, const float* sh_, const float* mean_,
                                                      const float* invstd_, const float* coef, long long P, int C,
                                                      T* __restrict__ dy) {
    // each thread owns one 8-channel chunk (C/8 divides 256): per-channel parameters stay in registers
    const int cpr = C / 8, ppi = 256 / cpr;
    const int c = (threadIdx.x % cpr) * 8, prow = threadIdx.x / cpr;
    if (prow >= ppi) return;  // C/8 not a power of two: the last threads idle
    float sc[8], sh[8], mu[8], is[8], k0[8], k1[8], k2[8];
    load8(sc_ + c, sc);
    load8(sh_ + c, sh);
    load8(mean_ + c, mu);
    load8(invstd_ + c, is);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        k0[i] = coef[3 * (c + i)];
        k1[i] = coef[3 * (c + i) + 1];
        k2[i] = coef[3 * (c + i) + 2];
    }
    for (long long px = (long long)blockIdx.x * ppi + prow; px < P; px += (long long)gridDim.x * ppi) {
        float v[8], yy[8], out[8];
        load8(da + px * C + c, v);
        load8(y + px * C + c, yy);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            const float z = __builtin_fmaf(yy[i], sc[i], sh[i]);
            const float dz = z > 0.f ? v[i] : 0.f;
            const float xh = (yy[i] - mu[i]) * is[i];
            out[i] = k0[i] * (dz - k1[i] - xh * k2[i]);
        }
        store8_nt(dy + px * C + c, out);
    }
}

// MaxPool2d backward + skip add. BNSUM: also the BatchNorm-backward partial sums of the layer
// whose output this is (what sd_bn_bwd_reduce computes), from values already in registers:
// dz = da (as stored) where y*scale+shift > 0, sums of dz and dz*(y-mean)*invstd. The grid stride
// is a multiple of C/8, so each thread keeps one 8-channel chunk; one partials row per block.
template <typename T, bool BNSUM>
__global__ __launch_bounds__(256) void k_pool_bwd_add(const T* __restrict__ y, const float* sc, const float* sh,
                                                      const T* __restrict__ dskip, const T* __restrict__ dpool,
                                                      int batch, int H, int W, int C, T* __restrict__ da,
                                                      const float* __restrict__ mean, const float* __restrict__ invstd,
                                                      float2* __restrict__ part) {
    const int cpr = C / 8, H2 = H / 2, W2 = W / 2;
    const long long total = (long long)batch * H2 * W2 * cpr;
    float s1[8], s2[8], mu[8], is[8];
    zero8(s1);
    zero8(s2);
    if (BNSUM) {
        const int c = (int)(threadIdx.x % cpr) * 8;
        load8(mean + c, mu);
        load8(invstd + c, is);
    }
    for (long long e = blockIdx.x * 256LL + threadIdx.x; e < total; e += (long long)gridDim.x * 256) {
        const long long win = e / cpr;
        const int c = (int)(e - win * cpr) * 8;
        const int w2 = (int)(win % W2);
        const long long t = win / W2;
        const int h2 = (int)(t % H2), b = (int)(t / H2);
        float v[4][8], yr[4][8], dp[8];
        size_t off[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            off[k] = (((size_t)b * H + 2 * h2 + (k >> 1)) * W + 2 * w2 + (k & 1)) * C + c;
            load8(y + off[k], v[k]);
#pragma unroll
            for (int i = 0; i < 8; ++i) yr[k][i] = v[k][i];
            xform8(v[k], sc, sh, c);
        }
        load8(dpool + (size_t)win * C + c, dp);
        int am[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) {  // first max in row-major window order (ATen CPU: strict >)
            float best = v[0][i];
            am[i] = 0;
#pragma unroll
            for (int k = 1; k < 4; ++k)
                if (v[k][i] > best) {
                    best = v[k][i];
                    am[i] = k;
                }
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            float o[8];
            if (dskip)
                load8(dskip + off[k], o);
            else
                zero8(o);
#pragma unroll
            for (int i = 0; i < 8; ++i) o[i] += (am[i] == k) ? dp[i] : 0.f;
            store8_nt(da + off[k], o);
            if (BNSUM) {
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    const float dz = v[k][i] > 0.f ? to_f32(from_f32<T>(o[i])) : 0.f;  // the stored value
                    s1[i] += dz;
                    s2[i] += dz * ((yr[k][i] - mu[i]) * is[i]);
                }
            }
        }
    }
    if (BNSUM) {
        __shared__ float red[256][17];
#pragma unroll
        for (int i = 0; i < 8; ++i) {
            red[threadIdx.x][i] = s1[i];
            red[threadIdx.x][8 + i] = s2[i];
        }
        __syncthreads();
        for (int cc = threadIdx.x; cc < C; cc += 256) {
            const int ch = cc / 8, ci = cc % 8;
            float a1 = 0.f, a2 = 0.f;
            for (int t = ch; t < 256; t += cpr) {
                a1 += red[t][ci];
                a2 += red[t][8 + ci];
            }
            part[(size_t)blockIdx.x * C + cc] = make_float2(a1, a2);
        }
    }
}

int grid_for(long long work) {
    long long g = (work + 255) / 256;
    if (g > 8192) g = 8192;
    return (int)(g < 1 ? 1 : g);
}

// Blocks of 256 threads of `kernel` resident on the whole device at once (occupancy x CUs), or
// `fallback` when the runtime cannot say. Grid-stride kernels launched with more blocks than this run a
// partial last round: with 1024 blocks at 768 resident the last quarter of the blocks ran on a third of
// the machine for as long as a full round.
static int resident_blocks(const void* kernel, int fallback) {
    int per_cu = 0, dev = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, 256, 0) != hipSuccess || per_cu < 1 || cus < 1) {
        (void)hipGetLastError();
        return fallback;
    }
    return per_cu * cus;
}


}  // namespace

extern "C" int sd_bn_fwd_finalize(const float* stats, int rows, int C, double count, const float* gamma,
                                  const float* beta, float* running_mean, float* running_var,
                                  int64_t* num_batches_tracked, float momentum, float eps, float* mean, float* invstd,
                                  float* scale, float* shift, sd_stream s) {
    SD_REQUIRE(stats && rows > 0 && C > 0 && count > 0 && gamma && beta && mean && invstd && scale && shift,
               "sd_bn_fwd_finalize: bad args");
    SD_REQUIRE((running_mean == nullptr) == (running_var == nullptr), "sd_bn_fwd_finalize: running stats pair");
    hipLaunchKernelGGL(k_bn_fwd_finalize, dim3(C), dim3(256), 0, to_stream(s), (const float2*)stats, rows, C, count,
                       gamma, beta, running_mean, running_var, num_batches_tracked, momentum, eps, mean, invstd, scale,
                       shift);
    return sd_check_launch("sd_bn_fwd_finalize");
}

extern "C" int sd_bn_rows_sum64(const float* rows, int nrows, int C, double pixels, double* sums, sd_stream s) {
    SD_REQUIRE(rows && sums && nrows > 0 && C > 0 && pixels > 0, "sd_bn_rows_sum64: bad args");
    hipLaunchKernelGGL(k_rows_sum64, dim3(C), dim3(256), 0, to_stream(s), (const float2*)rows, nrows, C, pixels, sums);
    return sd_check_launch("sd_bn_rows_sum64");
}

extern "C" int sd_bn_fwd_finalize64(const double* sums, int C, const float* gamma, const float* beta,
                                    float* running_mean, float* running_var, int64_t* num_batches_tracked,
                                    float momentum, float eps, float* mean, float* invstd, float* scale, float* shift,
                                    sd_stream s) {
    SD_REQUIRE(sums && C > 0 && gamma && beta && mean && invstd && scale && shift, "sd_bn_fwd_finalize64: bad args");
    SD_REQUIRE((running_mean == nullptr) == (running_var == nullptr), "sd_bn_fwd_finalize64: running stats pair");
    hipLaunchKernelGGL(k_bn_fwd_finalize64, dim3(cdiv(C, 256)), dim3(256), 0, to_stream(s), sums, C, gamma, beta,
                       running_mean, running_var, num_batches_tracked, momentum, eps, mean, invstd, scale, shift);
    return sd_check_launch("sd_bn_fwd_finalize64");
}

extern "C" int sd_bn_bwd_finalize64(const double* local_sums, const double* global_sums, int C, const float* gamma, const float* invstd, int batch_stats, float* dgamma,
                                    float* dbeta, float* coef, sd_stream s) {
    SD_REQUIRE(local_sums && global_sums && C > 0 && gamma && invstd && dgamma && dbeta && coef,
               "sd_bn_bwd_finalize64: bad args");
    hipLaunchKernelGGL(k_bn_bwd_finalize64, dim3(cdiv(C, 256)), dim3(256), 0, to_stream(s), local_sums, global_sums, C,
                       gamma, invstd, batch_stats, dgamma, dbeta, coef);
    return sd_check_launch("sd_bn_bwd_finalize64");
}

extern "C" int sd_bn_eval_coeffs(const float* running_mean, const float* running_var, const float* gamma,
                                 const float* beta, int C, float eps, float* mean, float* invstd, float* scale,
                                 float* shift, sd_stream s) {
    SD_REQUIRE(running_mean && running_var && gamma && beta && C > 0 && mean && invstd && scale && shift,
               "sd_bn_eval_coeffs: bad args");
    hipLaunchKernelGGL(k_bn_eval_coeffs, dim3(cdiv(C, 256)), dim3(256), 0, to_stream(s), running_mean, running_var,
                       gamma, beta, C, eps, mean, invstd, scale, shift);
    return sd_check_launch("sd_bn_eval_coeffs");
}

extern "C" int sd_chan_reduce_rows(int64_t pixels, int C) { return chan_rows(pixels, C); }

static int check_chan(int C, long long P, const char* what) {
    SD_REQUIRE(C > 0 && C % 8 == 0 && C <= 2048, "%s: C=%d must be a multiple of 8 in (0, 2048]", what, C);
    SD_REQUIRE(P > 0, "%s: no pixels", what);
    return SD_OK;
}

extern "C" int sd_bn_bwd_reduce(int dtype, const void* da, const void* y, const float* scale, const float* shift,
                                const float* mean, const float* invstd, int64_t pixels, int C, float* partials,
                                sd_stream s) {
    if (int e = check_chan(C, pixels, "sd_bn_bwd_reduce")) return e;
    SD_REQUIRE(da && y && scale && shift && mean && invstd && partials, "sd_bn_bwd_reduce: null pointer");
    ChanArgs a{da, y, scale, shift, mean, invstd, pixels, C, (float2*)partials};
    const int rows = chan_rows(pixels, C);
    if (dtype == SD_BF16)
        hipLaunchKernelGGL((k_chan_reduce<__bf16, OP_BNBWD>), dim3(rows), dim3(256), 0, to_stream(s), a);
    else
        hipLaunchKernelGGL((k_chan_reduce<float, OP_BNBWD>), dim3(rows), dim3(256), 0, to_stream(s), a);
    return sd_check_launch("sd_bn_bwd_reduce");
}

extern "C" int sd_bn_bwd_finalize(const float* partials, int rows, int C, double count, const float* gamma,
                                  const float* invstd, int batch_stats, float* dgamma, float* dbeta, float* coef,
                                  sd_stream s) {
    SD_REQUIRE(partials && rows > 0 && C > 0 && count > 0 && gamma && invstd && dgamma && dbeta && coef,
               "sd_bn_bwd_finalize: bad args");
    hipLaunchKernelGGL(k_bn_bwd_finalize, dim3(C), dim3(256), 0, to_stream(s), (const float2*)partials, rows, C,
                       count, gamma, invstd, batch_stats, dgamma, dbeta, coef);
    return sd_check_launch("sd_bn_bwd_finalize");
}

extern "C" int sd_bn_bwd_apply(int dtype, const void* da, const void* y, const float* scale, const float* shift,
                               const float* mean, const float* invstd, const float* coef, int64_t pixels, int C,
                               void* dy, sd_stream s) {
    if (int e = check_chan(C, pixels, "sd_bn_bwd_apply")) return e;
    SD_REQUIRE(da && y && scale && shift && mean && invstd && coef && dy, "sd_bn_bwd_apply: null pointer");
    const int g = grid_for(pixels * (C / 8));  // one-round grids (resident_blocks) measured no faster here
    if (dtype == SD_BF16)
        hipLaunchKernelGGL(k_bn_bwd_apply<__bf16>, dim3(g), dim3(256), 0, to_stream(s), (const __bf16*)da,
                           (const __bf16*)y, scale, shift, mean, invstd, coef, (long long)pixels, C, (__bf16*)dy);
    else
        hipLaunchKernelGGL(k_bn_bwd_apply<float>, dim3(g), dim3(256), 0, to_stream(s), (const float*)da,
                           (const float*)y, scale, shift, mean, invstd, coef, (long long)pixels, C, (float*)dy);
    return sd_check_launch("sd_bn_bwd_apply");
}

static int pool_bwd_grid(long long work) {  // = partials rows when the fused sums are requested
    static const int cap = resident_blocks((const void*)k_pool_bwd_add<__bf16, true>, 1024);
    const long long need = (work + 255) / 256;
    return (int)(need < 1 ? 1 : (need < cap ? need : cap));
}

extern "C" int sd_pool_bwd_rows(int batch, int H, int W, int C) {
    return pool_bwd_grid((long long)batch * (H / 2) * (W / 2) * (C / 8));
}

extern "C" int sd_pool_bwd_add(int dtype, const void* y, const float* scale, const float* shift, const void* dskip,
                               const void* dpool, int batch, int H, int W, int C, void* da, const float* mean,
                               const float* invstd, float* partials, sd_stream s) {
    SD_REQUIRE(y && scale && shift && dpool && da, "sd_pool_bwd_add: null pointer");
    SD_REQUIRE(batch > 0 && H > 0 && W > 0 && H % 2 == 0 && W % 2 == 0, "sd_pool_bwd_add: dims must be even");
    if (int e = check_chan(C, (long long)batch * H * W, "sd_pool_bwd_add")) return e;
    SD_REQUIRE(!partials || (mean && invstd && 256 % (C / 8) == 0),
               "sd_pool_bwd_add: fused BN sums need mean/invstd and C/8 dividing 256");
    const int g = pool_bwd_grid((long long)batch * (H / 2) * (W / 2) * (C / 8));
    auto* part = reinterpret_cast<float2*>(partials);
    if (dtype == SD_BF16) {
        if (partials)
            hipLaunchKernelGGL((k_pool_bwd_add<__bf16, true>), dim3(g), dim3(256), 0, to_stream(s), (const __bf16*)y,
                               scale, shift, (const __bf16*)dskip, (const __bf16*)dpool, batch, H, W, C, (__bf16*)da,
                               mean, invstd, part);
        else
            hipLaunchKernelGGL((k_pool_bwd_add<__bf16, false>), dim3(g), dim3(256), 0, to_stream(s), (const __bf16*)y,
                               scale, shift, (const __bf16*)dskip, (const __bf16*)dpool, batch, H, W, C, (__bf16*)da,
                               mean, invstd, part);
    } else {
        if (partials)
            hipLaunchKernelGGL((k_pool_bwd_add<float, true>), dim3(g), dim3(256), 0, to_stream(s), (const float*)y,
                               scale, shift, (const float*)dskip, (const float*)dpool, batch, H, W, C, (float*)da, mean,
                               invstd, part);
        else
            hipLaunchKernelGGL((k_pool_bwd_add<float, false>), dim3(g), dim3(256), 0, to_stream(s), (const float*)y,
                               scale, shift, (const float*)dskip, (const float*)dpool, batch, H, W, C, (float*)da, mean,
                               invstd, part);
    }
    return sd_check_launch("sd_pool_bwd_add");
}

extern "C" int sd_chan_sum(int dtype, const void* x, int64_t pixels, int C, float* partials, float* out,
                           sd_stream s) {
    if (int e = check_chan(C, pixels, "sd_chan_sum")) return e;
    SD_REQUIRE(x && partials && out, "sd_chan_sum: null pointer");
    ChanArgs a{x, nullptr, nullptr, nullptr, nullptr, nullptr, pixels, C, (float2*)partials};
    const int rows = chan_rows(pixels, C);
    if (dtype == SD_BF16)
        hipLaunchKernelGGL((k_chan_reduce<__bf16, OP_SUM>), dim3(rows), dim3(256), 0, to_stream(s), a);
    else
        hipLaunchKernelGGL((k_chan_reduce<float, OP_SUM>), dim3(rows), dim3(256), 0, to_stream(s), a);
    if (int e = sd_check_launch("sd_chan_sum")) return e;
    hipLaunchKernelGGL(k_sum_finalize, dim3(C), dim3(256), 0, to_stream(s), (const float2*)partials, rows, C, out);
    return sd_check_launch("sd_chan_sum(finalize)");
}

extern "C" int sd_stat_rows_sum(const float* stats, int rows, int ld, int C, float* out, sd_stream s) {
    SD_REQUIRE(stats && out && rows > 0 && C > 0 && C <= ld, "sd_stat_rows_sum: bad args");
    hipLaunchKernelGGL(k_sum_finalize, dim3(C), dim3(256), 0, to_stream(s), (const float2*)stats, rows, ld, out);
    return sd_check_launch("sd_stat_rows_sum");
}
