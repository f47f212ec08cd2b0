// Weight gradients as split-K GEMMs over pixels (replaces convolution_backward's wgrad for
// model.py:36,39 Conv2d and model.py:67-73 ConvTranspose2d).
//   conv3x3 : dW[co][(tap,ci)] = sum_p dy[p][co] * x_in[p + tap][ci]   (A = dy, B = 9-tap gather of x_in)
//   convT   : dW[ci][(t,co)]   = sum_p x_in[p][ci] * dout[2p + t][co]  (A = x_in, B = sub-pixel gather of dout)
// Both operands are staged pixel-major ([pixel][channel], straight NHWC rows) in LDS and read
// transposed into MFMA fragments (bf16: ds_read_b64_tr_b16).  Each z-slice of the grid reduces
// a contiguous pixel range into its own fp32 slab; sd_wgrad_reduce sums slabs in fixed order
// (deterministic) and scatters into the PyTorch weight layout.
#include "common.h"

namespace {

constexpr int BKP = 32;  // pixels per K tile

template <typename T> struct TrTile {
    static constexpr int PAD = 16;  // elements; conflict-free transposed reads (see frag_tr)
};

// transposed fragment with a consistent k permutation (k is the pixel index: any bijection
// applied to both operands leaves the sum unchanged).  bf16: lanes of 16-lane group g take LDS
// rows {16*(g>>1) + 4*(g&1) + q} then +8, so each ds_read_b64_tr_b16 covers 8 consecutive rows.
__device__ __forceinline__ bf16x8 frag_trp(const __bf16* lds, int ld, int col0, int lane) {
    const int i = lane & 15, g = lane >> 4;
    const int q = i >> 2, pp = i & 3;
    const int r0 = 16 * (g >> 1) + 4 * (g & 1) + q;
    const __bf16* a0 = lds + r0 * ld + col0 + 4 * pp;
    bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(a0));
    bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(a0 + 8 * ld));
    bf16x8 r;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        r[j] = lo[j];
        r[j + 4] = hi[j];
    }
    return r;
}
__device__ __forceinline__ float frag_trp(const float* lds, int ld, int col0, int lane, int ks) {
    return lds[(ks * 4 + (lane >> 4)) * ld + col0 + (lane & 15)];
}

template <typename T>
struct WgArgs {
    GatherSrc a, b;
    int H, W, P;  // pixel grid, P = batch*H*W
    int M, N;
    int pix_per_split;
    float* slab;
};

template <typename T, int BM, int BN, int WM, int WN>
__global__ __launch_bounds__(256) void k_wgemm(const WgArgs<T> p) {
    using MF = Mfma<T>;
    constexpr int LDA = BM + TrTile<T>::PAD, LDB = BN + TrTile<T>::PAD;
    constexpr int WTM = BM / WM, WTN = BN / WN, RM = WTM / 16, RN = WTN / 16;
    constexpr int ACH = BM / 8, BCH = BN / 8;  // chunks per pixel row
    constexpr int AL = (BKP * ACH + 255) / 256, BL = (BKP * BCH + 255) / 256;
    __shared__ __attribute__((aligned(16))) T smem[BKP * (LDA + LDB)];
    T* As = smem;
    T* Bs = smem + BKP * LDA;

    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wm = wid / WN, wn = wid % WN;
    const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;
    const int p_begin = blockIdx.z * p.pix_per_split;
    const int p_end = min(p.P, p_begin + p.pix_per_split);
    const int mch0 = m0 / 8, nch0 = n0 / 8;

    f32x4 acc[RM][RN];
#pragma unroll
    for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int j = 0; j < RN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    float av[AL][8], bv[BL][8];
    auto load_tile = [&](int pt) {
#pragma unroll
        for (int i = 0; i < AL; ++i) {
            const int idx = tid + i * 256;
            const int px = pt + idx / ACH, c = idx % ACH;
            if (idx < BKP * ACH && px < p_end && (m0 + c * 8) < p.M) {
                const int w = px % p.W, t = px / p.W;
                gather_chunk<T>(p.a, t / p.H, t % p.H, w, mch0 + c, av[i]);
            } else {
                zero8(av[i]);
            }
        }
#pragma unroll
        for (int i = 0; i < BL; ++i) {
            const int idx = tid + i * 256;
            const int px = pt + idx / BCH, c = idx % BCH;
            if (idx < BKP * BCH && px < p_end && (n0 + c * 8) < p.N) {
                const int w = px % p.W, t = px / p.W;
                gather_chunk<T>(p.b, t / p.H, t % p.H, w, nch0 + c, bv[i]);
            } else {
                zero8(bv[i]);
            }
        }
    };
    auto store_tile = [&]() {
#pragma unroll
        for (int i = 0; i < AL; ++i) {
            const int idx = tid + i * 256;
            if (idx < BKP * ACH) store8(As + (idx / ACH) * LDA + (idx % ACH) * 8, av[i]);
        }
#pragma unroll
        for (int i = 0; i < BL; ++i) {
            const int idx = tid + i * 256;
            if (idx < BKP * BCH) store8(Bs + (idx / BCH) * LDB + (idx % BCH) * 8, bv[i]);
        }
    };

    if (p_begin < p_end) load_tile(p_begin);
    for (int pt = p_begin; pt < p_end; pt += BKP) {
        store_tile();
        __syncthreads();
        if (pt + BKP < p_end) load_tile(pt + BKP);
#pragma unroll
        for (int ks = 0; ks < BKP / MF::KSTEP; ++ks) {
            typename MF::frag af[RM], bf[RN];
#pragma unroll
            for (int i = 0; i < RM; ++i) {
                if constexpr (sizeof(T) == 2)
                    af[i] = frag_trp(As, LDA, wm * WTM + i * 16, lane);
                else
                    af[i] = frag_trp(As, LDA, wm * WTM + i * 16, lane, ks);
            }
#pragma unroll
            for (int j = 0; j < RN; ++j) {
                if constexpr (sizeof(T) == 2)
                    bf[j] = frag_trp(Bs, LDB, wn * WTN + j * 16, lane);
                else
                    bf[j] = frag_trp(Bs, LDB, wn * WTN + j * 16, lane, ks);
            }
#pragma unroll
            for (int i = 0; i < RM; ++i)
#pragma unroll
                for (int j = 0; j < RN; ++j) acc[i][j] = MF::mma(af[i], bf[j], acc[i][j]);
        }
        __syncthreads();
    }

    float* slab = p.slab + (size_t)blockIdx.z * p.M * p.N;
    const int ccol = lane & 15, crow = (lane >> 4) * 4;
#pragma unroll
    for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int m = m0 + wm * WTM + i * 16 + crow + r;
            if (m >= p.M) continue;
#pragma unroll
            for (int j = 0; j < RN; ++j) {
                const int n = n0 + wn * WTN + j * 16 + ccol;
                if (n < p.N) slab[(size_t)m * p.N + n] = acc[i][j][r];
            }
        }
}

struct WCfg {
    int bm, bn;
};
WCfg pick_wcfg(int M, int N) {
    (void)N;
    return M <= 32 ? WCfg{32, 64} : WCfg{64, 64};
}

int compute_splits(long long P, int M, int N) {
    const WCfg c = pick_wcfg(M, N);
    const long long tiles = (long long)cdiv(M, c.bm) * cdiv(N, c.bn);
    long long splits = (2048 + tiles - 1) / tiles;
    const long long max_splits = (P + BKP * 8 - 1) / (BKP * 8);  // >= 8 K tiles per block
    if (splits > max_splits) splits = max_splits;
    if (splits < 1) splits = 1;
    return (int)splits;
}

// 256 threads = 8 split groups x 32 lanes; a lane owns 4 consecutive elements (16-B loads, 512 B per
// group and split). Each group sums splits g, g+8, g+16, ... into 4 independent accumulators (four
// loads in flight per lane instead of a dependent chain; the slab is read at HBM rate), then the
// 8 group partials are added in fixed order: deterministic for a given split count.
__device__ __forceinline__ void wg_store(float* dw, long long e, float v, int N, int layout, int ci_pad, int ci_real) {
    const int m = (int)(e / N), n = (int)(e % N);
    if (layout == SD_W_CONV3) {
        const int tap = n / ci_pad, ci = n % ci_pad;
        if (ci < ci_real) dw[((size_t)m * ci_real + ci) * 9 + tap] = v;
    } else {
        const int co = N / 4;
        const int t = n / co, o = n % co;
        dw[((size_t)m * co + o) * 4 + t] = v;
    }
}

// G split groups per block (8 or 32), 256 / G float4 outputs per block, 4 independent accumulators per lane: each
// output quad sums its splits in a fixed order (deterministic for a given split count and G). Small layers have
// few output quads and many splits (up to 512): G = 32 keeps 16 loads per output in flight instead of 4 (the
// 8-group form was one dependent memory round trip per 32 splits, 9-12 us for layers of a few KB)
template <int G>
__device__ __forceinline__ void wgrad_reduce_body(const float* __restrict__ slab, int splits, long long total4, int N,
                                                  int layout, int ci_pad, int ci_real, float* __restrict__ dw,
                                                  int bid, int nblocks, float4* part) {  // part: [G][256 / G]
    constexpr int QB = 256 / G;  // output quads per block
    const int el = threadIdx.x % QB, g = threadIdx.x / QB;
    const float4* s4 = reinterpret_cast<const float4*>(slab);
    for (long long q0 = (long long)bid * QB; q0 < total4; q0 += (long long)nblocks * QB) {
        const long long q = q0 + el;
        float4 acc[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) acc[u] = make_float4(0.f, 0.f, 0.f, 0.f);
        if (q < total4) {
            int z = g;
            for (; z + 3 * G < splits; z += 4 * G) {
#pragma unroll
                for (int u = 0; u < 4; ++u) {
                    const float4 v = s4[(size_t)(z + G * u) * total4 + q];
                    acc[u].x += v.x;
                    acc[u].y += v.y;
                    acc[u].z += v.z;
                    acc[u].w += v.w;
                }
            }
#pragma unroll
            for (int u = 0; u < 3; ++u) {  // the < 4 remaining splits of this group
                if (z + G * u < splits) {
                    const float4 v = s4[(size_t)(z + G * u) * total4 + q];
                    acc[u].x += v.x;
                    acc[u].y += v.y;
                    acc[u].z += v.z;
                    acc[u].w += v.w;
                }
            }
        }
        const float4 sum4 = make_float4((acc[0].x + acc[1].x) + (acc[2].x + acc[3].x), (acc[0].y + acc[1].y) + (acc[2].y + acc[3].y),
                                        (acc[0].z + acc[1].z) + (acc[2].z + acc[3].z), (acc[0].w + acc[1].w) + (acc[2].w + acc[3].w));
        if constexpr (G == 1) {  // one thread per output quad: no cross-thread sum
            if (q < total4) {
                const long long e = 4 * q;
                wg_store(dw, e, sum4.x, N, layout, ci_pad, ci_real);
                wg_store(dw, e + 1, sum4.y, N, layout, ci_pad, ci_real);
                wg_store(dw, e + 2, sum4.z, N, layout, ci_pad, ci_real);
                wg_store(dw, e + 3, sum4.w, N, layout, ci_pad, ci_real);
            }
            continue;
        }
        part[g * QB + el] = sum4;
        __syncthreads();
        if (g == 0 && q < total4) {
            float4 t = part[el];
#pragma unroll
            for (int k = 1; k < G; ++k) {
                const float4 v = part[k * QB + el];
                t.x += v.x;
                t.y += v.y;
                t.z += v.z;
                t.w += v.w;
            }
            const long long e = 4 * q;
            wg_store(dw, e, t.x, N, layout, ci_pad, ci_real);
            wg_store(dw, e + 1, t.y, N, layout, ci_pad, ci_real);
            wg_store(dw, e + 2, t.z, N, layout, ci_pad, ci_real);
            wg_store(dw, e + 3, t.w, N, layout, ci_pad, ci_real);
        }
        __syncthreads();
    }
}

// G split groups per block (8 or 32), 256 / G float4 outputs per block, 4 independent accumulators per lane: each
// output quad sums its splits in a fixed order (deterministic for a given split count and G). Small layers have
// few output quads and many splits (up to 512): G = 32 keeps 16 loads per output in flight instead of 4 (the
// 8-group form was one dependent memory round trip per 32 splits, 9-12 us for layers of a few KB)
template <int G>
__global__ __launch_bounds__(256) void k_wgrad_reduce(const float* __restrict__ slab, int splits, int M, int N,
                                                      int layout, int ci_pad, int ci_real, float* __restrict__ dw) {
    __shared__ float4 part[256];
    wgrad_reduce_body<G>(slab, splits, (long long)M * N / 4, N, layout, ci_pad, ci_real, dw, blockIdx.x, gridDim.x,
                         part);
}

// Many weight gradients' slab reduces in ONE launch (sd_wgrad_reduce_batch): job j owns blocks [b0, b0 + nblk) and
// runs exactly the single-job reduce of sd_wgrad_reduce (same G, same block count, so the same summation order and
// bit-identical gradients). A step's 22 reduces were 22 kernel boundaries with small, low-occupancy tails each.
// SD_W_ROWSUM jobs are the ConvTranspose2d bias gradients: column sums of the statistics rows the decoder dgrad
// epilogue left (what sd_stat_rows_sum computes in a launch of its own), one block per channel.
constexpr int WRED_MAX = 48;
struct WRedJob {
    const float* slab;
    float* dw;
    long long total4;
    int splits, N, layout, ci_pad, ci_real, g, b0, nblk;  // g: split groups per block (1, 4, 8 or 32)
};
struct WRedBatch {
    WRedJob j[WRED_MAX];
    int n;
};

__global__ __launch_bounds__(256) void k_wgrad_reduce_batch(const WRedBatch b) {
    __shared__ float4 part[256];
    int k = 0;
    for (int i = 1; i < b.n; ++i) k = (int)blockIdx.x >= b.j[i].b0 ? i : k;  // block-uniform (scalar) job lookup
    const WRedJob& j = b.j[k];
    const int bid = blockIdx.x - j.b0;
    if (j.layout == SD_W_ROWSUM) {
        // column bid of `splits` float2 rows of pitch N, .x summed in fp64: k_sum_finalize's order, bit-identical
        const float2* rows = reinterpret_cast<const float2*>(j.slab);
        double s = 0.0, ss = 0.0;
        for (int r = threadIdx.x; r < j.splits; r += 256) s += rows[(size_t)r * j.N + bid].x;
        block_sum2<256>(s, ss);
        if (threadIdx.x == 0) j.dw[bid] = (float)s;
        return;
    }
    if (j.g == 32)
        wgrad_reduce_body<32>(j.slab, j.splits, j.total4, j.N, j.layout, j.ci_pad, j.ci_real, j.dw, bid, j.nblk, part);
    else if (j.g == 8)
        wgrad_reduce_body<8>(j.slab, j.splits, j.total4, j.N, j.layout, j.ci_pad, j.ci_real, j.dw, bid, j.nblk, part);
    else if (j.g == 4)
        wgrad_reduce_body<4>(j.slab, j.splits, j.total4, j.N, j.layout, j.ci_pad, j.ci_real, j.dw, bid, j.nblk, part);
    else
        wgrad_reduce_body<1>(j.slab, j.splits, j.total4, j.N, j.layout, j.ci_pad, j.ci_real, j.dw, bid, j.nblk, part);
}

}  // namespace

int sd_validate_src(const sd_src* s, const char* what);
// bf16 fast path (conv_fast.hip)
const char* sd_fast_wgrad_name(const sd_src& a, const sd_src& b, int M, int N);
int sd_fast_wgrad_splits(long long P, int M, int N);
int sd_fast_wgrad_gemm(const sd_src& a, const sd_src& b, int batch, int H, int W, int M, int N, float* slab,
                       int splits, hipStream_t st);
// bf16 halo-tiled path for 3x3 weight gradients with M = 32 or M % 64 == 0 (conv_halo.hip)
bool sd_halo_wgrad_ok(const sd_src& a, const sd_src& b, int M);
bool sd_halo_wgrad_shape(int M, int N);
int sd_halo_wgrad_splits(int batch, int H, int W, int M, int N);
const char* sd_halo_wgrad_name(int M, int N, int c0, int H, int W, bool bnb);
int sd_halo_wgrad_bnbwd_blocks(const sd_src& a, const sd_src& b, int M, int N);
int sd_halo_wgrad(const sd_src& a, const sd_src& b, int batch, int H, int W, int M, int N, float* slab, int splits,
                  hipStream_t st, const HaloBnBwd* bnb = nullptr);

extern "C" const char* sd_wgrad_kernel_name(int dtype, const sd_src* a, const sd_src* b, int M, int N) {
    static thread_local char buf[96];
    if (dtype == SD_BF16 && a && b && sd_halo_wgrad_ok(*a, *b, M))
        return sd_halo_wgrad_name(M, N, b->chans[0], a->H, a->W, false);
    if (dtype == SD_BF16 && a && b && !a->pool && !b->pool) return sd_fast_wgrad_name(*a, *b, M, N);
    const WCfg c = pick_wcfg(M, N);
    snprintf(buf, sizeof(buf), "k_wgemm<%s, %d, %d, 2, 2>", dtype == SD_BF16 ? "__bf16" : "float", c.bm, c.bn);
    return buf;
}

// any split count is valid for every kernel (it only sizes the slab); this picks the one the
// dispatched kernel wants for the shape (3x3 wgrads with M = 32 or M % 64 == 0: halo kernel)
extern "C" int sd_wgrad_splits(int dtype, int batch, int H, int W, int M, int N) {
    if (dtype == SD_BF16 && sd_halo_wgrad_shape(M, N)) return sd_halo_wgrad_splits(batch, H, W, M, N);
    if (dtype == SD_BF16) return sd_fast_wgrad_splits((long long)batch * H * W, M, N);
    return compute_splits((long long)batch * H * W, M, N);
}

template <typename T>
static int launch_wg(const WgArgs<T>& p, int splits, hipStream_t st) {
    const WCfg c = pick_wcfg(p.M, p.N);
    dim3 grid(cdiv(p.M, c.bm), cdiv(p.N, c.bn), splits);
    if (c.bm == 32)
        hipLaunchKernelGGL((k_wgemm<T, 32, 64, 2, 2>), grid, dim3(256), 0, st, p);
    else
        hipLaunchKernelGGL((k_wgemm<T, 64, 64, 2, 2>), grid, dim3(256), 0, st, p);
    return sd_check_launch("sd_wgrad_gemm");
}

extern "C" int sd_wgrad_gemm(int dtype, const sd_src* a, const sd_src* b, int batch, int H, int W, int M, int N,
                             float* slab, int splits, sd_stream s) {
    if (int e = sd_validate_src(a, "sd_wgrad_gemm(a)")) return e;
    if (int e = sd_validate_src(b, "sd_wgrad_gemm(b)")) return e;
    SD_REQUIRE(dtype == SD_F32 || dtype == SD_BF16, "sd_wgrad_gemm: dtype %d", dtype);
    SD_REQUIRE(slab && splits > 0 && M > 0 && N > 0 && batch > 0 && H > 0 && W > 0, "sd_wgrad_gemm: bad args");
    GatherSrc ga = make_gather(*a), gb = make_gather(*b);
    SD_REQUIRE(ga.kchunks * 8 == M && gb.kchunks * 8 == N, "sd_wgrad_gemm: M=%d/N=%d do not match sources (%d/%d)", M,
               N, ga.kchunks * 8, gb.kchunks * 8);
    SD_REQUIRE(a->taps == 1 && ga.Hl == H && ga.Wl == W, "sd_wgrad_gemm: A must be a 1x1 source on the grid");
    if (b->taps == 4)
        SD_REQUIRE(gb.Hl == 2 * H && gb.Wl == 2 * W, "sd_wgrad_gemm: sub-pixel B must be 2x the grid");
    else
        SD_REQUIRE(gb.Hl == H && gb.Wl == W, "sd_wgrad_gemm: B grid mismatch");
    const long long P = (long long)batch * H * W;
    SD_REQUIRE(P < (1LL << 31), "sd_wgrad_gemm: too many pixels");
    if (dtype == SD_BF16 && sd_halo_wgrad_ok(*a, *b, M))
        return sd_halo_wgrad(*a, *b, batch, H, W, M, N, slab, splits, to_stream(s));
    if (dtype == SD_BF16 && !a->pool && !b->pool)
        return sd_fast_wgrad_gemm(*a, *b, batch, H, W, M, N, slab, splits, to_stream(s));
    const int pps = cdiv(cdiv(P, splits), BKP) * BKP;
    if (dtype == SD_BF16) {
        WgArgs<__bf16> p{ga, gb, H, W, (int)P, M, N, pps, slab};
        return launch_wg(p, splits, to_stream(s));
    }
    WgArgs<float> p{ga, gb, H, W, (int)P, M, N, pps, slab};
    return launch_wg(p, splits, to_stream(s));
}

extern "C" int sd_wgrad_bnbwd_ok(int dtype, const sd_src* a, const sd_src* b, int M, int N) {
    return dtype == SD_BF16 && a && b ? sd_halo_wgrad_bnbwd_blocks(*a, *b, M, N) : 0;
}

extern "C" const char* sd_wgrad_bnbwd_kernel_name(const sd_src* a, const sd_src* b, int M, int N) {
    if (!a || !b || !sd_halo_wgrad_bnbwd_blocks(*a, *b, M, N)) return "";
    return sd_halo_wgrad_name(M, N, b->chans[0], a->H, a->W, true);
}

extern "C" int sd_wgrad_gemm_bnbwd(int dtype, const sd_src* a, const sd_src* b, int batch, int H, int W, int M, int N,
                                   const void* da, const void* y, const float* scale, const float* shift,
                                   const float* mean, const float* invstd, const float* coef, float* slab, int splits,
                                   sd_stream s) {
    SD_REQUIRE(a, "sd_wgrad_gemm_bnbwd: null a");
    sd_src av = *a;  // a->ptr[0] may be NULL (dy not written): validate the shape with a stand-in pointer
    if (!av.ptr[0]) av.ptr[0] = (const void*)16;
    if (int e = sd_validate_src(&av, "sd_wgrad_gemm_bnbwd(a)")) return e;
    if (int e = sd_validate_src(b, "sd_wgrad_gemm_bnbwd(b)")) return e;
    SD_REQUIRE(dtype == SD_BF16, "sd_wgrad_gemm_bnbwd: bf16 only (dtype %d)", dtype);
    SD_REQUIRE(slab && splits > 0 && batch > 0 && H > 0 && W > 0, "sd_wgrad_gemm_bnbwd: bad args");
    SD_REQUIRE(da && y && scale && shift && mean && invstd && coef, "sd_wgrad_gemm_bnbwd: null pointer");
    SD_REQUIRE(a->taps == 1 && a->chans[0] == M && a->chans[1] == 0 && a->H == H && a->W == W && !a->scale[0],
               "sd_wgrad_gemm_bnbwd: A must be the plain 1x1 dy destination [pixels][M] on the grid");
    SD_REQUIRE(b->taps == 9 && b->H == H && b->W == W && (b->chans[0] + b->chans[1]) * 9 == N,
               "sd_wgrad_gemm_bnbwd: B must be the 3x3 x source on the grid (N = 9 * channels)");
    SD_REQUIRE((long long)batch * H * W < (1LL << 31), "sd_wgrad_gemm_bnbwd: too many pixels");
    SD_REQUIRE(sd_halo_wgrad_bnbwd_blocks(*a, *b, M, N) > 0, "sd_wgrad_gemm_bnbwd: no fused kernel for M=%d N=%d", M,
               N);
    const HaloBnBwd bn{da, y, scale, shift, mean, invstd, coef};
    return sd_halo_wgrad(*a, *b, batch, H, W, M, N, slab, splits, to_stream(s), &bn);
}

// validation and launch shape of one slab reduce (shared by sd_wgrad_reduce and sd_wgrad_reduce_batch)
static int wred_plan(const float* slab, int splits, int M, int N, int layout, int ci_real, float* dw, const char* what,
                     int& ci_pad, int& g, int& blocks) {
    SD_REQUIRE(slab && dw && splits > 0 && M > 0 && N > 0, "%s: bad args", what);
    SD_REQUIRE(layout == SD_W_CONV3 || layout == SD_W_CONVT, "%s: layout %d", what, layout);
    ci_pad = 0;
    if (layout == SD_W_CONV3) {
        SD_REQUIRE(N % 9 == 0, "%s: conv3 N=%d not 9*ci", what, N);
        ci_pad = N / 9;
        SD_REQUIRE(ci_real > 0 && ci_real <= ci_pad, "%s: ci_real %d", what, ci_real);
    } else {
        SD_REQUIRE(N % 4 == 0, "%s: convT N=%d not 4*co", what, N);
    }
    SD_REQUIRE(layout != SD_W_CONV3 || ci_pad % 4 == 0, "%s: ci_pad %d not a multiple of 4", what, ci_pad);
    SD_REQUIRE(((uintptr_t)slab & 15) == 0, "%s: slab not 16-B aligned", what);
    const long long total4 = (long long)M * N / 4;
    static const int g_env = [] {  // SD_WGRED_G=1/4/8/32 forces one form (A/B runs)
        const char* e = getenv("SD_WGRED_G");
        const int v = e ? atoi(e) : 0;
        return v == 1 || v == 4 || v == 8 || v == 32 ? v : 0;
    }();
    // split groups per block: 32 where 8 would leave fewer than two blocks per CU (small layers, many splits); 1 or 4
    // where the splits are few (deep layers: 4-64 splits over up to 0.6 M output quads), so that no thread idles and
    // the blocks stream whole 4-KB rows of each slab instead of summing 32 quads through LDS
    g = g_env ? g_env : ((total4 + 31) / 32 < 512 && splits >= 64 ? 32 : splits <= 16 ? 1 : splits <= 64 ? 4 : 8);
    const int qb = 256 / g;
    const long long nb = (total4 + qb - 1) / qb;
    blocks = (int)(nb > 8192 ? 8192 : nb);
    return 0;
}

extern "C" int sd_wgrad_reduce(const float* slab, int splits, int M, int N, int layout, int ci_real, float* dw,
                               sd_stream s) {
    int ci_pad = 0, blocks = 0, g = 8;
    if (int e = wred_plan(slab, splits, M, N, layout, ci_real, dw, "sd_wgrad_reduce", ci_pad, g, blocks)) return e;
    if (g == 32)
        hipLaunchKernelGGL(k_wgrad_reduce<32>, dim3(blocks), dim3(256), 0, to_stream(s), slab, splits, M, N, layout,
                           ci_pad, ci_real, dw);
    else if (g == 8)
        hipLaunchKernelGGL(k_wgrad_reduce<8>, dim3(blocks), dim3(256), 0, to_stream(s), slab, splits, M, N, layout,
                           ci_pad, ci_real, dw);
    else if (g == 4)
        hipLaunchKernelGGL(k_wgrad_reduce<4>, dim3(blocks), dim3(256), 0, to_stream(s), slab, splits, M, N, layout,
                           ci_pad, ci_real, dw);
    else
        hipLaunchKernelGGL(k_wgrad_reduce<1>, dim3(blocks), dim3(256), 0, to_stream(s), slab, splits, M, N, layout,
                           ci_pad, ci_real, dw);
    return sd_check_launch("sd_wgrad_reduce");
}

extern "C" int sd_wgrad_reduce_batch(const sd_wred_job* jobs, int njobs, sd_stream s) {
    SD_REQUIRE(jobs && njobs >= 0 && njobs <= WRED_MAX, "sd_wgrad_reduce_batch: njobs %d (max %d)", njobs, WRED_MAX);
    if (njobs == 0) return 0;
    WRedBatch b{};
    b.n = njobs;
    long long total_blocks = 0;
    for (int i = 0; i < njobs; ++i) {
        const sd_wred_job& q = jobs[i];
        int ci_pad = 0, blocks = 0, g = 8;
        if (q.layout == SD_W_ROWSUM) {  // rows = splits, pitch N float2, channels ci_real
            SD_REQUIRE(q.slab && q.dw && q.splits > 0 && q.M == 1 && q.ci_real > 0 && q.ci_real <= q.N &&
                           ((uintptr_t)q.slab & 7) == 0,
                       "sd_wgrad_reduce_batch: row-sum job %d: rows %d, M %d, N %d, C %d", i, q.splits, q.M, q.N,
                       q.ci_real);
            blocks = q.ci_real;
        } else if (int e = wred_plan(q.slab, q.splits, q.M, q.N, q.layout, q.ci_real, q.dw, "sd_wgrad_reduce_batch",
                                     ci_pad, g, blocks)) {
            return e;
        }
        b.j[i] = WRedJob{q.slab, q.dw, (long long)q.M * q.N / 4, q.splits, q.N, q.layout, ci_pad, q.ci_real, g,
                         (int)total_blocks, blocks};
        total_blocks += blocks;
    }
    SD_REQUIRE(total_blocks < (1LL << 30), "sd_wgrad_reduce_batch: too many blocks");
    hipLaunchKernelGGL(k_wgrad_reduce_batch, dim3((unsigned)total_blocks), dim3(256), 0, to_stream(s), b);
    return sd_check_launch("sd_wgrad_reduce_batch");
}
