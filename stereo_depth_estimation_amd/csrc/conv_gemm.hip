// Implicit-GEMM convolution on MFMA: conv3x3 forward, conv3x3 data-gradient (flipped weights),
// ConvTranspose2d(k2,s2) forward (pixel-shuffle epilogue) and its data-gradient (sub-pixel gather).
//
// Replaces the reference's mkldnn_convolution / convolution_backward(dgrad) on
// model.py:36,39 (Conv2d k3 p1), model.py:67-73 (ConvTranspose2d k2 s2) and the torch.cat of
// model.py:89-95 (dual-source K loop).  GEMM view: M = batch*H*W pixels (NHWC rows),
// N = output channels, K = taps * Cin.  A (im2col) is gathered straight from NHWC with the
// producer's BN+ReLU(+maxpool) applied on the fly; B is a pre-packed [N][Kpad] weight.
#include "common.h"

namespace {

constexpr int BK = 32;  // K elements per LDS tile (4 chunks of 8 channels)
constexpr int KC = BK / 8;

template <typename T> struct TileLd;
// bf16: 64-B rows, 16-B chunk slots XOR-swizzled so the 16 rows x 16 B of one ds_read_b128
// lane group cover all 64 banks (slot = chunk ^ f((row>>2)&3), f = {0,0,3,3}).
template <> struct TileLd<__bf16> {
    static constexpr int LD = BK;
    __device__ __forceinline__ static int off(int row, int chunk) {
        const int u = (row >> 2) & 3;
        return row * LD + ((chunk ^ ((u >> 1) * 3)) << 3);
    }
    __device__ __forceinline__ static int frag_off(int row, int lane, int ks) {
        // chunk index of k = ks*32 + 8*(lane>>4) is (lane>>4)
        return off(row, lane >> 4) + 0 * ks;
    }
};
// fp32: rows of 32 floats padded to 36 (16-B aligned chunks); 2-way conflicts at worst.
template <> struct TileLd<float> {
    static constexpr int LD = BK + 4;
    __device__ __forceinline__ static int off(int row, int chunk) { return row * LD + chunk * 8; }
    __device__ __forceinline__ static int frag_off(int row, int lane, int ks) { return row * LD + ks * 4 + (lane >> 4); }
};

template <typename T>
struct IgemmArgs {
    GatherSrc a;
    int H, W, M;  // GEMM grid (rows = batch*H*W)
    const T* wp;
    int N, kpad, ktiles;
    int epi;
    T* out0;
    T* out1;
    int n_split;
    const float* bias;
    float* stats;
};

template <typename T, int BM, int BN, int WM, int WN>
__global__ __launch_bounds__(256) void k_igemm(const IgemmArgs<T> p) {
    using MF = Mfma<T>;
    using L = TileLd<T>;
    constexpr int WTM = BM / WM, WTN = BN / WN;
    constexpr int RM = WTM / 16, RN = WTN / 16;
    constexpr int A_LOADS = BM * KC / 256;
    static_assert(WM * WN == 4, "4 waves");
    static_assert(BM * KC % 256 == 0, "A tile split");
    constexpr int A_ELEMS = BM * L::LD, B_ELEMS = BN * L::LD;
    __shared__ __attribute__((aligned(16))) T smem[A_ELEMS + B_ELEMS];
    T* As = smem;
    T* Bs = smem + A_ELEMS;

    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wm = wid / WN, wn = wid % WN;
    const int m0 = blockIdx.x * BM, n0 = blockIdx.y * BN;

    // this thread's A rows: row = tid/KC + i*(256/KC), chunk = tid % KC
    int rb[A_LOADS], rh[A_LOADS], rw[A_LOADS];
    bool rv[A_LOADS];
    const int a_chunk = tid % KC;
#pragma unroll
    for (int i = 0; i < A_LOADS; ++i) {
        const int m = m0 + tid / KC + i * (256 / KC);
        rv[i] = m < p.M;
        const int mm = rv[i] ? m : 0;
        rw[i] = mm % p.W;
        const int t = mm / p.W;
        rh[i] = t % p.H;
        rb[i] = t / p.H;
    }

    f32x4 acc[RM][RN];
#pragma unroll
    for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int j = 0; j < RN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    float av[A_LOADS][8];
    float bv[(BN * KC + 255) / 256][8];

    auto load_tile = [&](int kt) {
#pragma unroll
        for (int i = 0; i < A_LOADS; ++i) {
            if (rv[i])
                gather_chunk<T>(p.a, rb[i], rh[i], rw[i], kt * KC + a_chunk, av[i]);
            else
                zero8(av[i]);
        }
#pragma unroll
        for (int i = 0; i < (BN * KC + 255) / 256; ++i) {
            const int idx = tid + i * 256;
            const int n = n0 + idx / KC, c = idx % KC;
            if (idx < BN * KC && n < p.N)
                load8(p.wp + (size_t)n * p.kpad + kt * BK + c * 8, bv[i]);
            else
                zero8(bv[i]);
        }
    };
    auto store_tile = [&]() {
#pragma unroll
        for (int i = 0; i < A_LOADS; ++i) store8(As + L::off(tid / KC + i * (256 / KC), a_chunk), av[i]);
#pragma unroll
        for (int i = 0; i < (BN * KC + 255) / 256; ++i) {
            const int idx = tid + i * 256;
            if (idx < BN * KC) store8(Bs + L::off(idx / KC, idx % KC), bv[i]);
        }
    };

    load_tile(0);
    for (int kt = 0; kt < p.ktiles; ++kt) {
        store_tile();
        __syncthreads();
        if (kt + 1 < p.ktiles) load_tile(kt + 1);
#pragma unroll
        for (int ks = 0; ks < BK / MF::KSTEP; ++ks) {
            typename MF::frag af[RM], bf[RN];
#pragma unroll
            for (int i = 0; i < RM; ++i) {
                const int row = wm * WTM + i * 16 + (lane & 15);
                if constexpr (sizeof(T) == 2)
                    af[i] = frag_row(As, 0, 0, L::frag_off(row, lane, ks));
                else
                    af[i] = As[L::frag_off(row, lane, ks)];
            }
#pragma unroll
            for (int j = 0; j < RN; ++j) {
                const int row = wn * WTN + j * 16 + (lane & 15);
                if constexpr (sizeof(T) == 2)
                    bf[j] = frag_row(Bs, 0, 0, L::frag_off(row, lane, ks));
                else
                    bf[j] = Bs[L::frag_off(row, lane, ks)];
            }
#pragma unroll
            for (int i = 0; i < RM; ++i)
#pragma unroll
                for (int j = 0; j < RN; ++j) acc[i][j] = MF::mma(af[i], bf[j], acc[i][j]);
        }
        __syncthreads();
    }

    // ---------------------------------------------------------------- epilogue
    const int ccol = lane & 15, crow = (lane >> 4) * 4;
    if (p.epi == SD_EPI_STATS) {
        // per-column (sum, sumsq) of this block's valid rows -> stats[blockIdx.x][n]
        float* red = reinterpret_cast<float*>(smem);  // [WM][BN][2]
#pragma unroll
        for (int j = 0; j < RN; ++j) {
            float s = 0.f, ss = 0.f;
#pragma unroll
            for (int i = 0; i < RM; ++i)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int m = m0 + wm * WTM + i * 16 + crow + r;
                    const float v = m < p.M ? acc[i][j][r] : 0.f;
                    s += v;
                    ss += v * v;
                }
            s += __shfl_xor(s, 16);
            ss += __shfl_xor(ss, 16);
            s += __shfl_xor(s, 32);
            ss += __shfl_xor(ss, 32);
            if (lane < 16) {
                const int col = wn * WTN + j * 16 + lane;
                red[(wm * BN + col) * 2] = s;
                red[(wm * BN + col) * 2 + 1] = ss;
            }
        }
        __syncthreads();
        if (tid < BN && n0 + tid < p.N) {
            float s = 0.f, ss = 0.f;
#pragma unroll
            for (int w = 0; w < WM; ++w) {
                s += red[(w * BN + tid) * 2];
                ss += red[(w * BN + tid) * 2 + 1];
            }
            reinterpret_cast<float2*>(p.stats)[(size_t)blockIdx.x * p.N + n0 + tid] = make_float2(s, ss);
        }
    }
#pragma unroll
    for (int i = 0; i < RM; ++i) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int m = m0 + wm * WTM + i * 16 + crow + r;
            if (m >= p.M) continue;
#pragma unroll
            for (int j = 0; j < RN; ++j) {
                const int n = n0 + wn * WTN + j * 16 + ccol;
                if (n >= p.N) continue;
                const float v = acc[i][j][r];
                if (p.epi == SD_EPI_STORE || p.epi == SD_EPI_STATS) {
                    p.out0[(size_t)m * p.N + n] = from_f32<T>(v);
                } else if (p.epi == SD_EPI_SPLIT) {
                    if (n < p.n_split)
                        p.out0[(size_t)m * p.n_split + n] = from_f32<T>(v);
                    else
                        p.out1[(size_t)m * (p.N - p.n_split) + (n - p.n_split)] = from_f32<T>(v);
                } else {  // SD_EPI_PIXSHUF
                    const int C = p.N >> 2;
                    const int t = n / C, o = n - t * C;
                    const int w = m % p.W, tt = m / p.W, h = tt % p.H, b = tt / p.H;
                    const size_t pix = ((size_t)b * 2 * p.H + 2 * h + (t >> 1)) * (2 * p.W) + 2 * w + (t & 1);
                    p.out0[pix * C + o] = from_f32<T>(v + p.bias[o]);
                }
            }
        }
    }
}

struct Cfg {
    int bm, bn;
};

Cfg pick_cfg(long long M, int N) {
    if (N <= 32) return {128, 32};
    if (N <= 64) return {128, 64};
    if (M >= 128LL * 64) return {128, 128};
    return {64, 128};
}

template <typename T>
int launch_igemm(const IgemmArgs<T>& a, hipStream_t st) {
    const Cfg c = pick_cfg(a.M, a.N);
    dim3 grid(cdiv(a.M, c.bm), cdiv(a.N, c.bn));
    if (c.bm == 128 && c.bn == 32)
        hipLaunchKernelGGL((k_igemm<T, 128, 32, 4, 1>), grid, dim3(256), 0, st, a);
    else if (c.bm == 128 && c.bn == 64)
        hipLaunchKernelGGL((k_igemm<T, 128, 64, 2, 2>), grid, dim3(256), 0, st, a);
    else if (c.bm == 128)
        hipLaunchKernelGGL((k_igemm<T, 128, 128, 2, 2>), grid, dim3(256), 0, st, a);
    else
        hipLaunchKernelGGL((k_igemm<T, 64, 128, 2, 2>), grid, dim3(256), 0, st, a);
    return sd_check_launch("sd_conv_gemm");
}

int validate_src(const sd_src* s, const char* what) {
    SD_REQUIRE(s != nullptr, "%s: null sd_src", what);
    SD_REQUIRE(s->ptr[0] != nullptr, "%s: null source 0", what);
    SD_REQUIRE(s->chans[0] > 0 && s->chans[0] % 8 == 0, "%s: chans[0]=%d must be a positive multiple of 8", what,
               s->chans[0]);
    SD_REQUIRE(s->chans[1] >= 0 && s->chans[1] % 8 == 0, "%s: chans[1]=%d must be a multiple of 8", what, s->chans[1]);
    SD_REQUIRE(s->chans[1] == 0 || s->ptr[1] != nullptr, "%s: null source 1", what);
    SD_REQUIRE(s->taps == 1 || s->taps == 4 || s->taps == 9, "%s: taps=%d", what, s->taps);
    SD_REQUIRE(!(s->pool && s->taps == 4), "%s: pool with sub-pixel taps", what);
    SD_REQUIRE(s->H > 0 && s->W > 0, "%s: bad source dims", what);
    SD_REQUIRE(!s->pool || (s->H % 2 == 0 && s->W % 2 == 0), "%s: pooled source dims must be even", what);
    for (int i = 0; i < 2; ++i)
        if (i == 0 || s->chans[1] > 0)
            SD_REQUIRE(s->xform[i] == SD_IDENT || (s->scale[i] && s->shift[i]), "%s: BN transform without affine",
                       what);
    return SD_OK;
}

}  // namespace

int sd_validate_src(const sd_src* s, const char* what) { return validate_src(s, what); }

// bf16 fast path (conv_fast.hip)
int sd_fast_fwd_rows(long long M, int N);
const char* sd_fast_fwd_name(const sd_src& a, long long M, int N, int epi);
int sd_fast_conv_gemm(const sd_src& a, int batch, int H, int W, const void* wpack, int N, int kpad, int epi, void* out0,
                      void* out1, int n_split, const float* bias, float* stats, hipStream_t st);
// bf16 halo-tiled path for small output-channel 3x3 convs (conv_halo.hip)
bool sd_halo_fwd_ok(const sd_src& a, int N, int epi);
bool sd_halo_fwd_shape(int N);
int sd_halo_fwd_rows(int batch, int H, int W, int N);
const char* sd_halo_fwd_name(int H, int W, int N, int epi, int c0, int c1, bool bns = false, bool wsplit = false,
                             bool oaff = false, bool raw = false);
int sd_halo_conv_fwd(const sd_src& a, int batch, int H, int W, const void* wpack, int N, int kpad, int epi, void* out0,
                     void* out1, int n_split, float* stats, hipStream_t st, const HaloBnSum* bns = nullptr,
                     bool wsplit = false, const float* osc = nullptr, const float* osh = nullptr, void* ws = nullptr,
                     long long ws_bytes = 0);
long long sd_halo_split_ws_bytes(const sd_src& a, int batch, int H, int W, int N, int epi, bool wsplit);
int sd_halo_store_rows(int batch, int H, int W, int N, int ctot);
bool sd_halo_bnsum_ok(const sd_src& a, int N);

bool sd_convt_fwd_ok(const sd_src& a, long long M, int N, int epi);
const char* sd_convt_fwd_name(const sd_src& a, int N);
int sd_convt_fwd(const sd_src& a, int batch, int H, int W, const void* wpack, int N, int kpad, const float* bias,
                 void* out, hipStream_t st);
bool sd_convt_dgrad_ok(const sd_src& a, int N, int epi);
const char* sd_convt_dgrad_name(const sd_src& a, int N, bool bns);
int sd_convt_dgrad_rows(const sd_src& a, int batch, int H, int W, int N);
int sd_convt_dgrad(const sd_src& a, int batch, int H, int W, const void* wpack, int N, int kpad, void* out,
                   const HaloBnSum* bns, float* partials, hipStream_t st);

extern "C" const char* sd_conv_gemm_kernel_name(int dtype, const sd_src* a, int batch, int H, int W, int N, int epi) {
    static thread_local char buf[96];
    const long long M = (long long)batch * H * W;
    if (dtype == SD_BF16 && a && sd_halo_fwd_ok(*a, N, epi))
        return sd_halo_fwd_name(H, W, N, epi, a->chans[0], a->chans[1], false, false, false,
                                a->xform[0] != SD_BNRELU && (a->chans[1] == 0 || a->xform[1] != SD_BNRELU));
    if (dtype == SD_BF16 && a && sd_convt_fwd_ok(*a, (long long)batch * H * W, N, epi)) return sd_convt_fwd_name(*a, N);
    if (dtype == SD_BF16 && a && sd_convt_dgrad_ok(*a, N, epi)) return sd_convt_dgrad_name(*a, N, false);
    if (dtype == SD_BF16 && a && !a->pool) return sd_fast_fwd_name(*a, M, N, epi);
    const Cfg c = pick_cfg(M, N);
    const int wm = c.bn == 32 ? 4 : 2, wn = c.bn == 32 ? 1 : 2;
    snprintf(buf, sizeof(buf), "k_igemm<%s, %d, %d, %d, %d>", dtype == SD_BF16 ? "__bf16" : "float", c.bm, c.bn, wm, wn);
    return buf;
}

// STATS epilogues are only used by forward 3x3 convs (taps 9): the bf16 row count follows the
// kernel that shape dispatches to (halo for N = 32 or N % 64 == 0, else the fast implicit GEMM)
extern "C" int sd_conv_gemm_stat_rows(int dtype, int batch, int H, int W, int N) {
    const long long M = (long long)batch * H * W;
    if (dtype == SD_BF16) return sd_halo_fwd_shape(N) ? sd_halo_fwd_rows(batch, H, W, N) : sd_fast_fwd_rows(M, N);
    return cdiv(M, pick_cfg(M, N).bm);
}

extern "C" int sd_conv_gemm(int dtype, const sd_src* a, int batch, int H, int W, const void* wpack, int N, int kpad,
                            int epi, void* out0, void* out1, int n_split, const float* bias, float* stats,
                            sd_stream s) {
    if (int e = validate_src(a, "sd_conv_gemm")) return e;
    SD_REQUIRE(a->xform[0] != SD_AFFINE && a->xform[1] != SD_AFFINE,
               "sd_conv_gemm: SD_AFFINE is the fp8 gather's transform (sd_conv3x3_fp8)");
    SD_REQUIRE(dtype == SD_F32 || dtype == SD_BF16, "sd_conv_gemm: dtype %d", dtype);
    SD_REQUIRE(batch > 0 && H > 0 && W > 0, "sd_conv_gemm: bad grid %dx%dx%d", batch, H, W);
    SD_REQUIRE(wpack && out0 && N > 0, "sd_conv_gemm: null weights/output or N<=0");
    GatherSrc g = make_gather(*a);
    SD_REQUIRE(kpad % 64 == 0 && kpad >= g.kchunks * 8, "sd_conv_gemm: kpad %d < K %d or not a multiple of 64", kpad,
               g.kchunks * 8);
    // the tap grid must match the GEMM grid
    if (a->taps == 4)
        SD_REQUIRE(g.Hl == 2 * H && g.Wl == 2 * W, "sd_conv_gemm: sub-pixel source must be 2x the grid");
    else
        SD_REQUIRE(g.Hl == H && g.Wl == W, "sd_conv_gemm: source grid %dx%d != GEMM grid %dx%d", g.Hl, g.Wl, H, W);
    SD_REQUIRE(epi >= SD_EPI_STORE && epi <= SD_EPI_SPLIT_STATS, "sd_conv_gemm: epi %d", epi);
    if (epi == SD_EPI_STATS || epi == SD_EPI_SPLIT_STATS)
        SD_REQUIRE(stats != nullptr, "sd_conv_gemm: STATS needs stats buffer");
    if (epi == SD_EPI_SPLIT || epi == SD_EPI_SPLIT_STATS)
        SD_REQUIRE(out1 && n_split > 0 && n_split < N, "sd_conv_gemm: SPLIT needs out1 and 0<n_split<N");
    if (epi == SD_EPI_SPLIT_STATS)
        SD_REQUIRE(dtype == SD_BF16 && sd_halo_fwd_ok(*a, N, epi),
                   "sd_conv_gemm: SPLIT_STATS is the bf16 3x3 halo epilogue (N = 32 or N %% 64 == 0)");
    if (epi == SD_EPI_PIXSHUF) SD_REQUIRE(bias && N % 4 == 0, "sd_conv_gemm: PIXSHUF needs bias and N%%4==0");
    const long long M = (long long)batch * H * W;
    SD_REQUIRE(M < (1LL << 31), "sd_conv_gemm: M too large");
    if (dtype == SD_BF16)  // bf16 epilogues store whole 8-channel (16-B) pieces
        SD_REQUIRE(N % 8 == 0 && ((epi != SD_EPI_SPLIT && epi != SD_EPI_SPLIT_STATS) || n_split % 8 == 0) &&
                       (epi != SD_EPI_PIXSHUF || N % 32 == 0),
                   "sd_conv_gemm: bf16 needs N (and n_split, N/4 for PIXSHUF) multiples of 8");
    if (dtype == SD_BF16 && epi == SD_EPI_STATS && sd_halo_fwd_shape(N))
        SD_REQUIRE(sd_halo_fwd_ok(*a, N, epi), "sd_conv_gemm: bf16 STATS with N=%d needs a 3x3 unpooled source", N);
    if (dtype == SD_BF16 && sd_halo_fwd_ok(*a, N, epi))
        return sd_halo_conv_fwd(*a, batch, H, W, wpack, N, kpad, epi, out0, out1, n_split, stats, to_stream(s));
    if (dtype == SD_BF16 && sd_convt_fwd_ok(*a, (long long)batch * H * W, N, epi))
        return sd_convt_fwd(*a, batch, H, W, wpack, N, kpad, bias, out0, to_stream(s));
    if (dtype == SD_BF16 && sd_convt_dgrad_ok(*a, N, epi))
        return sd_convt_dgrad(*a, batch, H, W, wpack, N, kpad, out0, nullptr, nullptr, to_stream(s));
    if (dtype == SD_BF16 && !a->pool)
        return sd_fast_conv_gemm(*a, batch, H, W, wpack, N, kpad, epi, out0, out1, n_split, bias, stats, to_stream(s));
    // bf16 with an in-gather max pool: generic kernel (its stat-row count differs from the bf16 query)
    SD_REQUIRE(!(dtype == SD_BF16 && epi == SD_EPI_STATS),
               "sd_conv_gemm: bf16 STATS needs an unpooled source (materialise the pool with sd_bnrelu_pool)");
    if (dtype == SD_BF16) {
        IgemmArgs<__bf16> p{g, H, W, (int)M, (const __bf16*)wpack, N, kpad, cdiv(g.kchunks, KC), epi,
                            (__bf16*)out0, (__bf16*)out1, n_split, bias, stats};
        return launch_igemm(p, to_stream(s));
    }
    IgemmArgs<float> p{g, H, W, (int)M, (const float*)wpack, N, kpad, cdiv(g.kchunks, KC), epi,
                       (float*)out0, (float*)out1, n_split, bias, stats};
    return launch_igemm(p, to_stream(s));
}

// the ConvTranspose2d dgrad (4-tap sub-pixel source) through k_convt, where sd_convt_dgrad_ok routes it
static bool convt_bnsum_ok(const sd_src& a, int N) { return a.taps == 4 && sd_convt_dgrad_ok(a, N, SD_EPI_STORE); }

extern "C" int sd_conv_gemm_bnsum_ok(int dtype, const sd_src* a, int N) {
    if (dtype != SD_BF16 || !a || a->xform[0] == SD_AFFINE || a->xform[1] == SD_AFFINE) return 0;
    return sd_halo_bnsum_ok(*a, N) || convt_bnsum_ok(*a, N) ? 1 : 0;
}

extern "C" int sd_conv_gemm_bnsum_rows(const sd_src* a, int batch, int H, int W, int N) {
    if (!a) return 0;
    if (convt_bnsum_ok(*a, N)) return sd_convt_dgrad_rows(*a, batch, H, W, N);
    return sd_halo_store_rows(batch, H, W, N, a->chans[0] + a->chans[1]);
}

extern "C" const char* sd_conv_gemm_bnsum_kernel_name(const sd_src* a, int H, int W, int N) {
    if (a && convt_bnsum_ok(*a, N)) return sd_convt_dgrad_name(*a, N, true);
    if (!a || !sd_halo_bnsum_ok(*a, N)) return "";
    return sd_halo_fwd_name(H, W, N, SD_EPI_STORE, a->chans[0], a->chans[1], true);
}

extern "C" int sd_conv_gemm_bnsum(int dtype, const sd_src* a, int batch, int H, int W, const void* wpack, int N,
                                  int kpad, void* out, const void* y, const float* scale, const float* shift,
                                  const float* mean, const float* invstd, float* partials, sd_stream s) {
    if (int e = validate_src(a, "sd_conv_gemm_bnsum")) return e;
    SD_REQUIRE(sd_conv_gemm_bnsum_ok(dtype, a, N), "sd_conv_gemm_bnsum: bf16 CK = 32 halo shapes only (_ok)");
    SD_REQUIRE(batch > 0 && H > 0 && W > 0 && wpack && out && y && scale && shift && mean && invstd && partials,
               "sd_conv_gemm_bnsum: bad args");
    GatherSrc g = make_gather(*a);
    const HaloBnSum bns{y, scale, shift, mean, invstd};
    if (convt_bnsum_ok(*a, N)) {
        SD_REQUIRE(kpad % 64 == 0 && kpad >= g.kchunks * 8 && g.Hl == 2 * H && g.Wl == 2 * W,
                   "sd_conv_gemm_bnsum: kpad/grid");
        return sd_convt_dgrad(*a, batch, H, W, wpack, N, kpad, out, &bns, partials, to_stream(s));
    }
    SD_REQUIRE(kpad % 64 == 0 && kpad >= g.kchunks * 8 && g.Hl == H && g.Wl == W, "sd_conv_gemm_bnsum: kpad/grid");
    return sd_halo_conv_fwd(*a, batch, H, W, wpack, N, kpad, SD_EPI_STORE, out, nullptr, 0, partials, to_stream(s),
                            &bns);
}

extern "C" int sd_conv3x3_ex_ok(const sd_src* a, int N) {
    return a && a->taps == 9 && a->xform[0] != SD_AFFINE && a->xform[1] != SD_AFFINE && sd_halo_fwd_ok(*a, N, SD_EPI_STORE)
               ? 1
               : 0;
}

extern "C" const char* sd_conv3x3_ex_kernel_name(const sd_src* a, int H, int W, int N, int epi, int flags, int oaff) {
    if (!sd_conv3x3_ex_ok(a, N)) return "";
    return sd_halo_fwd_name(H, W, N, epi, a->chans[0], a->chans[1], false, (flags & SD_CONV_WSPLIT) != 0, oaff != 0,
                            a->xform[0] != SD_BNRELU && (a->chans[1] == 0 || a->xform[1] != SD_BNRELU));
}

extern "C" long long sd_conv3x3_ex_ws_bytes(const sd_src* a, int batch, int H, int W, int N, int epi, int flags) {
    if (!a || !sd_conv3x3_ex_ok(a, N) || batch <= 0) return 0;
    return sd_halo_split_ws_bytes(*a, batch, H, W, N, epi, (flags & SD_CONV_WSPLIT) != 0);
}

extern "C" int sd_conv3x3_ex_ws(const sd_src* a, int batch, int H, int W, const void* wpack, int N, int kpad, int epi,
                                int flags, const float* out_scale, const float* out_shift, void* out, float* stats,
                                void* ws, long long ws_bytes, sd_stream s) {
    if (int e = validate_src(a, "sd_conv3x3_ex")) return e;
    SD_REQUIRE(sd_conv3x3_ex_ok(a, N), "sd_conv3x3_ex: bf16 3x3 halo shapes only (N = 32 or N %% 64 == 0)");
    SD_REQUIRE(epi == SD_EPI_STORE || epi == SD_EPI_STATS, "sd_conv3x3_ex: epi %d (STORE or STATS)", epi);
    SD_REQUIRE((flags & ~SD_CONV_WSPLIT) == 0, "sd_conv3x3_ex: flags %d", flags);
    SD_REQUIRE(!out_scale == !out_shift && (!out_scale || epi == SD_EPI_STORE),
               "sd_conv3x3_ex: the output affine needs both arrays and the STORE epilogue");
    SD_REQUIRE(batch > 0 && H > 0 && W > 0 && wpack && out && N % 8 == 0 && (epi != SD_EPI_STATS || stats),
               "sd_conv3x3_ex: bad args");
    GatherSrc g = make_gather(*a);
    SD_REQUIRE(g.Hl == H && g.Wl == W, "sd_conv3x3_ex: source grid %dx%d != GEMM grid %dx%d", g.Hl, g.Wl, H, W);
    const bool wsp = (flags & SD_CONV_WSPLIT) != 0;
    SD_REQUIRE(kpad % 64 == 0 && kpad >= (wsp ? 2 : 1) * g.kchunks * 8, "sd_conv3x3_ex: kpad %d < K (%d)", kpad,
               (wsp ? 2 : 1) * g.kchunks * 8);
    return sd_halo_conv_fwd(*a, batch, H, W, wpack, N, kpad, epi, out, nullptr, 0, stats, to_stream(s), nullptr, wsp,
                            out_scale, out_shift, ws, ws_bytes);
}

extern "C" int sd_conv3x3_ex(const sd_src* a, int batch, int H, int W, const void* wpack, int N, int kpad, int epi,
                             int flags, const float* out_scale, const float* out_shift, void* out, float* stats,
                             sd_stream s) {
    return sd_conv3x3_ex_ws(a, batch, H, W, wpack, N, kpad, epi, flags, out_scale, out_shift, out, stats, nullptr, 0,
                            s);
}
