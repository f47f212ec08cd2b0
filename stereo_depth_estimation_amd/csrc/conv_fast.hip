// bf16 fast path of the implicit-GEMM convolutions (forward / dgrad / ConvTranspose) and the
// split-K weight gradient.  Same contracts as conv_gemm.hip / wgrad.hip (which remain the fp32
// parity-mode kernels); dispatched for dtype == SD_BF16 and unpooled sources.
//
// Structure (both kernels): 256 threads = 4 waves, K tile = 64 (two 16x16x32 bf16 MFMA k-steps),
// two LDS buffers, register-staged prefetch: the global loads of tile t+1 are issued before the
// MFMAs of tile t and written to the other LDS buffer after them, so one barrier per K tile and
// HBM/L2 latency hides under the MFMAs.  The BN+ReLU of the producing layer is applied to the
// staged registers on the way into LDS.  Row (pixel) decodes use multiply-shift division;
// per-thread tap/channel state advances incrementally (no runtime division in the K loop).
#include "common.h"

namespace {

constexpr int FBK = 64;      // K elements per tile (8 chunks of 8 channels)
constexpr int FKC = FBK / 8;  // chunks per tile


// 128-B LDS rows of 8 16-B chunks; chunk slot XOR (row>>1)&7 makes every ds_read_b128 lane
// group of a 16x32 bf16 MFMA fragment read (and every 8-lane ds_write_b128 group) conflict-free.
__device__ __forceinline__ int swz(int row, int chunk) { return row * FBK + ((chunk ^ ((row >> 1) & 7)) << 3); }

__device__ __forceinline__ uint4 xform_bf16x8(uint4 raw, const float* sc, const float* sh) {
    float v[8];
    const unsigned w[4] = {raw.x, raw.y, raw.z, raw.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        v[2 * i] = __uint_as_float(w[i] << 16);
        v[2 * i + 1] = __uint_as_float(w[i] & 0xffff0000u);
    }
    xform8(v, sc, sh, 0);
    bf16x8 b;
#pragma unroll
    for (int i = 0; i < 8; ++i) b[i] = (__bf16)v[i];
    return *reinterpret_cast<uint4*>(&b);
}

// per-chunk BN affine held in registers (loaded once per K tile, unconditionally)
struct Affine8 {
    float4 s0, s1, h0, h1;
};
__device__ __forceinline__ Affine8 load_affine(bool bn, const float* sc, const float* sh, const void* dummy) {
    const float* s = bn ? sc : (const float*)dummy;
    const float* h = bn ? sh : (const float*)dummy;
    Affine8 a;
    a.s0 = *reinterpret_cast<const float4*>(s);
    a.s1 = *reinterpret_cast<const float4*>(s + 4);
    a.h0 = *reinterpret_cast<const float4*>(h);
    a.h1 = *reinterpret_cast<const float4*>(h + 4);
    return a;
}
// relu(scale*x + shift) of 8 bf16 values: the ReLU is taken on the rounded bf16 pair (v_pk_max_i16 against 0: a
// bf16 is <= 0 exactly when its sign bit is set or it is zero, and rounding preserves the sign), one conversion
// and one max per pair (the per-element form took ~4.5 VALU per element in loaders that are VALU-bound)
__device__ __forceinline__ uint4 xform_reg(uint4 raw, const Affine8& a) {
    const unsigned w[4] = {raw.x, raw.y, raw.z, raw.w};
    const float s[8] = {a.s0.x, a.s0.y, a.s0.z, a.s0.w, a.s1.x, a.s1.y, a.s1.z, a.s1.w};
    const float h[8] = {a.h0.x, a.h0.y, a.h0.z, a.h0.w, a.h1.x, a.h1.y, a.h1.z, a.h1.w};
    unsigned o[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const float lo = __builtin_fmaf(__uint_as_float(w[i] << 16), s[2 * i], h[2 * i]);
        const float hi = __builtin_fmaf(__uint_as_float(w[i] & 0xffff0000u), s[2 * i + 1], h[2 * i + 1]);
        asm("v_cvt_pk_bf16_f32 %0, %1, %2\n\tv_pk_max_i16 %0, %0, 0" : "=v"(o[i]) : "v"(lo), "v"(hi));
    }
    return make_uint4(o[0], o[1], o[2], o[3]);
}

struct SrcF {  // unpooled gather source, bf16
    const __bf16* p0;
    const __bf16* p1;
    const float *sc0, *sh0, *sc1, *sh1;
    int c0, c1, x0, x1;
    int Hs, Ws;  // stored dims
    int taps, cpt, kchunks;
};

static inline SrcF make_srcf(const sd_src& s) {
    SrcF f;
    f.p0 = (const __bf16*)s.ptr[0];
    f.p1 = (const __bf16*)s.ptr[1];
    f.sc0 = s.scale[0];
    f.sh0 = s.shift[0];
    f.sc1 = s.scale[1];
    f.sh1 = s.shift[1];
    f.c0 = s.chans[0];
    f.c1 = s.chans[1];
    f.x0 = s.xform[0];
    f.x1 = s.xform[1];
    f.Hs = s.H;
    f.Ws = s.W;
    f.taps = s.taps;
    f.cpt = (s.chans[0] + s.chans[1]) / 8;
    f.kchunks = f.taps * f.cpt;
    return f;
}

// Per-thread cursor over the K chunks of a gather source (fixed chunk column, advancing tiles).
struct KCursor {
    int tap, cc;  // current tap and chunk-within-tap
    __device__ __forceinline__ void init(int q, int cpt) {
        tap = q / cpt;
        cc = q - tap * cpt;
    }
    __device__ __forceinline__ void advance(int n, int cpt) {
        cc += n;
        while (cc >= cpt) {
            cc -= cpt;
            ++tap;
        }
    }
};

// source-pixel of GEMM-grid pixel (h, w) for a tap; false if outside (zero padding)
__device__ __forceinline__ bool tap_pixel(const SrcF& s, int tap, int h, int w, int& hs, int& ws) {
    if (s.taps == 9) {
        hs = h + tap / 3 - 1;
        ws = w + tap % 3 - 1;
    } else if (s.taps == 4) {
        hs = 2 * h + (tap >> 1);
        ws = 2 * w + (tap & 1);
    } else {
        hs = h;
        ws = w;
    }
    // non-short-circuit: no divergent branches around the caller's loads
    return (tap < s.taps) & (hs >= 0) & (ws >= 0) & (hs < s.Hs) & (ws < s.Ws);
}

// source selection of chunk `cc` (8 channels): base pointer, channel stride/offset, transform
struct ChunkSrc {
    const __bf16* base;
    int C, c, xf;
    const float *sc, *sh;
};
__device__ __forceinline__ ChunkSrc select_chunk(const SrcF& s, int cc) {
    // branch-free (selects): lanes of one wave may sit in different sources
    ChunkSrc r;
    const int c = cc * 8;
    const bool first = c < s.c0;
    r.c = first ? c : c - s.c0;
    r.base = first ? s.p0 : s.p1;
    r.C = first ? s.c0 : s.c1;
    r.xf = first ? s.x0 : s.x1;
    r.sc = (first ? s.sc0 : s.sc1) + r.c;
    r.sh = (first ? s.sh0 : s.sh1) + r.c;
    return r;
}
// Unconditional 16-B load from a clamped address: a per-lane `ok ? load : 0` makes hipcc branch
// around every load and drain vmcnt at each join (serialising the gather's latencies).
__device__ __forceinline__ uint4 load_px(const SrcF& s, const ChunkSrc& cs, bool ok, int b, int hs, int ws) {
    const size_t off = ok ? ((size_t)((size_t)b * s.Hs + hs) * s.Ws + ws) * cs.C + cs.c : 0;
    return *reinterpret_cast<const uint4*>(cs.base + off);
}
__device__ __forceinline__ uint4 zero_unless(bool ok, uint4 v) {
    return ok ? v : make_uint4(0, 0, 0, 0);
}

// =====================================================================================
// forward-style implicit GEMM: out[m][n] = sum_k A[m][k] W[n][k]
// =====================================================================================
struct FwdArgs {
    SrcF a;
    int H, W, M;
    FastDiv fW, fH;
    const __bf16* wp;
    int N, kpad, ktiles;
    int epi;
    __bf16* out0;
    __bf16* out1;
    int n_split;
    const float* bias;
    float* stats;
    int xcd;  // 1: XCD-aware tile order (gridDim.x * gridDim.y % 8 == 0), see k_conv_fwd_bf16
};

// The forward epilogue of one BM x BN tile (accumulators in the MFMA 16x16 layout of 2x2 waves): STATS rows, then
// the bf16 tile staged through `smem` (>= BM x (BN + 8) elements, free of other readers on entry) and written as whole
// 16-B pieces. bcol[jj]: PIXSHUF's bias of this lane's column jj (the caller loads it: k_conv_fwd_ring from LDS, so no
// global load here makes the compiler drain its LDS-DMA ring). Shared by k_conv_fwd_bf16 and k_conv_fwd_ring.
template <int BM, int BN, int WM, int WN>
__device__ __forceinline__ void fwd_epilogue(const FwdArgs& p, f32x4 (&acc)[BM / WM / 16][BN / WN / 16],
                                             const float (&bcol)[BN / WN / 16], __bf16* smem, int m0, int n0, int mt) {
    constexpr int WTM = BM / WM, WTN = BN / WN, RM = WTM / 16, RN = WTN / 16;
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wm = wid / WN, wn = wid % WN;
    const int ccol = lane & 15, crow = (lane >> 4) * 4;
    if (p.epi == SD_EPI_STATS) {
        float* red = reinterpret_cast<float*>(smem);  // [WM][BN][2]
#pragma unroll
        for (int jj = 0; jj < RN; ++jj) {
            float s = 0.f, ss = 0.f;
#pragma unroll
            for (int i = 0; i < RM; ++i)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int m = m0 + wm * WTM + i * 16 + crow + r;
                    // statistics of the values as stored (bf16), like a BN reading the stored tensor
                    const float v = m < p.M ? (float)(__bf16)acc[i][jj][r] : 0.f;
                    s += v;
                    ss += v * v;
                }
            s += __shfl_xor(s, 16);
            ss += __shfl_xor(ss, 16);
            s += __shfl_xor(s, 32);
            ss += __shfl_xor(ss, 32);
            if (lane < 16) {
                const int col = wn * WTN + jj * 16 + lane;
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
            reinterpret_cast<float2*>(p.stats)[(size_t)mt * p.N + n0 + tid] = make_float2(s, ss);
        }
    }
    // Stage the bf16 tile (bias added for PIXSHUF) through LDS as [row][col], then write whole 16-B
    // pieces: rows of the NHWC output, SPLIT halves, or the 2x2 sub-pixel scatter of a convT.
    constexpr int OLD = BN + 8;
    __syncthreads();  // the STATS reduction and the last k-tile are done with smem
    __bf16* st = smem;
    const int C4 = p.N >> 2;
#pragma unroll
    for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r)
#pragma unroll
            for (int jj = 0; jj < RN; ++jj) {
                const int nl = wn * WTN + jj * 16 + ccol;
                float v = acc[i][jj][r];
                if (p.epi == SD_EPI_PIXSHUF) v += bcol[jj];
                st[(wm * WTM + i * 16 + crow + r) * OLD + nl] = (__bf16)v;
            }
    __syncthreads();
    for (int item = tid; item < BM * (BN / 8); item += 256) {
        const int ml = item / (BN / 8), s8 = item - ml * (BN / 8);
        const int m = m0 + ml, n = n0 + s8 * 8;
        if (m >= p.M || n >= p.N) continue;
        const uint4 v = *reinterpret_cast<const uint4*>(st + ml * OLD + s8 * 8);
        if (p.epi == SD_EPI_STORE || p.epi == SD_EPI_STATS) {
            *reinterpret_cast<uint4*>(p.out0 + (size_t)m * p.N + n) = v;
        } else if (p.epi == SD_EPI_SPLIT) {
            if (n < p.n_split)
                *reinterpret_cast<uint4*>(p.out0 + (size_t)m * p.n_split + n) = v;
            else
                *reinterpret_cast<uint4*>(p.out1 + (size_t)m * (p.N - p.n_split) + (n - p.n_split)) = v;
        } else {  // SD_EPI_PIXSHUF: column n = t*C + o, t = 2*dy + dx of the 2x2 output pixel block
            const int t = n / C4, o = n - t * C4;
            const uint32_t tt = fdiv(m, p.fW);
            const int w = m - tt * p.W;
            const int b = fdiv(tt, p.fH), h = tt - b * p.H;
            const size_t pix = ((size_t)b * 2 * p.H + 2 * h + (t >> 1)) * (2 * p.W) + 2 * w + (t & 1);
            *reinterpret_cast<uint4*>(p.out0 + pix * C4 + o) = v;
        }
    }
}

// FA: one unpooled source tensor with 1 tap (on the grid) or 4 sub-pixel taps (at twice its resolution), K a whole
// number of 64-wide tiles, 32-bit offsets: each row's base offset is computed once and a K tile adds the tap's
// constant offset (the general gather's per-load tap test and 64-bit address math paced the ConvTranspose GEMMs)
// NBUF = 1: one LDS buffer (load k-tile t+1 into registers, MFMAs on t, barrier, store t+1, barrier): 24 KB at 64 x 128,
// six blocks per CU instead of three, so other blocks' MFMAs cover each block's load latency. The 64 x 128 FA tiles
// run the ConvTranspose layers at 15x20..30x40 (up1 forward, up3/up4 dgrad: K = 512-1024 over 300-1200 M tiles), where
// one block's k-tile is 16 MFMAs against a 1-2 us load: latency at three blocks per CU, not bandwidth.
template <int BM, int BN, int WM, int WN, bool FA, int NBUF = 2>
__global__ __launch_bounds__(256) void k_conv_fwd_bf16(const FwdArgs p) {
    constexpr int WTM = BM / WM, WTN = BN / WN, RM = WTM / 16, RN = WTN / 16;
    constexpr int AR = BM / 32, BR = (BN + 31) / 32;  // rows per thread (8 chunks per row, 32 rows per pass)
    static_assert(WM * WN == 4, "4 waves");
    static_assert(NBUF == 1 || NBUF == 2, "one or two LDS buffers");
    constexpr int ABUF = BM * FBK, BBUF = BN * FBK;
    constexpr int SMEM = NBUF * (ABUF + BBUF) > BM * (BN + 8) ? NBUF * (ABUF + BBUF) : BM * (BN + 8);  // + staging
    __shared__ __attribute__((aligned(16))) __bf16 smem[SMEM];

    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wm = wid / WN, wn = wid % WN;
    // p.xcd: workgroups are dealt to the 8 XCDs round-robin in launch order (x fastest); renumbered so that each XCD
    // owns a contiguous range of tiles with the N tiles of one M tile adjacent, the N tiles that re-read one A tile run
    // on one XCD at about the same time and share its L2 (launch order put consecutive N tiles of an M tile on
    // different XCDs, so each re-read went to the fabric)
    int mt = blockIdx.x, nt = blockIdx.y;
    if (p.xcd) {
        const int lin = blockIdx.y * gridDim.x + blockIdx.x, tot = gridDim.x * gridDim.y;
        const int l2 = (lin & 7) * (tot >> 3) + (lin >> 3);
        mt = l2 / gridDim.y;
        nt = l2 - mt * gridDim.y;
    }
    const int m0 = mt * BM, n0 = nt * BN;
    const int j = tid & 7, r0 = tid >> 3;

    // A rows owned by this thread
    int rb[AR], rh[AR], rw[AR];
    bool rv[AR];
#pragma unroll
    for (int i = 0; i < AR; ++i) {
        const int m = m0 + r0 + 32 * i;
        rv[i] = m < p.M;
        const uint32_t mm = rv[i] ? m : 0;
        const uint32_t t = fdiv(mm, p.fW);
        rw[i] = mm - t * p.W;
        rb[i] = fdiv(t, p.fH);
        rh[i] = t - rb[i] * p.H;
    }
    KCursor kc;
    kc.init(j, p.a.cpt);
    // FA: the row's source pixel for tap 0 (taps 4: (2h, 2w) at 2x resolution)
    uint32_t pbase[AR];
#pragma unroll
    for (int i = 0; i < AR; ++i) {
        const uint32_t r = (uint32_t)rb[i] * p.H + rh[i];
        pbase[i] = p.a.taps == 4 ? 4 * r * p.W + 2 * rw[i] : r * p.W + rw[i];
    }

    f32x4 acc[RM][RN];
#pragma unroll
    for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int jj = 0; jj < RN; ++jj) acc[i][jj] = f32x4{0.f, 0.f, 0.f, 0.f};

    uint4 ra[AR], rbw[BR];
    bool ain[AR], bok[BR];
    ChunkSrc acs;
    acs.xf = SD_IDENT;
    Affine8 aff;

    auto load_tile = [&](int kt) {
        const int tap = kc.tap;
        if constexpr (FA) {
            const int c = kc.cc * 8;
            acs.xf = p.a.x0;
            aff = load_affine(acs.xf == SD_BNRELU, p.a.sc0 + c, p.a.sh0 + c, p.wp);
            const uint32_t toff = p.a.taps == 4 ? (uint32_t)((tap >> 1) * 2 * p.W + (tap & 1)) : 0u;
#pragma unroll
            for (int i = 0; i < AR; ++i) {
                ain[i] = rv[i];
                const uint32_t off = rv[i] ? (pbase[i] + toff) * (uint32_t)p.a.c0 + c : 0u;
                ra[i] = *reinterpret_cast<const uint4*>(p.a.p0 + off);
            }
        } else {
        acs = select_chunk(p.a, kc.cc);
        aff = load_affine(acs.xf == SD_BNRELU, acs.sc, acs.sh, p.wp);
#pragma unroll
        for (int i = 0; i < AR; ++i) {
            int hs = 0, ws = 0;
            ain[i] = rv[i] & tap_pixel(p.a, tap, rh[i], rw[i], hs, ws);
            ra[i] = load_px(p.a, acs, ain[i], rb[i], hs, ws);
        }
        }
#pragma unroll
        for (int i = 0; i < BR; ++i) {
            const int n = n0 + r0 + 32 * i;
            bok[i] = ((r0 + 32 * i) < BN) & (n < p.N);
            // raw load now, zero-select at store time (a select here would wait for the load)
            rbw[i] = *reinterpret_cast<const uint4*>(p.wp + (size_t)(bok[i] ? n : 0) * p.kpad + kt * FBK + j * 8);
        }
        kc.advance(FKC, p.a.cpt);
    };
    auto store_tile = [&](int buf) {
        __bf16* As = smem + buf * (ABUF + BBUF);
        __bf16* Bs = As + ABUF;
        const bool bn = acs.xf == SD_BNRELU;
#pragma unroll
        for (int i = 0; i < AR; ++i) {
            // zero padding (outside the image, K padding, rows past M) stays exactly zero
            const uint4 t = bn ? xform_reg(ra[i], aff) : ra[i];
            *reinterpret_cast<uint4*>(As + swz(r0 + 32 * i, j)) = zero_unless(ain[i], t);
        }
#pragma unroll
        for (int i = 0; i < BR; ++i)
            if ((r0 + 32 * i) < BN) *reinterpret_cast<uint4*>(Bs + swz(r0 + 32 * i, j)) = zero_unless(bok[i], rbw[i]);
    };

    load_tile(0);
    store_tile(0);
    __syncthreads();
    for (int kt = 0; kt < p.ktiles; ++kt) {
        const int buf = NBUF == 2 ? kt & 1 : 0;
        if (kt + 1 < p.ktiles) load_tile(kt + 1);
        const __bf16* As = smem + buf * (ABUF + BBUF);
        const __bf16* Bs = As + ABUF;
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
            bf16x8 af[RM], bf[RN];
#pragma unroll
            for (int i = 0; i < RM; ++i)
                af[i] = *reinterpret_cast<const bf16x8*>(As + swz(wm * WTM + i * 16 + (lane & 15), kk * 4 + (lane >> 4)));
#pragma unroll
            for (int jj = 0; jj < RN; ++jj)
                bf[jj] = *reinterpret_cast<const bf16x8*>(Bs + swz(wn * WTN + jj * 16 + (lane & 15), kk * 4 + (lane >> 4)));
#pragma unroll
            for (int i = 0; i < RM; ++i)
#pragma unroll
                for (int jj = 0; jj < RN; ++jj)
                    acc[i][jj] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bf[jj], acc[i][jj], 0, 0, 0);
        }
        if constexpr (NBUF == 1) __syncthreads();  // every wave is done reading the one buffer
        if (kt + 1 < p.ktiles) store_tile(NBUF == 2 ? buf ^ 1 : 0);
        __syncthreads();
    }

    float bcol[RN];
#pragma unroll
    for (int jj = 0; jj < RN; ++jj) {
        const int nl = wn * WTN + jj * 16 + (lane & 15), C4 = p.N >> 2;
        const int n = n0 + nl < p.N ? n0 + nl : 0;
        bcol[jj] = p.epi == SD_EPI_PIXSHUF ? p.bias[n - (n / C4) * C4] : 0.f;
    }
    fwd_epilogue<BM, BN, WM, WN>(p, acc, bcol, smem, m0, n0, mt);
}

// =====================================================================================
// k_conv_fwd_ring (opt-in): the data gradients of the 15x20 / 30x40 ConvTranspose layers (up3 / up4: K = 512-1024 over
// 600-1200 tiles) as a persistent kernel with an LDS-DMA ring. k_conv_fwd_bf16 keeps one K tile per block in flight (its layers
// ran at 1.7 TB/s with MFMA busy 0.15, PMC r06a). Here one 512-thread block per CU owns a fixed set of 128 x 128 tiles
// (half the weight re-reads of 64 x 128); waves 4-7 stream the A / B tiles of every (tile, K tile) step global -> LDS
// with buffer_load ... lds into a 4-stage ring, three steps ahead and across tile boundaries, while waves 0-3 run the
// MFMAs and the epilogue. The MFMA order (K tiles ascending, two 16x16x32 k-steps each, the swz() fragments) is
// k_conv_fwd_bf16's: bit-identical outputs. Measured (bench per-layer times, same box): up4 dgrad (K = 1024) 43-44 us
// against 46-48 for 64 x 128 tiles but 41 for the single-buffered 128 x 128 ones (now the default there), up3 dgrad
// (K = 512: an epilogue every 8 steps with no other block to overlap it) 46-47; with the MFMA waves issuing the DMA
// themselves 69 / 69 us (8 pieces per step, each holding its wave 60-185 cycles, outlasted the step's 32 MFMAs). The
// up4 forward (BN+ReLU source) measured slower with the transform on either side (MFMA waves, after the fragment
// read: 58 vs 52 us; loader waves, in LDS one step ahead: 67 us). Opt-in: SD_FWD_RING=1 (ring_mode).
// =====================================================================================
constexpr int RG_BM = 128, RG_BN = 128, RG_ST = 4;
constexpr int RG_STAGE = RG_BM * (RG_BN + 8);  // elements per stage: A + B tiles, or the epilogue's staging tile
static_assert(RG_STAGE >= (RG_BM + RG_BN) * FBK, "a stage holds the A and B tiles");
constexpr int RG_C4MAX = 512;  // PIXSHUF: bias entries (N / 4)

__global__ __launch_bounds__(512, 1) void k_conv_fwd_ring(const FwdArgs p, int lcpt, unsigned a_bytes) {
    constexpr int BM = RG_BM, BN = RG_BN, WM = 2, WN = 2, WTM = BM / WM, WTN = BN / WN, RM = WTM / 16, RN = WTN / 16;
    constexpr unsigned OOB = 0x80000000u;
    __shared__ __attribute__((aligned(16))) __bf16 ring[RG_ST * RG_STAGE];
    __shared__ float sbias[RG_C4MAX];
    // waves 0-3 run the MFMAs and the epilogue, waves 4-7 issue the LDS-DMA (a piece costs its issuing wave 60-185
    // cycles, MI355X_MICROARCH.md: issued by the MFMA waves, the 8 pieces per step outlasted the step's 32 MFMAs)
    const int tid = threadIdx.x & 255, lane = tid & 63, wid = tid >> 6;
    const bool loader = threadIdx.x >= 256;
    const int wm = wid / WN, wn = wid % WN;
    const int ntn = (p.N + BN - 1) / BN, ntm = (p.M + BM - 1) / BM, T = ntm * ntn;
    // tiles of this block: XCD x (= blockIdx % 8, the hardware's round-robin) owns the contiguous range [lo, hi) of the
    // N-fastest tile order, and its blocks take every (grid / 8)-th tile of it: the N tiles that re-read one A tile and
    // the whole weight matrix stay in one L2
    const int xcd = blockIdx.x & 7, li = blockIdx.x >> 3, nb8 = gridDim.x >> 3;
    const int lo = (int)((long long)xcd * T / 8), hi = (int)((long long)(xcd + 1) * T / 8);
    const int ntile = hi - lo > li ? (hi - lo - li + nb8 - 1) / nb8 : 0;
    if (p.epi == SD_EPI_PIXSHUF)
        for (int c = threadIdx.x; c < (p.N >> 2); c += 512) sbias[c] = p.bias[c];
    if (ntile == 0) return;  // block-uniform; no barrier has been passed
    const int S = ntile * p.ktiles;
    const int cmask = (1 << lcpt) - 1;
    const bool taps4 = p.a.taps == 4;

    // DMA geometry: wave-instruction g = 4 * wid + j fills LDS slots 64 g .. 64 g + 63 (16 B each, 8 per 64-element
    // row) of the A tile and of the B tile; lane l's slot is row 8 g + l / 8, physical chunk l % 8, i.e. logical chunk
    // (l % 8) ^ ((row / 2) % 8) (swz())
    int rrow[4], clog[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int row = (4 * wid + j) * 8 + (lane >> 3);
        rrow[j] = row;
        clog[j] = (lane & 7) ^ ((row >> 1) & 7);
    }
    const __amdgpu_buffer_rsrc_t rsa = __builtin_amdgcn_make_buffer_rsrc((void*)p.a.p0, (short)0, (int)a_bytes, 0x00020000);
    const __amdgpu_buffer_rsrc_t rsb =
        __builtin_amdgcn_make_buffer_rsrc((void*)p.wp, (short)0, p.N * p.kpad * 2, 0x00020000);
    const unsigned lds0 = (unsigned)(uintptr_t)ring + (unsigned)wid * 4096u;

    // DMA cursor: the (tile, K tile) step the next issue() loads
    int d_i = 0, d_kt = 0;
    unsigned a_pb[4], b_off[4];  // per row: source pixel of tap 0 (OOB past M), weight row byte offset (OOB past N)
    auto tile_of = [&](int i, int& mt, int& nt) {
        const int lin = lo + li + i * nb8;
        mt = lin / ntn;
        nt = lin - mt * ntn;
    };
    auto issue = [&](int s) __attribute__((always_inline)) {
        const bool live = s < S;
        if (live && d_kt == 0) {
            int mt, nt;
            tile_of(d_i, mt, nt);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const int m = mt * BM + rrow[j];
                const uint32_t mm = m < p.M ? m : 0;
                const uint32_t t = fdiv(mm, p.fW);
                const uint32_t w = mm - t * p.W;  // t = b * H + h
                a_pb[j] = m < p.M ? (taps4 ? 4 * t * p.W + 2 * w : t * p.W + w) : OOB;
                const int n = nt * BN + rrow[j];
                b_off[j] = n < p.N ? (unsigned)(n * p.kpad) * 2u : OOB;
            }
        }
        const unsigned m0b = __builtin_amdgcn_readfirstlane(lds0 + (unsigned)((s % RG_ST) * RG_STAGE * 2));
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int q = d_kt * FKC + clog[j];
            const int tap = q >> lcpt, cc = q & cmask;
            const unsigned toff = taps4 ? (unsigned)((tap >> 1) * 2 * p.W + (tap & 1)) : 0u;
            const unsigned off =
                live && a_pb[j] != OOB ? ((a_pb[j] + toff) * (unsigned)p.a.c0 + (unsigned)cc * 8u) * 2u : OOB;
            unsigned keep;
            asm volatile(
                "s_mov_b32 %0, m0\n\t"
                "s_mov_b32 m0, %2\n\t"
                "s_nop 0\n\t"
                "buffer_load_dwordx4 %1, %3, 0 offen lds\n\t"
                "s_mov_b32 m0, %0"
                : "=&s"(keep)
                : "v"(off), "s"(m0b + (unsigned)j * 1024u), "s"(rsa)
                : "memory");
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const unsigned off =
                live && b_off[j] != OOB ? b_off[j] + (unsigned)(d_kt * FBK + clog[j] * 8) * 2u : OOB;
            unsigned keep;
            asm volatile(
                "s_mov_b32 %0, m0\n\t"
                "s_mov_b32 m0, %2\n\t"
                "s_nop 0\n\t"
                "buffer_load_dwordx4 %1, %3, 0 offen lds\n\t"
                "s_mov_b32 m0, %0"
                : "=&s"(keep)
                : "v"(off), "s"(m0b + (unsigned)(BM * FBK * 2) + (unsigned)j * 1024u), "s"(rsb)
                : "memory");
        }
        if (live && ++d_kt == p.ktiles) {
            d_kt = 0;
            ++d_i;
        }
    };

    if (loader) {
        // the same step sequence and barriers as the MFMA waves: one per step, two more in each tile's epilogue
#pragma unroll
        for (int s = 0; s < RG_ST - 1; ++s) issue(s);
        int kt = 0;
        for (int s = 0; s < S; ++s) {
            // step s's loads (this wave's) have landed when at most the two later steps' 16 are outstanding; the
            // barrier makes every loader's visible and retires step s - 1's readers of the stage refilled next
            asm volatile("s_waitcnt vmcnt(%0)" ::"i"((RG_ST - 2) * 8) : "memory");
            __syncthreads();
            issue(s + RG_ST - 1);
            if (++kt == p.ktiles) {
                kt = 0;
                __syncthreads();  // fwd_epilogue: MFMA waves done with the stage
                __syncthreads();  // fwd_epilogue: staging tile written
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the trailing (out-of-range) ring loads land before exit
        return;
    }
    f32x4 acc[RM][RN];
#pragma unroll
    for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int jj = 0; jj < RN; ++jj) acc[i][jj] = f32x4{0.f, 0.f, 0.f, 0.f};
    int c_i = 0, c_kt = 0, mt, nt;
    tile_of(0, mt, nt);
    for (int s = 0; s < S; ++s) {
        __syncthreads();
        const __bf16* As = ring + (s % RG_ST) * RG_STAGE;
        const __bf16* Bs = As + BM * FBK;
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
            bf16x8 af[RM], bf[RN];
#pragma unroll
            for (int i = 0; i < RM; ++i)
                af[i] = *reinterpret_cast<const bf16x8*>(As + swz(wm * WTM + i * 16 + (lane & 15), kk * 4 + (lane >> 4)));
#pragma unroll
            for (int jj = 0; jj < RN; ++jj)
                bf[jj] = *reinterpret_cast<const bf16x8*>(Bs + swz(wn * WTN + jj * 16 + (lane & 15), kk * 4 + (lane >> 4)));
#pragma unroll
            for (int i = 0; i < RM; ++i)
#pragma unroll
                for (int jj = 0; jj < RN; ++jj)
                    acc[i][jj] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bf[jj], acc[i][jj], 0, 0, 0);
        }
        if (++c_kt == p.ktiles) {
            const int m0 = mt * BM, n0 = nt * BN;
            float bcol[RN];
#pragma unroll
            for (int jj = 0; jj < RN; ++jj) {
                const int n = n0 + wn * WTN + jj * 16 + (lane & 15), C4 = p.N >> 2;
                const int nc = n < p.N ? n : 0;
                bcol[jj] = p.epi == SD_EPI_PIXSHUF ? sbias[nc - (nc / C4) * C4] : 0.f;
            }
            // the epilogue's first barrier retires this stage's readers; its staging tile is this stage, refilled
            // only after the next step's barrier
            fwd_epilogue<BM, BN, WM, WN>(p, acc, bcol, ring + (s % RG_ST) * RG_STAGE, m0, n0, mt);
#pragma unroll
            for (int i = 0; i < RM; ++i)
#pragma unroll
                for (int jj = 0; jj < RN; ++jj) acc[i][jj] = f32x4{0.f, 0.f, 0.f, 0.f};
            c_kt = 0;
            if (++c_i < ntile) tile_of(c_i, mt, nt);
        }
    }
}

// =====================================================================================
// weight gradient: slab[z][m][n] = sum_p A(p, m) * B(p, n) over the z-th pixel range
// =====================================================================================
struct WgfArgs {
    SrcF a, b;
    int H, W, P;
    FastDiv fW, fH;
    int M, N;
    int pix_per_split;
    float* slab;
    int xcd;  // 1: XCD-aware block order (grid size % 8 == 0), see k_wgrad_bf16
};

// transposed bf16 fragment with the consistent per-k-step pixel permutation of wgrad.hip
__device__ __forceinline__ bf16x8 frag_tr64(const __bf16* lds, int ld, int col0, int lane, int kk) {
    const int i = lane & 15, g = lane >> 4;
    const int q = i >> 2, pp = i & 3;
    const int rr = 32 * kk + 16 * (g >> 1) + 4 * (g & 1) + q;
    const __bf16* a0 = lds + rr * ld + col0 + 4 * pp;
    bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(a0));
    bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((lds_bf16x4*)(a0 + 8 * ld));
    bf16x8 r;
#pragma unroll
    for (int t = 0; t < 4; ++t) {
        r[t] = lo[t];
        r[t + 4] = hi[t];
    }
    return r;
}

// CT: the ConvTranspose2d weight gradient (A = a 1x1 source on the GEMM grid, B = the 4-tap sub-pixel source at
// twice its resolution). Pixel m = r*W + w of the grid reads A at m*Ca and B at (4*r*W + 2*w + toff)*Cb with 32-bit
// element offsets: one division per B load instead of two per load plus the general tap test (the loader's VALU,
// ~240 per 64-pixel tile per lane in the general form, paced these layers at ~300 TFLOP/s)
// (A single-buffered form at twice the resident blocks per CU, as k_conv_fwd_bf16's NBUF = 1, measured no faster here:
// 49.8-51.0 vs 50.3-50.4 us at 128 x 128, 87.1-87.5 vs 86.7-87.2 us at 64 x 128; same box, two rounds.)
template <int BM, int BN, int WM, int WN, bool CT>
__global__ __launch_bounds__(256) void k_wgrad_bf16(const WgfArgs p) {
    constexpr int BKP = 64;
    constexpr int LDA = BM + 16, LDB = BN + 16;
    constexpr int WTM = BM / WM, WTN = BN / WN, RM = WTM / 16, RN = WTN / 16;
    constexpr int ACH = BM / 8, BCH = BN / 8;          // chunks per pixel row
    constexpr int APR = 256 / ACH, BPR = 256 / BCH;    // pixel rows per pass
    constexpr int AL = BKP / APR, BL = BKP / BPR;      // passes
    static_assert(WM * WN == 4, "4 waves");
    constexpr int ABUF = BKP * LDA, BBUF = BKP * LDB;
    __shared__ __attribute__((aligned(16))) __bf16 smem[2 * (ABUF + BBUF)];

    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int wm = wid / WN, wn = wid % WN;
    // p.xcd: the (M, N) tiles of one pixel split read the same pixel range of both operands (each a slice of it); in
    // launch order they were dealt to different XCDs, so each XCD fetched the range again (4A + 2B bytes for 2 x 4
    // tiles, measured 309 MB per launch against ~120 MB of operands). Renumbered so that each XCD owns a contiguous
    // range of splits with all their tiles, which then share its L2.
    int bx = blockIdx.x, by = blockIdx.y, bz = blockIdx.z;
    if (p.xcd) {
        const int gxy = gridDim.x * gridDim.y;
        const int lin = blockIdx.z * gxy + blockIdx.y * gridDim.x + blockIdx.x, tot = gxy * gridDim.z;
        const int l2 = (lin & 7) * (tot >> 3) + (lin >> 3);
        bz = l2 / gxy;
        const int r = l2 - bz * gxy;
        by = r / gridDim.x;
        bx = r - by * gridDim.x;
    }
    const int m0 = bx * BM, n0 = by * BN;
    const int p_begin = bz * p.pix_per_split;
    const int p_end = min(p.P, p_begin + p.pix_per_split);
    const int ntiles = p_end > p_begin ? (p_end - p_begin + BKP - 1) / BKP : 0;

    // fixed chunk columns of this thread: A (channel chunk), B (tap, channel chunk)
    const int ajc = tid % ACH, apr = tid / ACH;
    const int bjc = tid % BCH, bpr = tid / BCH;
    const int aq = m0 / 8 + ajc, bq = n0 / 8 + bjc;
    const bool a_ok = aq < p.a.kchunks, b_ok = bq < p.b.kchunks;
    int a_tap = 0, a_cc = 0, b_tap = 0, b_cc = 0;
    if (a_ok) { a_tap = aq / p.a.cpt; a_cc = aq - a_tap * p.a.cpt; }
    if (b_ok) { b_tap = bq / p.b.cpt; b_cc = bq - b_tap * p.b.cpt; }
    const ChunkSrc acs = select_chunk(p.a, a_cc), bcs = select_chunk(p.b, b_cc);
    // chunk columns are fixed per thread: the BN affines live in registers for the whole kernel
    const Affine8 aaff = load_affine(acs.xf == SD_BNRELU, acs.sc, acs.sh, p.slab);
    const Affine8 baff = load_affine(bcs.xf == SD_BNRELU, bcs.sc, bcs.sh, p.slab);

    f32x4 acc[RM][RN];
#pragma unroll
    for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int jj = 0; jj < RN; ++jj) acc[i][jj] = f32x4{0.f, 0.f, 0.f, 0.f};

    uint4 ra[AL], rbv[BL];
    bool av[AL], bv_[BL];
    // CT: B's tap offset in sub-pixels, and the sources' element bases of this thread's fixed chunk columns
    const uint32_t btoff = (uint32_t)((b_tap >> 1) * 2 * p.W + (b_tap & 1));
    const __bf16* abase = acs.base + acs.c;
    const __bf16* bbase = bcs.base + bcs.c;
    // branch-free gathers (see load_px): every lane issues its loads, invalid ones read a safe address
    auto load_tile = [&](int t) {
        const int pt = p_begin + t * BKP;
        if constexpr (CT) {
#pragma unroll
            for (int i = 0; i < AL; ++i) {
                const int px = pt + apr + i * APR;
                av[i] = a_ok & (px < p_end);
                const uint32_t m = av[i] ? px : 0;
                ra[i] = *reinterpret_cast<const uint4*>(abase + m * (uint32_t)acs.C);
            }
#pragma unroll
            for (int i = 0; i < BL; ++i) {
                const int px = pt + bpr + i * BPR;
                bv_[i] = b_ok & (px < p_end);
                const uint32_t m = bv_[i] ? px : 0;
                const uint32_t r = fdiv(m, p.fW), w = m - r * p.W;
                rbv[i] = *reinterpret_cast<const uint4*>(bbase + ((4 * r * p.W + 2 * w + btoff) * (uint32_t)bcs.C));
            }
            return;
        }
#pragma unroll
        for (int i = 0; i < AL; ++i) {
            const int px = pt + apr + i * APR;
            const uint32_t pxc = px < p_end ? px : 0;
            const uint32_t tt = fdiv(pxc, p.fW);
            const int w = pxc - tt * p.W;
            const int b = fdiv(tt, p.fH), h = tt - b * p.H;
            int hs = 0, ws = 0;
            av[i] = a_ok & (px < p_end) & tap_pixel(p.a, a_tap, h, w, hs, ws);
            ra[i] = load_px(p.a, acs, av[i], b, hs, ws);
        }
#pragma unroll
        for (int i = 0; i < BL; ++i) {
            const int px = pt + bpr + i * BPR;
            const uint32_t pxc = px < p_end ? px : 0;
            const uint32_t tt = fdiv(pxc, p.fW);
            const int w = pxc - tt * p.W;
            const int b = fdiv(tt, p.fH), h = tt - b * p.H;
            int hs = 0, ws = 0;
            bv_[i] = b_ok & (px < p_end) & tap_pixel(p.b, b_tap, h, w, hs, ws);
            rbv[i] = load_px(p.b, bcs, bv_[i], b, hs, ws);
        }
    };
    auto store_tile = [&](int buf) {
        __bf16* As = smem + buf * (ABUF + BBUF);
        __bf16* Bs = As + ABUF;
        const bool abn = acs.xf == SD_BNRELU, bbn = bcs.xf == SD_BNRELU;
#pragma unroll
        for (int i = 0; i < AL; ++i) {
            const uint4 v = abn ? xform_reg(ra[i], aaff) : ra[i];
            *reinterpret_cast<uint4*>(As + (apr + i * APR) * LDA + ajc * 8) = zero_unless(av[i], v);
        }
#pragma unroll
        for (int i = 0; i < BL; ++i) {
            const uint4 v = bbn ? xform_reg(rbv[i], baff) : rbv[i];
            *reinterpret_cast<uint4*>(Bs + (bpr + i * BPR) * LDB + bjc * 8) = zero_unless(bv_[i], v);
        }
    };

    if (ntiles > 0) {
        load_tile(0);
        store_tile(0);
    }
    __syncthreads();
    for (int t = 0; t < ntiles; ++t) {
        const int buf = t & 1;
        if (t + 1 < ntiles) load_tile(t + 1);
        const __bf16* As = smem + buf * (ABUF + BBUF);
        const __bf16* Bs = As + ABUF;
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {
            bf16x8 af[RM], bf[RN];
#pragma unroll
            for (int i = 0; i < RM; ++i) af[i] = frag_tr64(As, LDA, wm * WTM + i * 16, lane, kk);
#pragma unroll
            for (int jj = 0; jj < RN; ++jj) bf[jj] = frag_tr64(Bs, LDB, wn * WTN + jj * 16, lane, kk);
#pragma unroll
            for (int i = 0; i < RM; ++i)
#pragma unroll
                for (int jj = 0; jj < RN; ++jj)
                    acc[i][jj] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bf[jj], acc[i][jj], 0, 0, 0);
        }
        if (t + 1 < ntiles) store_tile(buf ^ 1);
        __syncthreads();
    }

    float* slab = p.slab + (size_t)bz * p.M * p.N;
    const int ccol = lane & 15, crow = (lane >> 4) * 4;
#pragma unroll
    for (int i = 0; i < RM; ++i)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
            const int m = m0 + wm * WTM + i * 16 + crow + r;
            if (m >= p.M) continue;
#pragma unroll
            for (int jj = 0; jj < RN; ++jj) {
                const int n = n0 + wn * WTN + jj * 16 + ccol;
                if (n < p.N) slab[(size_t)m * p.N + n] = acc[i][jj][r];
            }
        }
}

// ------------------------------------------------------------------ BN + ReLU + MaxPool2d(2) materialisation
// out[b][h2][w2][c] = max over the 2x2 window of relu(scale*y + shift)   (model.py:59,83-86)
__global__ __launch_bounds__(256) void k_bnrelu_pool_bf16(const __bf16* __restrict__ y, const float* sc,
                                                         const float* sh, int batch, int H, int W, int C,
                                                         __bf16* __restrict__ out) {
    const int cpr = C / 8, H2 = H / 2, W2 = W / 2;
    const long long total = (long long)batch * H2 * W2 * cpr;
    for (long long e = blockIdx.x * 256LL + threadIdx.x; e < total; e += (long long)gridDim.x * 256) {
        const long long win = e / cpr;
        const int c = (int)(e - win * cpr) * 8;
        const int w2 = (int)(win % W2);
        const long long t = win / W2;
        const int h2 = (int)(t % H2), b = (int)(t / H2);
        float o[8];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            float v[8];
            load8(y + (((size_t)b * H + 2 * h2 + (k >> 1)) * W + 2 * w2 + (k & 1)) * C + c, v);
            xform8(v, sc, sh, c);
#pragma unroll
            for (int i = 0; i < 8; ++i) o[i] = k == 0 ? v[i] : fmaxf(o[i], v[i]);
        }
        store8_nt(out + (size_t)win * C + c, o);
    }
}

struct FCfg {
    int bm, bn, wm, wn;
};
// fa1: the shape runs the single-buffered FA instances (k_conv_fwd_bf16<..., true, 1>)
FCfg pick_fwd(long long M, int N, bool fa1) {
    const char* e = getenv("SD_FWD_BM");  // 64 / 128: the row tile for N > 64 at large M (read per call: A/B, tests)
    const int bm_env = e && *e ? atoi(e) : 0;
    if (N <= 32) return {256, 32, 4, 1};
    if (N <= 64) return {128, 64, 2, 2};
    // 128 x 128 at large M in the single-buffered FA form: a third fewer bytes staged per MAC than 64 x 128, at three
    // blocks per CU (the up3 / up4 ConvTranspose GEMMs, r06 gpurun_out/g10ab: up4 fwd 51 -> 44 us, up4 dgrad 46 ->
    // 41, up3 dgrad 46 -> 40). The double-buffered 128-row tiles hold two blocks per CU and measured slower than
    // 64 x 128 (r03: up4 dgrad 67 vs 54 us), so the general gather keeps 64 rows.
    if (M >= 128LL * 96 && (bm_env == 128 || (bm_env != 64 && fa1))) return {128, 128, 2, 2};
    return {64, 128, 2, 2};
}
FCfg pick_wg(int M, int N) {
    (void)N;
    if (M <= 32) return {32, 128, 1, 4};
    if (M <= 64) return {64, 128, 2, 2};
    return {128, 128, 2, 2};
}

}  // namespace

// SD_FFA=0: the general gather for the ConvTranspose-shaped implicit GEMMs too (A/B runs)
static bool ffa_shape(const sd_src& a) {
    static const bool on = [] {
        const char* e = getenv("SD_FFA");
        return !(e && atoi(e) == 0);
    }();
    return on && !a.pool && a.chans[1] == 0 && (a.taps == 1 || a.taps == 4) && (a.chans[0] * (a.taps == 4 ? 4 : 1)) % 64 == 0;
}

// ---------------------------------------------------------------------- host dispatch (bf16)
static int fwd_nbuf();

// the FA gather (one unpooled source, 1 or 4 taps, K a whole number of tiles, 32-bit element offsets)
static bool fa_path(const sd_src& a, long long M) {
    return ffa_shape(a) && M * (a.taps == 4 ? 4 : 1) * a.chans[0] < (1LL << 31);
}

// the STATS epilogue's row count (3x3 sources: never the FA gather)
int sd_fast_fwd_rows(long long M, int N) { return cdiv(M, pick_fwd(M, N, false).bm); }

// k_conv_fwd_ring's shapes, opt-in (SD_FWD_RING=1, read per call; -1: not routed there): untransformed FA sources with
// N > 64 and K >= 1024 (the up4 ConvTranspose dgrad), a power-of-two channel count, a STORE / SPLIT / PIXSHUF epilogue
// (the STATS row count stays the tiled kernel's) and at least 256 of its 128 x 128 tiles (one per CU). Measured slower
// than the single-buffered 128 x 128 tiles (up4 dgrad 44 vs 41 us), faster than the 64 x 128 ones.
static int ring_mode(const sd_src& a, long long M, int N, int epi) {
    const char* e = getenv("SD_FWD_RING");
    if (!(e && *e && atoi(e) == 1)) return -1;
    const int c0 = a.chans[0], taps = a.taps;
    if (!(fa_path(a, M) && N > 64)) return -1;
    if (epi != SD_EPI_STORE && epi != SD_EPI_SPLIT && epi != SD_EPI_PIXSHUF) return -1;
    if (c0 < 8 || (c0 & (c0 - 1)) != 0 || (taps * c0) % FBK != 0) return -1;
    if (taps * c0 < 16 * FBK) return -1;  // >= 16 K tiles per output tile: at 8 (up3 dgrad) its epilogues cost the gain
    if (M * taps * c0 * 2 > 0x7fffffffLL || (long long)N * 2048 > 0x7fffffffLL) return -1;
    if (a.xform[0] != SD_IDENT) return -1;
    if (epi == SD_EPI_PIXSHUF && N / 4 > RG_C4MAX) return -1;
    if (cdiv(M, RG_BM) * cdiv(N, RG_BN) < 256) return -1;
    return 0;
}

const char* sd_fast_fwd_name(const sd_src& a, long long M, int N, int epi) {
    static thread_local char buf[96];
    const int rm = ring_mode(a, M, N, epi);
    if (rm >= 0) return "k_conv_fwd_ring";
    const bool fa = fa_path(a, M);
    const FCfg c = pick_fwd(M, N, fa && fwd_nbuf() == 1);
    const bool one = fa && c.bn == 128 && fwd_nbuf() == 1;  // the single-buffered instances
    snprintf(buf, sizeof(buf), "k_conv_fwd_bf16<%d, %d, %d, %d, %s%s>", c.bm, c.bn, c.wm, c.wn, fa ? "true" : "false",
             one ? ", 1" : "");
    return buf;
}

// SD_FWG_CT=0: the general gather for the ConvTranspose weight gradients too (A/B runs)
static bool fwg_ct_enabled() {
    static const bool on = [] {
        const char* e = getenv("SD_FWG_CT");
        return !(e && atoi(e) == 0);
    }();
    return on;
}

static bool fwg_ct_shape(const sd_src& a, const sd_src& b) {
    return a.taps == 1 && b.taps == 4 && !a.pool && !b.pool && a.chans[1] == 0 && b.chans[1] == 0 && b.H == 2 * a.H &&
           b.W == 2 * a.W && fwg_ct_enabled();
}

const char* sd_fast_wgrad_name(const sd_src& a, const sd_src& b, int M, int N) {
    static thread_local char buf[96];
    const FCfg c = pick_wg(M, N);
    snprintf(buf, sizeof(buf), "k_wgrad_bf16<%d, %d, %d, %d, %s>", c.bm, c.bn, c.wm, c.wn,
             fwg_ct_shape(a, b) ? "true" : "false");
    return buf;
}

int sd_fast_wgrad_splits(long long P, int M, int N) {
    static const int target = [] {  // SD_FWG_BLOCKS: split-K blocks of the ConvTranspose weight gradients (A/B runs)
        const char* e = getenv("SD_FWG_BLOCKS");
        return e && atoi(e) > 0 ? atoi(e) : 512;  // one round at two blocks per CU (measured 9 us faster per layer than 1024)
    }();
    const FCfg c = pick_wg(M, N);
    const long long tiles = (long long)cdiv(M, c.bm) * cdiv(N, c.bn);
    long long splits = (target + tiles - 1) / tiles;
    const long long max_splits = (P + 64 * 8 - 1) / (64 * 8);  // >= 8 K tiles per block
    if (splits > max_splits) splits = max_splits;
    if (splits < 1) splits = 1;
    return (int)splits;
}

// SD_FAST_NBUF=2: the double-buffered 64 x 128 FA tiles (A/B runs)
static int fwd_nbuf() {
    static const int v = [] {
        const char* e = getenv("SD_FAST_NBUF");
        return e && atoi(e) == 2 ? 2 : 1;
    }();
    return v;
}

int sd_fast_conv_gemm(const sd_src& a, int batch, int H, int W, const void* wpack, int N, int kpad, int epi, void* out0,
                      void* out1, int n_split, const float* bias, float* stats, hipStream_t st) {
    const long long M = (long long)batch * H * W;
    FwdArgs p;
    p.a = make_srcf(a);
    p.H = H;
    p.W = W;
    p.M = (int)M;
    p.fW = make_fdiv(W);
    p.fH = make_fdiv(H);
    p.wp = (const __bf16*)wpack;
    p.N = N;
    p.kpad = kpad;
    p.ktiles = cdiv(p.a.kchunks, FKC);
    p.epi = epi;
    p.out0 = (__bf16*)out0;
    p.out1 = (__bf16*)out1;
    p.n_split = n_split;
    p.bias = bias;
    p.stats = stats;
    const bool fa = fa_path(a, M);
    const FCfg c = pick_fwd(M, N, fa && fwd_nbuf() == 1);
    dim3 grid(cdiv(M, c.bm), cdiv(N, c.bn));
    static const bool xcd_env = [] {
        const char* e = getenv("SD_FAST_XCD");
        return !(e && atoi(e) == 0);
    }();
    p.xcd = xcd_env && grid.y > 1 && (grid.x * grid.y) % 8 == 0;
    const int rm = ring_mode(a, M, N, epi);
    if (rm >= 0) {
        static const int ncu = [] {
            int d = 0, n = 0;
            (void)hipGetDevice(&d);
            (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, d);
            return n >= 8 ? n : 8;
        }();
        int lcpt = 0;
        while ((8 << lcpt) < a.chans[0]) ++lcpt;
        const unsigned a_bytes = (unsigned)(M * a.taps * a.chans[0] * 2);
        const dim3 rgrid(ncu & ~7);  // one block per CU (139 KB of LDS), a multiple of the 8 XCDs
        hipLaunchKernelGGL(k_conv_fwd_ring, rgrid, dim3(512), 0, st, p, lcpt, a_bytes);
        return sd_check_launch("sd_conv_gemm(bf16 ring)");
    }
    if (fa) {
        if (c.bn == 32)
            hipLaunchKernelGGL((k_conv_fwd_bf16<256, 32, 4, 1, true>), grid, dim3(256), 0, st, p);
        else if (c.bn == 64)
            hipLaunchKernelGGL((k_conv_fwd_bf16<128, 64, 2, 2, true>), grid, dim3(256), 0, st, p);
        else if (c.bm == 128 && fwd_nbuf() == 1)
            hipLaunchKernelGGL((k_conv_fwd_bf16<128, 128, 2, 2, true, 1>), grid, dim3(256), 0, st, p);
        else if (c.bm == 128)
            hipLaunchKernelGGL((k_conv_fwd_bf16<128, 128, 2, 2, true>), grid, dim3(256), 0, st, p);
        else if (fwd_nbuf() == 1)
            hipLaunchKernelGGL((k_conv_fwd_bf16<64, 128, 2, 2, true, 1>), grid, dim3(256), 0, st, p);
        else
            hipLaunchKernelGGL((k_conv_fwd_bf16<64, 128, 2, 2, true>), grid, dim3(256), 0, st, p);
    } else if (c.bn == 32)
        hipLaunchKernelGGL((k_conv_fwd_bf16<256, 32, 4, 1, false>), grid, dim3(256), 0, st, p);
    else if (c.bn == 64)
        hipLaunchKernelGGL((k_conv_fwd_bf16<128, 64, 2, 2, false>), grid, dim3(256), 0, st, p);
    else if (c.bm == 128)
        hipLaunchKernelGGL((k_conv_fwd_bf16<128, 128, 2, 2, false>), grid, dim3(256), 0, st, p);
    else
        hipLaunchKernelGGL((k_conv_fwd_bf16<64, 128, 2, 2, false>), grid, dim3(256), 0, st, p);
    return sd_check_launch("sd_conv_gemm(bf16 fast)");
}

int sd_fast_wgrad_gemm(const sd_src& a, const sd_src& b, int batch, int H, int W, int M, int N, float* slab,
                       int splits, hipStream_t st) {
    WgfArgs p;
    p.a = make_srcf(a);
    p.b = make_srcf(b);
    p.H = H;
    p.W = W;
    p.P = batch * H * W;
    p.fW = make_fdiv(W);
    p.fH = make_fdiv(H);
    p.M = M;
    p.N = N;
    p.pix_per_split = cdiv(cdiv(p.P, splits), 64) * 64;
    p.slab = slab;
    const FCfg c = pick_wg(M, N);
    dim3 grid(cdiv(M, c.bm), cdiv(N, c.bn), splits);
    static const bool xcd_env = [] {
        const char* e = getenv("SD_FAST_XCD");
        return !(e && atoi(e) == 0);
    }();
    p.xcd = xcd_env && (grid.x * grid.y * grid.z) % 8 == 0;
    // ConvTranspose2d shape: one 1x1 source without a pool, a 4-tap sub-pixel source of one tensor, 32-bit offsets
    const bool ct = fwg_ct_shape(a, b) && a.H == H && a.W == W && (long long)p.P * a.chans[0] < (1LL << 31) &&
                    4LL * p.P * b.chans[0] < (1LL << 31);
    if (ct) {
        if (c.bm == 32)
            hipLaunchKernelGGL((k_wgrad_bf16<32, 128, 1, 4, true>), grid, dim3(256), 0, st, p);
        else if (c.bm == 64)
            hipLaunchKernelGGL((k_wgrad_bf16<64, 128, 2, 2, true>), grid, dim3(256), 0, st, p);
        else
            hipLaunchKernelGGL((k_wgrad_bf16<128, 128, 2, 2, true>), grid, dim3(256), 0, st, p);
    } else if (c.bm == 32)
        hipLaunchKernelGGL((k_wgrad_bf16<32, 128, 1, 4, false>), grid, dim3(256), 0, st, p);
    else if (c.bm == 64)
        hipLaunchKernelGGL((k_wgrad_bf16<64, 128, 2, 2, false>), grid, dim3(256), 0, st, p);
    else
        hipLaunchKernelGGL((k_wgrad_bf16<128, 128, 2, 2, false>), grid, dim3(256), 0, st, p);
    return sd_check_launch("sd_wgrad_gemm(bf16 fast)");
}

extern "C" int sd_bnrelu_pool(int dtype, const void* y, const float* scale, const float* shift, int batch, int H, int W,
                              int C, void* out, sd_stream s) {
    SD_REQUIRE(dtype == SD_BF16, "sd_bnrelu_pool: bf16 only (fp32 mode pools inside the gather)");
    SD_REQUIRE(y && scale && shift && out && batch > 0 && H % 2 == 0 && W % 2 == 0 && C % 8 == 0,
               "sd_bnrelu_pool: bad args");
    long long g = ((long long)batch * (H / 2) * (W / 2) * (C / 8) + 255) / 256;
    if (g > 8192) g = 8192;
    hipLaunchKernelGGL(k_bnrelu_pool_bf16, dim3((int)g), dim3(256), 0, to_stream(s), (const __bf16*)y, scale, shift,
                       batch, H, W, C, (__bf16*)out);
    return sd_check_launch("sd_bnrelu_pool");
}
