// ConvTranspose2d(kernel 2, stride 2, bias) forward (model.py:67-73, used :88-94) as a persistent
// register-streaming GEMM: out[b][2h+dy][2w+dx][o] = bias[o] + sum_ci x[b][h][w][ci] * W[ci][o][dy][dx],
// x = BN+ReLU(y) of the source conv applied on the fly.
//
// GEMM view: C[m][n] = sum_k A[m][k] * Wp[n][k], m = input pixel, n = t*C + o (t = 2*dy + dx),
// k = ci (Wp = sd_pack_convT_w fwd layout). K is small (64..512) and the layer is HBM-bound at the
// full-resolution end (up1: 7.4 MB per pair moved for 0.3 GFLOP), so:
//   * a block keeps its 128-column slice of Wp in LDS for its whole life (persistent over M tiles);
//   * A never touches LDS: each lane loads the 16-B piece of its pixel row that IS its MFMA operand
//     fragment (computing C^T = Wp * A^T with v_mfma_f32_32x32x16_bf16, lane l holds pixel l&31,
//     channels 8*(l>>5)..+7 of the k-step), applies the BN affine + ReLU in registers, and
//     prefetches the next 64-channel chunk while the current one is in the matrix core;
//   * the C^T accumulator puts 4 consecutive output channels of one pixel in each lane, so the
//     pixel-shuffle epilogue is direct 8-B stores (+bias) to the 2x2 output block.
#include "common.h"

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

struct CtArgs {
    const __bf16* x;      // [M][K] NHWC source (the conv output before its BN)
    const float *sc, *sh; // BN affine of the source (nullptr: identity, no ReLU)
    const __bf16* wp;     // [N][kpad]
    const float* bias;    // [C]
    __bf16* out;          // [B][2H][2W][C]
    int M, H, W, K, kpad, N, C;
    int nblk, gper, tiles;
    FastDiv fW, fH, fC;
};

constexpr int CT_NB = 128;   // columns per block (4 n-tiles of 32)
constexpr int CT_MT = 128;   // pixels per tile (32 per wave)
constexpr int CT_KC = 64;    // channels per prefetch chunk (4 k-steps)
constexpr int CT_SLD = CT_NB + 8;  // staging row (136 bf16 = 17 16-B slots)

template <bool BN>
__global__ __launch_bounds__(256, 2) void k_convt_fwd(const CtArgs p) {
    extern __shared__ __attribute__((aligned(16))) __bf16 wl[];  // [CT_NB][K + 8], then 4 staging tiles
    __shared__ float bl[CT_NB];
    __shared__ __attribute__((aligned(16))) float scl[BN ? 256 : 1], shl[BN ? 256 : 1];  // source BN affine (K <= 256)
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int nb = blockIdx.x % p.nblk, slot = blockIdx.x / p.nblk;
    const int n0 = nb * CT_NB;
    const int WLD = p.K + 8;  // odd number of 16-B slots per row: conflict-free fragment reads
    __bf16* stg = wl + CT_NB * WLD + wid * 32 * CT_SLD;  // this wave's epilogue staging tile
    for (int i = tid; i < CT_NB * (p.K / 8); i += 256) {
        const int r = i / (p.K / 8), c8 = i - r * (p.K / 8);
        *reinterpret_cast<uint4*>(wl + r * WLD + c8 * 8) =
            *reinterpret_cast<const uint4*>(p.wp + (size_t)(n0 + r) * p.kpad + c8 * 8);
    }
    if (tid < CT_NB) bl[tid] = p.bias[(n0 + tid) % p.C];
    if constexpr (BN) {
        for (int k = tid; k < p.K; k += 256) {
            scl[k] = p.sc[k];
            shl[k] = p.sh[k];
        }
    }
    __syncthreads();


    const int kchunks = p.K / CT_KC;
    const int my_tiles = slot < p.tiles ? (p.tiles - 1 - slot) / p.gper + 1 : 0;
    const int total = my_tiles * kchunks;
    const int kh = 8 * (lane >> 5);  // this lane's 8 channels within each 16-channel k-step

    // chunk iteration it -> (tile, kc). A ring of 3 register sets keeps the loads of iterations
    // it+1..it+2 in flight while it computes (one iteration of MFMA work is far shorter than the HBM
    // round trip), and unrolling by the ring size keeps every index static (no register copies that
    // would wait on pending loads).
    auto load_chunk = [&](int it, uint4 (&r)[4]) {
        const int ti = it / kchunks, kc = it - ti * kchunks;
        const int m = (slot + ti * p.gper) * CT_MT + wid * 32 + (lane & 31);
        const __bf16* src = p.x + (size_t)(m < p.M ? m : 0) * p.K + kc * CT_KC + kh;
#pragma unroll
        for (int s = 0; s < 4; ++s) r[s] = *reinterpret_cast<const uint4*>(src + s * 16);
    };
    f32x16 acc[4];
    auto compute = [&](int it, const uint4 (&cur)[4]) {
        const int ti = it / kchunks, kc = it - ti * kchunks;
        if (kc == 0) {
#pragma unroll
            for (int t = 0; t < 4; ++t)
#pragma unroll
                for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;
        }
#pragma unroll
        for (int s = 0; s < 4; ++s) {
            const int kb = kc * CT_KC + s * 16, k = kb + kh;
            bf16x8 bfrag;
            if constexpr (BN) {
                // the lane's 8 channels' affine from LDS (staged once per block). Scalar loads of it here
                // put a scalar-cache round trip (lgkmcnt(0)) in front of every k-step, which at one wave
                // per SIMD (K = 256) was most of the kernel's time
                const float4* s4 = reinterpret_cast<const float4*>(scl + k);
                const float4* h4 = reinterpret_cast<const float4*>(shl + k);
                const float4 sa = s4[0], sb = s4[1], ha = h4[0], hb = h4[1];
                const float scv[8] = {sa.x, sa.y, sa.z, sa.w, sb.x, sb.y, sb.z, sb.w};
                const float shv[8] = {ha.x, ha.y, ha.z, ha.w, hb.x, hb.y, hb.z, hb.w};
                const unsigned w[4] = {cur[s].x, cur[s].y, cur[s].z, cur[s].w};
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const float v = j & 1 ? __uint_as_float(w[j >> 1] & 0xffff0000u) : __uint_as_float(w[j >> 1] << 16);
                    bfrag[j] = (__bf16)fmaxf(__builtin_fmaf(v, scv[j], shv[j]), 0.f);
                }
            } else {
                bfrag = *reinterpret_cast<const bf16x8*>(&cur[s]);
            }
#pragma unroll
            for (int t = 0; t < 4; ++t) {
                const bf16x8 afrag = *reinterpret_cast<const bf16x8*>(wl + (t * 32 + (lane & 31)) * WLD + k);
                acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(afrag, bfrag, acc[t], 0, 0, 0);
            }
        }
        if (kc == kchunks - 1) {
            // ------------------------------------------------ pixel-shuffle epilogue of the tile
            // (+bias, bf16) -> this wave's LDS staging tile [32 pixels][128 columns], then 16-B pieces
            // with consecutive lanes on consecutive channels of one output pixel: each store
            // instruction writes whole runs of the 2x2 output blocks instead of 8-B pieces 128 B apart
#pragma unroll
            for (int t = 0; t < 4; ++t)
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    const int nl = t * 32 + 8 * g + 4 * (lane >> 5);  // 4 consecutive columns
                    const float4 bb = *reinterpret_cast<const float4*>(bl + nl);
                    bf16x4 v;
                    v[0] = (__bf16)(acc[t][4 * g + 0] + bb.x);
                    v[1] = (__bf16)(acc[t][4 * g + 1] + bb.y);
                    v[2] = (__bf16)(acc[t][4 * g + 2] + bb.z);
                    v[3] = (__bf16)(acc[t][4 * g + 3] + bb.w);
                    *reinterpret_cast<bf16x4*>(stg + (lane & 31) * CT_SLD + nl) = v;
                }
            __builtin_amdgcn_wave_barrier();  // one wave's LDS ops complete in order
            const int mt = (slot + ti * p.gper) * CT_MT + wid * 32;
#pragma unroll
            for (int i = 0; i < 8; ++i) {
                const int q = lane + 64 * i, pl = q >> 4, n8 = (q & 15) * 8;  // pixel, first column
                const int m = mt + pl;
                const uint4 v = *reinterpret_cast<const uint4*>(stg + pl * CT_SLD + n8);
                if (m < p.M) {
                    const uint32_t bh = fdiv(m, p.fW), b = fdiv(bh, p.fH);
                    const int w = m - bh * p.W, h = bh - b * p.H;
                    const int n = n0 + n8, sub = fdiv(n, p.fC), o = n - sub * p.C;
                    const size_t pix = ((size_t)b * 2 * p.H + 2 * h + (sub >> 1)) * (2 * p.W) + 2 * w + (sub & 1);
                    *reinterpret_cast<uint4*>(p.out + pix * p.C + o) = v;
                }
            }
            __builtin_amdgcn_wave_barrier();  // reads done before the next tile's writes
        }
    };
    constexpr int RING = 3;
    uint4 ring[RING][4];
#pragma unroll
    for (int u = 0; u < RING - 1; ++u)
        if (u < total) load_chunk(u, ring[u]);
    for (int it0 = 0; it0 < total; it0 += RING) {
#pragma unroll
        for (int u = 0; u < RING; ++u) {
            const int it = it0 + u;
            if (it >= total) break;
            if (it + RING - 1 < total) load_chunk(it + RING - 1, ring[(u + RING - 1) % RING]);
            compute(it, ring[u]);
        }
    }
}

}  // namespace

// bf16 ConvTranspose2d forward through k_convt_fwd: one unpooled 1-tap source, K % 64 == 0 and
// K <= 256, N = 4*C with C % 32 == 0 and N % 128 == 0 (up1..up3; up4's K = 512 weight slice would
// hold one block per CU, and the tiled GEMM measured faster there: 79 vs 115 us at B=64)
bool sd_convt_fwd_ok(const sd_src& a, int N, int epi) {
    static const int kmax = [] {  // SD_CONVT_KMAX: largest K for k_convt_fwd (A/B runs)
        const char* e = getenv("SD_CONVT_KMAX");
        return e && atoi(e) > 0 ? atoi(e) : 256;
    }();
    const int K = a.chans[0] + a.chans[1];
    return epi == SD_EPI_PIXSHUF && a.taps == 1 && !a.pool && a.chans[1] == 0 && K % CT_KC == 0 && K <= kmax &&
           N % CT_NB == 0 && (N / 4) % 32 == 0 && (a.xform[0] == SD_IDENT || a.xform[0] == SD_BNRELU);
}

const char* sd_convt_fwd_name(const sd_src& a) {
    return a.xform[0] == SD_BNRELU ? "k_convt_fwd<true>" : "k_convt_fwd<false>";
}

int sd_convt_fwd(const sd_src& a, int batch, int H, int W, const void* wpack, int N, int kpad, const float* bias,
                 void* out, hipStream_t st) {
    CtArgs p;
    p.x = (const __bf16*)a.ptr[0];
    const bool bn = a.xform[0] == SD_BNRELU;
    p.sc = bn ? a.scale[0] : nullptr;
    p.sh = bn ? a.shift[0] : nullptr;
    p.wp = (const __bf16*)wpack;
    p.bias = bias;
    p.out = (__bf16*)out;
    p.M = batch * H * W;
    p.H = H;
    p.W = W;
    p.K = a.chans[0];
    p.kpad = kpad;
    p.N = N;
    p.C = N / 4;
    p.nblk = N / CT_NB;
    p.tiles = (p.M + CT_MT - 1) / CT_MT;
    p.fW = make_fdiv(W);
    p.fH = make_fdiv(H);
    p.fC = make_fdiv(p.C);
    SD_REQUIRE(a.H == H && a.W == W && kpad >= p.K && bias && (!bn || (p.sc && p.sh)), "sd_conv_gemm(convT): bad args");
    const size_t lds = ((size_t)CT_NB * (p.K + 8) + 4 * 32 * CT_SLD) * sizeof(__bf16);
    // blocks per CU: as many as the LDS slice allows, at most 2 (2 waves per SIMD: ~230 VGPRs)
    int per_cu = (int)((160 * 1024) / (lds + CT_NB * sizeof(float) + 2 * 256 * sizeof(float) + 1024));
    if (per_cu > 2) per_cu = 2;
    if (per_cu < 1) per_cu = 1;
    static bool attr_set = false;  // dynamic LDS beyond 64 KB (K = 512: 130 KB)
    if (!attr_set) {
        (void)hipFuncSetAttribute((const void*)k_convt_fwd<true>, hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024);
        (void)hipFuncSetAttribute((const void*)k_convt_fwd<false>, hipFuncAttributeMaxDynamicSharedMemorySize, 150 * 1024);
        attr_set = true;
    }
    int gper = 256 * per_cu / p.nblk;
    if (gper < 1) gper = 1;
    if (gper > p.tiles) gper = p.tiles;
    p.gper = gper;
    const dim3 grid(p.gper * p.nblk);
    if (bn)
        hipLaunchKernelGGL(k_convt_fwd<true>, grid, dim3(256), lds, st, p);
    else
        hipLaunchKernelGGL(k_convt_fwd<false>, grid, dim3(256), lds, st, p);
    return sd_check_launch("sd_conv_gemm(convT)");
}
