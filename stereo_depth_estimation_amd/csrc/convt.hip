// ConvTranspose2d(kernel 2, stride 2, bias) forward and data gradient (model.py:67-73, used :88-94) as a
// persistent register-streaming GEMM whose weight slice stays in LDS.
//
// forward : out[b][2h+dy][2w+dx][o] = bias[o] + sum_ci x[b][h][w][ci] * W[ci][o][dy][dx],
//           x = BN+ReLU(y) of the source conv applied on the fly.
//           GEMM view C[m][n] = sum_k A[m][k] * Wp[n][k], m = input pixel, n = t*C + o (t = 2*dy + dx),
//           k = ci (Wp = sd_pack_convT_w fwd layout); pixel-shuffle epilogue.
// dgrad   : dx[b][h][w][ci] = sum_{t, o} du[b][2h+t/2][2w+t%2][o] * W[ci][o][t]
//           GEMM view with m = input pixel, n = ci, k = t*Cs + o (Wp = sd_pack_convT_w dgrad layout): each A
//           row is the 2x2 sub-pixel block of du, gathered as 4 contiguous Cs-channel runs; plain NHWC store.
//           DGRAD_BNS: dx is the upstream gradient da of the source conv's BatchNorm (model.py:40), and the
//           epilogue also sums its BatchNorm backward (sum dz, sum dz*xhat per channel, what sd_bn_bwd_reduce
//           computes in a pass of its own) into one partials row per block slot.
//
// K is small (64..1024) and the full-resolution layers are HBM-bound (up1: 7.4 MB per pair for 0.3 GFLOP), so
//   * a block keeps its NB-column slice of Wp in LDS for its whole life (persistent over 128-pixel M tiles);
//   * A never touches LDS: each lane loads the 16-B piece of its pixel row that IS its MFMA operand fragment
//     (computing C^T = Wp * A^T with v_mfma_f32_32x32x16_bf16, lane l holds pixel l&31, channels 8*(l>>5)..+7
//     of the k-step), applies the BN affine + ReLU in registers (forward), and keeps RING-1 64-channel chunks
//     in flight while the current one is in the matrix core;
//   * the C^T accumulator puts 4 consecutive output channels of one pixel in each lane; the epilogue stages the
//     wave's 32-pixel tile in LDS and leaves as 16-B pieces, consecutive lanes on consecutive channels.
#include "common.h"

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

enum { CT_FWD = 0, CT_FWD_BN = 1, CT_DGRAD = 2, CT_DGRAD_BNS = 3 };

struct CtArgs {
    const __bf16* x;      // forward: [M][K] NHWC source (the conv output before its BN); dgrad: du [B][2H][2W][Cs]
    const float *sc, *sh; // forward BN affine of the source
    const __bf16* wp;     // [N][kpad]
    const float* bias;    // forward: [C]
    __bf16* out;          // forward: [B][2H][2W][C]; dgrad: [M][N]
    int M, H, W, K, kpad, N, C;
    int cs_log2;          // dgrad: log2(Cs), K = 4*Cs
    int nblk, gper, tiles;
    FastDiv fW, fH, fC;
    // DGRAD_BNS: the BatchNorm layer whose da is `out` (raw output by [M][N]); partials [gper][N] float2
    const __bf16* by;
    const float *bsc, *bsh, *bmu, *bis;
    float2* part;
};

constexpr int CT_MT = 128;   // pixels per tile (32 per wave)
constexpr int CT_KC = 64;    // channels per prefetch chunk (4 k-steps)
constexpr int CT_KMAX_BN = 512;  // forward BN affine staged in LDS

template <int MODE, int NB, int RING>
__global__ __launch_bounds__(256, RING > 3 ? 1 : 2) void k_convt(const CtArgs p) {
    constexpr bool FWD = MODE == CT_FWD || MODE == CT_FWD_BN, BN = MODE == CT_FWD_BN, BNS = MODE == CT_DGRAD_BNS;
    constexpr int NT = NB / 32;        // 32-column n-tiles per wave
    constexpr int SLD = NB + 8;        // staging row (odd number of 16-B slots)
    constexpr int PPX = NB / 8;        // 16-B pieces per staged pixel row
    constexpr int EI = 32 * PPX / 64;  // epilogue store instructions per wave and tile
    extern __shared__ __attribute__((aligned(16))) __bf16 wl[];  // [NB][K + 8], then 4 staging tiles
    __shared__ float bl[FWD ? NB : 1];
    __shared__ __attribute__((aligned(16))) float scl[BN ? CT_KMAX_BN : 1], shl[BN ? CT_KMAX_BN : 1];
    __shared__ float red[BNS ? 4 * NB * 2 : 1];
    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    const int nb = blockIdx.x % p.nblk, slot = blockIdx.x / p.nblk;
    const int n0 = nb * NB;
    const int WLD = p.K + 8;  // odd number of 16-B slots per row: conflict-free fragment reads
    __bf16* stg = wl + NB * WLD + wid * 32 * SLD;  // this wave's epilogue staging tile
    {
        // the slice is up to 128 KB: WU unconditional 16-B loads per thread in flight before their LDS stores (a
        // load-store loop made one dependent global round trip per 4 KB, ~70 us for the K = 1024 slice)
        constexpr int WU = 16;
        const int pieces = NB * (p.K / 8);
        for (int base = 0; base < pieces; base += 256 * WU) {
            uint4 v[WU];
#pragma unroll
            for (int u = 0; u < WU; ++u) {
                const int i = min(base + tid + 256 * u, pieces - 1);
                const int r = i / (p.K / 8), c8 = i - r * (p.K / 8);
                v[u] = *reinterpret_cast<const uint4*>(p.wp + (size_t)(n0 + r) * p.kpad + c8 * 8);
            }
#pragma unroll
            for (int u = 0; u < WU; ++u) {
                const int i = base + tid + 256 * u;
                const int r = i / (p.K / 8), c8 = i - r * (p.K / 8);
                if (i < pieces) *reinterpret_cast<uint4*>(wl + r * WLD + c8 * 8) = v[u];
            }
        }
    }
    if constexpr (FWD) {
        if (tid < NB) bl[tid] = p.bias[(n0 + tid) % p.C];
    }
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

    // BNS: the 8 channels this lane stores (fixed: piece lane % PPX of every staged row) and their BatchNorm
    // constants; the y pieces of a tile's stores travel in the register ring with the tile's last chunk
    constexpr int NBK = BNS ? 8 : 1, YI = BNS ? EI : 1;
    float bk_sc[NBK], bk_sh[NBK], bk_mu[NBK], bk_is[NBK], own[BNS ? 16 : 1];
    if constexpr (BNS) {
        const int c = n0 + (lane % PPX) * 8;
#pragma unroll
        for (int q = 0; q < 8; ++q) {
            bk_sc[q] = p.bsc[c + q];
            bk_sh[q] = p.bsh[c + q];
            bk_mu[q] = p.bmu[c + q];
            bk_is[q] = p.bis[c + q];
        }
#pragma unroll
        for (int j = 0; j < 16; ++j) own[j] = 0.f;
    }

    // chunk iteration it -> (tile, kc). A ring of RING register sets keeps the loads of iterations
    // it+1..it+RING-1 in flight while it computes (one iteration of MFMA work is far shorter than the HBM
    // round trip), and unrolling by the ring size keeps every index static (no register copies that
    // would wait on pending loads). Every iteration issues the same buffer loads (past the block's last chunk,
    // past M, or a y piece of a chunk that is not its tile's last: out of range = zeros, no traffic): a load on
    // only some paths makes hipcc's vmcnt bookkeeping merge to the smallest count, and the ring then had less
    // than one chunk in flight (vmcnt(3) at RING = 3), one memory round trip per chunk.
    constexpr unsigned OOB = 0x80000000u;
    const __amdgpu_buffer_rsrc_t xrs =
        __builtin_amdgcn_make_buffer_rsrc((void*)p.x, (short)0, p.M * p.K * 2, 0x00020000);
    const __amdgpu_buffer_rsrc_t yrs =
        __builtin_amdgcn_make_buffer_rsrc((void*)(BNS ? p.by : p.x), (short)0, BNS ? p.M * p.N * 2 : 0, 0x00020000);
    auto load_chunk = [&](int it, uint4 (&r)[4], uint4 (&yr)[YI]) __attribute__((always_inline)) {
        const int ti = it / kchunks, kc = it - ti * kchunks;
        const int mt = (slot + ti * p.gper) * CT_MT + wid * 32;
        const int m0 = mt + (lane & 31);
        const bool live = (it < total) & (m0 < p.M);
        const uint32_t m = live ? m0 : 0;
        if constexpr (FWD) {
            const unsigned off = live ? (unsigned)(m * p.K + kc * CT_KC + kh) * 2u : OOB;
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                const auto v = __builtin_amdgcn_raw_buffer_load_b128(xrs, off, s * 32, 0);
                r[s] = make_uint4(v[0], v[1], v[2], v[3]);
            }
        } else {
            // sub-pixel gather: k = t*Cs + o, t = 2*dy + dx of the 2x2 block of du above input pixel m
            const uint32_t bh = fdiv(m, p.fW), b = fdiv(bh, p.fH);
            const int w = m - bh * p.W, h = bh - b * p.H;
            const unsigned W2 = 2 * p.W;
            const unsigned pb = ((b * 2 * p.H + 2 * h) * W2 + 2 * w);  // du pixel of t = 0
            const int cmask = (1 << p.cs_log2) - 1;
#pragma unroll
            for (int s = 0; s < 4; ++s) {
                const int k = kc * CT_KC + s * 16;  // wave-uniform
                const int t = k >> p.cs_log2, o = (k & cmask) + kh;
                const unsigned px = pb + (t >> 1) * W2 + (t & 1);
                const unsigned off = live ? ((px << p.cs_log2) + o) * 2u : OOB;
                const auto v = __builtin_amdgcn_raw_buffer_load_b128(xrs, off, 0, 0);
                r[s] = make_uint4(v[0], v[1], v[2], v[3]);
            }
        }
        if constexpr (BNS) {
            const bool last = (it < total) & (kc == kchunks - 1);
#pragma unroll
            for (int i = 0; i < EI; ++i) {
                const int q = lane + 64 * i, pl = q / PPX, n8 = (q % PPX) * 8;
                const unsigned off = (last & (mt + pl < p.M)) ? (unsigned)((mt + pl) * p.N + n0 + n8) * 2u : OOB;
                const auto v = __builtin_amdgcn_raw_buffer_load_b128(yrs, off, 0, 0);
                yr[i] = make_uint4(v[0], v[1], v[2], v[3]);
            }
        }
    };
    f32x16 acc[NT];
    auto compute = [&](int it, const uint4 (&cur)[4], const uint4 (&yq)[YI]) __attribute__((always_inline)) {
        const int ti = it / kchunks, kc = it - ti * kchunks;
        if (kc == 0) {
#pragma unroll
            for (int t = 0; t < NT; ++t)
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
            for (int t = 0; t < NT; ++t) {
                const bf16x8 afrag = *reinterpret_cast<const bf16x8*>(wl + (t * 32 + (lane & 31)) * WLD + k);
                acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(afrag, bfrag, acc[t], 0, 0, 0);
            }
        }
        if (kc == kchunks - 1) {
            // ------------------------------------------------ epilogue of the tile
            // (+bias, bf16) -> this wave's LDS staging tile [32 pixels][NB columns], then 16-B pieces with
            // consecutive lanes on consecutive channels of one output pixel
#pragma unroll
            for (int t = 0; t < NT; ++t)
#pragma unroll
                for (int g = 0; g < 4; ++g) {
                    const int nl = t * 32 + 8 * g + 4 * (lane >> 5);  // 4 consecutive columns
                    float4 bb = make_float4(0.f, 0.f, 0.f, 0.f);
                    if constexpr (FWD) bb = *reinterpret_cast<const float4*>(bl + nl);
                    bf16x4 v;
                    v[0] = (__bf16)(acc[t][4 * g + 0] + bb.x);
                    v[1] = (__bf16)(acc[t][4 * g + 1] + bb.y);
                    v[2] = (__bf16)(acc[t][4 * g + 2] + bb.z);
                    v[3] = (__bf16)(acc[t][4 * g + 3] + bb.w);
                    *reinterpret_cast<bf16x4*>(stg + (lane & 31) * SLD + nl) = v;
                }
            __builtin_amdgcn_wave_barrier();  // one wave's LDS ops complete in order
            const int mt = (slot + ti * p.gper) * CT_MT + wid * 32;
#pragma unroll
            for (int i = 0; i < EI; ++i) {
                const int q = lane + 64 * i, pl = q / PPX, n8 = (q % PPX) * 8;  // pixel, first column
                const int m = mt + pl;
                const uint4 v = *reinterpret_cast<const uint4*>(stg + pl * SLD + n8);
                if constexpr (FWD) {
                    if (m < p.M) {
                        const uint32_t bh = fdiv(m, p.fW), b = fdiv(bh, p.fH);
                        const int w = m - bh * p.W, h = bh - b * p.H;
                        const int n = n0 + n8, sub = fdiv(n, p.fC), o = n - sub * p.C;
                        const size_t pix = ((size_t)b * 2 * p.H + 2 * h + (sub >> 1)) * (2 * p.W) + 2 * w + (sub & 1);
                        store16_nt(p.out + pix * p.C + o, v);
                    }
                } else {
                    if (m < p.M) store16_nt(p.out + (size_t)m * p.N + n0 + n8, v);
                    if constexpr (BNS) {
                        // the stored (bf16) da: dz = da where y*scale+shift > 0, xhat = (y-mean)*invstd
                        const bool live = m < p.M;
                        const unsigned dw[4] = {v.x, v.y, v.z, v.w}, yw[4] = {yq[i].x, yq[i].y, yq[i].z, yq[i].w};
#pragma unroll
                        for (int c = 0; c < 8; ++c) {
                            const float d = __uint_as_float(c & 1 ? dw[c >> 1] & 0xffff0000u : dw[c >> 1] << 16);
                            const float yy = __uint_as_float(c & 1 ? yw[c >> 1] & 0xffff0000u : yw[c >> 1] << 16);
                            const float z = __builtin_fmaf(yy, bk_sc[c], bk_sh[c]);
                            const float dz = (live & (z > 0.f)) ? d : 0.f;
                            own[2 * c] += dz;
                            own[2 * c + 1] = __builtin_fmaf(dz, (yy - bk_mu[c]) * bk_is[c], own[2 * c + 1]);
                        }
                    }
                }
            }
            __builtin_amdgcn_wave_barrier();  // reads done before the next tile's writes
        }
    };
    uint4 ring[RING][4], yring[RING][YI];
#pragma unroll
    for (int u = 0; u < RING - 1; ++u) load_chunk(u, ring[u], yring[u]);
    const int padded = (total + RING - 1) / RING * RING;
    for (int it0 = 0; it0 < padded; it0 += RING) {
#pragma unroll
        for (int u = 0; u < RING; ++u) {
            const int it = it0 + u;
            load_chunk(it + RING - 1, ring[(u + RING - 1) % RING], yring[(u + RING - 1) % RING]);
            if (it < total) compute(it, ring[u], yring[u]);
        }
    }

    if constexpr (BNS) {
        // lanes l, l + PPX, l + 2*PPX, ... hold the same 8 channels: one partials row per block slot
#pragma unroll
        for (int k = 0; k < 16; ++k)
#pragma unroll
            for (int o = PPX; o < 64; o <<= 1) own[k] += __shfl_xor(own[k], o);
        if (lane < PPX) {
#pragma unroll
            for (int c = 0; c < 8; ++c) {
                red[(wid * NB + lane * 8 + c) * 2] = own[2 * c];
                red[(wid * NB + lane * 8 + c) * 2 + 1] = own[2 * c + 1];
            }
        }
        __syncthreads();
        if (tid < NB) {
            float s = 0.f, ss = 0.f;
#pragma unroll
            for (int w = 0; w < 4; ++w) {
                s += red[(w * NB + tid) * 2];
                ss += red[(w * NB + tid) * 2 + 1];
            }
            p.part[(size_t)slot * p.N + n0 + tid] = make_float2(s, ss);
        }
    }
}

int env_int(const char* name, int dflt) {
    const char* e = getenv(name);
    return e && *e ? atoi(e) : dflt;
}

// SD_CONVT_RING: register-ring depth (A/B runs): 3 (two chunks in flight, two blocks per CU where the LDS
// allows) or 6 (five in flight, one block per CU)
int ring_depth() {
    static const int r = env_int("SD_CONVT_RING", 3) >= 6 ? 6 : 3;
    return r;
}

size_t ct_lds(int NB, int K) { return ((size_t)NB * (K + 8) + 4 * 32 * (NB + 8)) * sizeof(__bf16); }
constexpr size_t CT_LDS_MAX = 160 * 1024 - 8 * 1024;  // dynamic part (the static arrays take < 8 KB)

// the column-slice width for a shape: 128 where the slice and staging fit, else 64 (always 64 with the BNS
// epilogue: its y ring and BatchNorm constants spill at 128)
int pick_nb(int N, int K, bool bns = false) {
    if (!bns && N % 128 == 0 && ct_lds(128, K) <= CT_LDS_MAX) return 128;
    if (N % 64 == 0 && ct_lds(64, K) <= CT_LDS_MAX) return 64;
    return 0;
}

template <int MODE, int NB, int RING>
int launch_ct(CtArgs& p, size_t lds, hipStream_t st) {
    static bool attr_set = false;  // dynamic LDS beyond 64 KB
    if (!attr_set) {
        (void)hipFuncSetAttribute((const void*)k_convt<MODE, NB, RING>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)CT_LDS_MAX);
        attr_set = true;
    }
    // blocks per CU: as many as the LDS slice allows, at most 2 (RING 3: ~230 VGPRs) or 1 (RING 6)
    int per_cu = (int)((160 * 1024) / (lds + 8 * 1024));
    if (per_cu > (RING > 3 ? 1 : 2)) per_cu = RING > 3 ? 1 : 2;
    if (per_cu < 1) per_cu = 1;
    int gper = 256 * per_cu / p.nblk;
    if (gper < 1) gper = 1;
    if (gper > p.tiles) gper = p.tiles;
    p.gper = gper;
    hipLaunchKernelGGL((k_convt<MODE, NB, RING>), dim3(p.gper * p.nblk), dim3(256), lds, st, p);
    return SD_OK;
}

template <int MODE>
int launch_mode(CtArgs& p, int NB, hipStream_t st) {
    const size_t lds = ct_lds(NB, p.K);
    p.nblk = p.N / NB;
    if constexpr (MODE == CT_DGRAD_BNS) {  // NB = 64 only (pick_nb)
        return ring_depth() == 6 ? launch_ct<MODE, 64, 6>(p, lds, st) : launch_ct<MODE, 64, 3>(p, lds, st);
    } else {
        if (ring_depth() == 6)
            return NB == 128 ? launch_ct<MODE, 128, 6>(p, lds, st) : launch_ct<MODE, 64, 6>(p, lds, st);
        return NB == 128 ? launch_ct<MODE, 128, 3>(p, lds, st) : launch_ct<MODE, 64, 3>(p, lds, st);
    }
}

// The gper (= BNS partials rows) launch_ct would choose, without launching
int ct_gper(int nblk, int NB, int K, long long M) {
    const size_t lds = ct_lds(NB, K);
    const int cap = ring_depth() > 3 ? 1 : 2;
    int per_cu = (int)((160 * 1024) / (lds + 8 * 1024));
    if (per_cu > cap) per_cu = cap;
    if (per_cu < 1) per_cu = 1;
    int gper = 256 * per_cu / nblk;
    if (gper < 1) gper = 1;
    const int tiles = (int)((M + CT_MT - 1) / CT_MT);
    return gper > tiles ? tiles : gper;
}

}  // namespace

// bf16 ConvTranspose2d forward through k_convt: one unpooled 1-tap source, K % 64 == 0, N = 4*C with C % 32 == 0 and
// N % 64 == 0, and K <= 128, or K <= SD_CONVT_KMAX (default 256, read per call) at M >= 16384 GEMM rows. up4's
// K = 512 slice holds one block per CU, and the tiled GEMM measured faster there (79 vs 115 us at B=64). up3 (K = 256):
// at B = 64 (M = 76800) k_convt and the tiled GEMM's 128 x 128 tiles measured even over the step (per layer 64 vs 55
// us, bench 7708 vs 7681 mean of three, gpurun_out/g14ab-g16ab); at the live app's B = 1 (M = 10800) the tiled GEMM
// took the fp8 forward 0.587-0.593 -> 0.579 ms (gpurun_out/g15)
bool sd_convt_fwd_ok(const sd_src& a, long long M, int N, int epi) {
    const int kmax = env_int("SD_CONVT_KMAX", 256);
    const int K = a.chans[0] + a.chans[1];
    return epi == SD_EPI_PIXSHUF && a.taps == 1 && !a.pool && a.chans[1] == 0 && K % CT_KC == 0 &&
           (K <= 128 || (K <= kmax && M >= 16384)) &&
           K <= CT_KMAX_BN && (N / 4) % 32 == 0 && pick_nb(N, K) != 0 &&
           (a.xform[0] == SD_IDENT || a.xform[0] == SD_BNRELU);
}

const char* sd_convt_fwd_name(const sd_src& a, int N) {
    static thread_local char buf[64];
    const int K = a.chans[0] + a.chans[1];
    snprintf(buf, sizeof(buf), "k_convt<%d, %d, %d>", a.xform[0] == SD_BNRELU ? CT_FWD_BN : CT_FWD, pick_nb(N, K),
             ring_depth());
    return buf;
}

int sd_convt_fwd(const sd_src& a, int batch, int H, int W, const void* wpack, int N, int kpad, const float* bias,
                 void* out, hipStream_t st) {
    CtArgs p{};
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
    p.tiles = (p.M + CT_MT - 1) / CT_MT;
    p.fW = make_fdiv(W);
    p.fH = make_fdiv(H);
    p.fC = make_fdiv(p.C);
    SD_REQUIRE(a.H == H && a.W == W && kpad >= p.K && bias && (!bn || (p.sc && p.sh)), "sd_conv_gemm(convT): bad args");
    const int NB = pick_nb(N, p.K);
    if (bn)
        launch_mode<CT_FWD_BN>(p, NB, st);
    else
        launch_mode<CT_FWD>(p, NB, st);
    return sd_check_launch("sd_conv_gemm(convT)");
}

// ConvTranspose2d data gradient through k_convt: a 4-tap sub-pixel source of one unpooled raw (identity) tensor
// with Cs a power of two >= 16, K = 4*Cs % 64 == 0, N % 64 == 0 and the weight slice in LDS. SD_CONVT_DG: bit
// mask over Cs = 32, 64, 128, 256 (bits 0..3; up1..up4) of the layers routed here (A/B runs). Default up1 + up2,
// measured at B=64 with the fused BatchNorm-backward sums (gpurun_out/ct3): up1 163 -> 114 us (dgrad + the reduce
// pass it replaces), up2 96 -> 82 us; up3 71 -> 82 and up4 63 -> 83 us lose. Every A load instruction of this
// kernel touches 32 cache lines (lane = pixel), so at small M the address path, not the matrix core, paces it
bool sd_convt_dgrad_ok(const sd_src& a, int N, int epi) {
    static const int mask = env_int("SD_CONVT_DG", 3);
    const int Cs = a.chans[0];
    if (epi != SD_EPI_STORE || a.taps != 4 || a.pool || a.chans[1] != 0 || a.xform[0] != SD_IDENT) return false;
    if (Cs < 16 || (Cs & (Cs - 1)) != 0 || (4 * Cs) % CT_KC != 0 || pick_nb(N, 4 * Cs) == 0) return false;
    const int bit = Cs == 32 ? 1 : Cs == 64 ? 2 : Cs == 128 ? 4 : Cs == 256 ? 8 : 0;
    return (mask & bit) != 0;
}

const char* sd_convt_dgrad_name(const sd_src& a, int N, bool bns) {
    static thread_local char buf[64];
    snprintf(buf, sizeof(buf), "k_convt<%d, %d, %d>", bns ? CT_DGRAD_BNS : CT_DGRAD, pick_nb(N, 4 * a.chans[0], bns),
             ring_depth());
    return buf;
}

int sd_convt_dgrad_rows(const sd_src& a, int batch, int H, int W, int N) {
    const int NB = pick_nb(N, 4 * a.chans[0], true);
    return NB ? ct_gper(N / NB, NB, 4 * a.chans[0], (long long)batch * H * W) : 0;
}

int sd_convt_dgrad(const sd_src& a, int batch, int H, int W, const void* wpack, int N, int kpad, void* out,
                   const HaloBnSum* bns, float* partials, hipStream_t st) {
    CtArgs p{};
    p.x = (const __bf16*)a.ptr[0];
    p.wp = (const __bf16*)wpack;
    p.out = (__bf16*)out;
    p.M = batch * H * W;
    p.H = H;
    p.W = W;
    const int Cs = a.chans[0];
    p.K = 4 * Cs;
    int lg = 0;
    while ((1 << lg) < Cs) ++lg;
    p.cs_log2 = lg;
    p.kpad = kpad;
    p.N = N;
    p.C = N;
    p.tiles = (p.M + CT_MT - 1) / CT_MT;
    p.fW = make_fdiv(W);
    p.fH = make_fdiv(H);
    p.fC = make_fdiv(N);
    SD_REQUIRE(a.H == 2 * H && a.W == 2 * W && kpad >= p.K, "sd_conv_gemm(convT dgrad): bad args");
    const int NB = pick_nb(N, p.K, bns != nullptr);
    if (bns) {
        SD_REQUIRE(bns->y && bns->scale && bns->shift && bns->mean && bns->invstd && partials,
                   "sd_conv_gemm_bnsum(convT dgrad): bad args");
        p.by = (const __bf16*)bns->y;
        p.bsc = bns->scale;
        p.bsh = bns->shift;
        p.bmu = bns->mean;
        p.bis = bns->invstd;
        p.part = reinterpret_cast<float2*>(partials);
        launch_mode<CT_DGRAD_BNS>(p, NB, st);
    } else {
        launch_mode<CT_DGRAD>(p, NB, st);
    }
    return sd_check_launch("sd_conv_gemm(convT dgrad)");
}
