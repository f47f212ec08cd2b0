// Halo-tiled bf16 kernels for the 3x3 convolutions (model.py:36,39): forward and dgrad of every
// conv with N = 32 or N % 64 == 0, and weight gradients with M = 32 or M % 64 == 0.
// Replaces mkldnn_convolution / convolution_backward for those layers.
//
// Instead of re-gathering each of the 9 taps from L2 (implicit GEMM), a block stages the
// (th+2) x (tw+2) pixel input halo of its th x tw output tile in LDS once per 32-channel chunk
// and reads all 9 taps from it:
//   forward/dgrad : C[pixel][co] = sum_{tap, ci} halo[pixel+tap][ci] * W[co][tap][ci]
//                   (v_mfma_f32_32x32x16_bf16; halo pixel stride 80 B = 5 16-B slots, odd, so
//                   every ds_read_b128 lane group of an A fragment is conflict-free at any tap offset)
//   wgrad         : dW[co][tap][ci] += sum_{pixel} dy[pixel][co] * halo[pixel+tap][ci]
//                   (v_mfma_f32_16x16x32_bf16 with ds_read_b64_tr_b16 transposed reads; each dy
//                   fragment is reused by all 9 taps; blocks loop over a range of tiles = split-K)
// Tile shapes are runtime (8x32 at 240x320, 6x40 at 60x80, a whole 15x20 image ...): pixels of a
// tile are flattened into 32-pixel MFMA rows / k-steps and each lane carries its pixel's halo offset.
#include "common.h"
#include "halo_util.h"

namespace {

constexpr int CK = 32;                           // channels per chunk
#ifndef WG_EXP
#define WG_EXP 0  // timing experiments only. wgrad<64>: bit 0 no MFMA phase, 1 no tile loads after the first,
                  // 2 no LDS stores; halo conv: bit 3 no MFMA phase, 5 no halo LDS stores, 12 no epilogue stores
                  // stores; k_halo_wgrad_ws: bit 6 no MFMA phase, 7 no LDS stores, 8 no loads and no stores;
                  // BNB: bit 19 no dy transform, 20 no dy global stores, 21 no y loads
#endif
typedef float f32x16 __attribute__((ext_vector_type(16)));

struct HaloSrc {
    const __bf16* p0;
    const __bf16* p1;
    const float *sc0, *sh0, *sc1, *sh1;
    int c0, c1, x0, x1;
    int ctot;
};
static inline HaloSrc make_halo_src(const sd_src& s) {
    HaloSrc h;
    h.p0 = (const __bf16*)s.ptr[0];
    h.p1 = (const __bf16*)s.ptr[1];
    h.sc0 = s.scale[0];
    h.sh0 = s.shift[0];
    h.sc1 = s.scale[1];
    h.sh1 = s.shift[1];
    h.c0 = s.chans[0];
    h.c1 = s.chans[1];
    h.x0 = s.xform[0];
    h.x1 = s.xform[1];
    h.ctot = s.chans[0] + s.chans[1];
    return h;
}

__device__ __forceinline__ uint4 bnrelu8(uint4 raw, const float* sc, const float* sh) {
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

// The 8-channel piece a thread stages is at a fixed channel offset for a whole chunk
// ((tid & 3) * 8), so source selection and the BN affine are per thread and per chunk.
// Loads are branch-free: invalid pieces (outside the image / past the channels) read the source
// base and are zeroed after the transform (the conv's zero padding applies after the activation).
struct HaloCol {
    const __bf16* base;
    int C, c;  // channel stride, local channel offset
    bool cok, bn;
    float4 s0, s1, h0, h1;
};
__device__ __forceinline__ HaloCol halo_col(const HaloSrc& s, int cglob, const void* dummy) {
    HaloCol r;
    r.cok = cglob < s.ctot;
    // channel padding past ctot reads (and discards) source 0: source 1 may be NULL
    const bool first = cglob < s.c0 || !r.cok;
    r.c = first ? cglob : cglob - s.c0;
    if (!r.cok) r.c = 0;
    r.base = first ? s.p0 : s.p1;
    r.C = first ? s.c0 : s.c1;
    r.bn = r.cok && (first ? s.x0 : s.x1) == SD_BNRELU;
    const float* sc = r.bn ? (first ? s.sc0 : s.sc1) + r.c : (const float*)dummy;
    const float* sh = r.bn ? (first ? s.sh0 : s.sh1) + r.c : (const float*)dummy;
    r.s0 = *reinterpret_cast<const float4*>(sc);
    r.s1 = *reinterpret_cast<const float4*>(sc + 4);
    r.h0 = *reinterpret_cast<const float4*>(sh);
    r.h1 = *reinterpret_cast<const float4*>(sh + 4);
    return r;
}
__device__ __forceinline__ uint4 halo_load(const HaloCol& hc, bool ok, int b, int H, int W, int h, int w) {
    const size_t off = ok ? ((size_t)((size_t)b * H + h) * W + w) * hc.C + hc.c : 0;
    return *reinterpret_cast<const uint4*>(hc.base + off);
}
__device__ __forceinline__ uint4 halo_finish(const HaloCol& hc, bool ok, uint4 raw) {
    uint4 v = raw;
    if (hc.bn) {
        const unsigned w[4] = {raw.x, raw.y, raw.z, raw.w};
        const float s[8] = {hc.s0.x, hc.s0.y, hc.s0.z, hc.s0.w, hc.s1.x, hc.s1.y, hc.s1.z, hc.s1.w};
        const float h[8] = {hc.h0.x, hc.h0.y, hc.h0.z, hc.h0.w, hc.h1.x, hc.h1.y, hc.h1.z, hc.h1.w};
        bf16x8 o;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            o[2 * i] = (__bf16)fmaxf(__builtin_fmaf(__uint_as_float(w[i] << 16), s[2 * i], h[2 * i]), 0.f);
            o[2 * i + 1] =
                (__bf16)fmaxf(__builtin_fmaf(__uint_as_float(w[i] & 0xffff0000u), s[2 * i + 1], h[2 * i + 1]), 0.f);
        }
        v = *reinterpret_cast<uint4*>(&o);
    }
    return ok ? v : make_uint4(0, 0, 0, 0);
}

// halo_finish with the ReLU taken on the rounded bf16 pair (v_pk_max_i16 against 0: a bf16 is <= 0 exactly
// when its sign bit is set or it is zero, and rounding preserves the sign), one instruction per pair
// instead of two v_max_f32. Same values as halo_finish for every finite input.
__device__ __forceinline__ uint4 halo_finish_pk(const HaloCol& hc, bool ok, uint4 raw) {
    uint4 v = raw;
    if (hc.bn) {
        const unsigned w[4] = {raw.x, raw.y, raw.z, raw.w};
        const float s[8] = {hc.s0.x, hc.s0.y, hc.s0.z, hc.s0.w, hc.s1.x, hc.s1.y, hc.s1.z, hc.s1.w};
        const float h[8] = {hc.h0.x, hc.h0.y, hc.h0.z, hc.h0.w, hc.h1.x, hc.h1.y, hc.h1.z, hc.h1.w};
        unsigned o[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const float lo = __builtin_fmaf(__uint_as_float(w[i] << 16), s[2 * i], h[2 * i]);
            const float hi = __builtin_fmaf(__uint_as_float(w[i] & 0xffff0000u), s[2 * i + 1], h[2 * i + 1]);
            // one v_cvt_pk_bf16_f32 per pair (the compiler's per-element conversion took two plus a v_perm), and
            // the operands are opaque to the SLP vectorizer, which otherwise pairs the FMAs into v_pk_fma_f32
            // (~22 extra cycles each on a SIMD that is issuing MFMAs, MI355X_MICROARCH.md)
            asm("v_cvt_pk_bf16_f32 %0, %1, %2\n\tv_pk_max_i16 %0, %0, 0" : "=v"(o[i]) : "v"(lo), "v"(hi));
        }
        v = make_uint4(o[0], o[1], o[2], o[3]);
    }
    return ok ? v : make_uint4(0, 0, 0, 0);
}


// Partner value for the BN-statistics reduce-scatter level o (16, 8, 4, 2, 1) within each 32-lane
// half: lanes l and partner(l) differ in bit o and agree above it, which is all the reduce-scatter
// needs. The partners are chosen to be cheap: lane ^ 16 by ds_swizzle (bit-mask mode, no address
// register), then DPP row_mirror (l ^ 15), row_half_mirror (l ^ 7) and quad perms (l ^ 2, l ^ 1):
// VALU moves instead of five rounds of ds_bpermute through the LDS pipe.
__device__ __forceinline__ float rs_partner(float v, int o) {
    const int x = __float_as_int(v);
    int r;
    switch (o) {
        case 16: r = __builtin_amdgcn_ds_swizzle(x, 0x401F); break;             // and 0x1F, xor 0x10
        case 8: r = __builtin_amdgcn_update_dpp(0, x, 0x140, 0xF, 0xF, false); break;  // row_mirror
        case 4: r = __builtin_amdgcn_update_dpp(0, x, 0x141, 0xF, 0xF, false); break;  // row_half_mirror
        case 2: r = __builtin_amdgcn_update_dpp(0, x, 0x4E, 0xF, 0xF, false); break;   // quad_perm [2,3,0,1]
        default: r = __builtin_amdgcn_update_dpp(0, x, 0xB1, 0xF, 0xF, false); break;  // quad_perm [1,0,3,2]
    }
    return __int_as_float(r);
}

// =====================================================================================
// forward / dgrad: any 3x3 conv with N = 32 or a multiple of 64 (N-blocks of 32*NT channels)
// =====================================================================================
// One 512-thread block per CU, persistent over work items (spatial tiles of one N-block):
//   waves 4-7 (loaders): global -> registers -> BN+ReLU -> LDS, into the buffer the MFMA waves
//                        are NOT reading (LDS double buffer), one CK-channel chunk ahead;
//   waves 0-3 (MFMA)   : C^T[co][pixel] += W[co][tap,ci] * halo[pixel+tap][ci] on the other buffer,
//                        then the epilogue straight from registers.
// So the LDS staging and the BN transform overlap the matrix core instead of alternating with it.
// Each MFMA wave owns RT 32-pixel column tiles x NT 32-channel row tiles, so a block item is a
// th x tw output tile of up to 128*RT pixels (runtime shape, flattened; each lane carries its
// pixel's halo offset and adds the tap offset kh*(tw+2)+kw).
// LDS budget per chunk and what bounds it: every k-step a wave reads RT+NT 1-KiB fragments for
// RT*NT MFMAs, and the loaders write the chunk's halo and NT*32 weight rows. A CK = 16 variant
// (RT = 4, 512-pixel tiles, weights re-staged per 512 pixels instead of 256) models ~60 % LDS
// busy instead of ~85 %, but measured slower than CK = 32 at every layer: it is kept behind
// SD_HALO_CK=16 and the default for N % 64 is CK = 32 with RT = 2..3.
// Computing the transposed product puts 4 consecutive output channels of one pixel in each lane
// (C layout of 32x32x16: col = lane&31 = pixel, rows (r&3) + 8*(r>>2) + 4*(lane>>5) = channels):
// the epilogue pairs lanes l / l+32 (v_permlane32_swap) and stores 16-B pieces directly, and BN
// statistics (taken before the swap) accumulate per lane across all of a
// block's items and are reduced across lanes once, into ONE stats row per block.
struct HFwdArgs {
    HaloSrc a;
    int H, W;             // image (GEMM grid)
    int th, tw, tiles_x;  // spatial tile and tiling
    int tiles, nsp;       // tiles per image, batch * tiles
    int nblk, gper;       // N-blocks, blocks per N-block (= stats rows)
    int hw, nhalo;        // halo width (tw+2) and pixel count ((th+2)*(tw+2))
    const __bf16* wp;     // packed [co][kpad], k = tap*ctot + c (wsplit: k = tap*2*ctot + {hi c | ctot + lo c})
    int N, kpad;
    int wsplit;           // 1: hi/lo bf16 weight pairs (SD_PACK_CONV3_FWD_SPLIT): each item's chunks run twice
    const float* osc;     // OAFF: the stored value is bf16(acc * osc[n] + osh[n]) (eval BN applied before rounding)
    const float* osh;
    int epi;
    __bf16* out0;
    __bf16* out1;
    int n_split;
    float* stats;         // [gper][N] float2 (sum, sumsq of the stored bf16 values)
    int xcd;              // 1: XCD-contiguous block numbering (grid % 8 == 0)
    int prio;             // s_setprio 1 for the MFMA waves (1) or the loader waves (2), 0: none
    unsigned long long* dbg;  // timing-diagnostic builds only (WG_EXP & 1024): per-wave cycle counters
    // BNS (sd_conv_gemm_bnsum): the stored output is the upstream gradient da of a BatchNorm layer whose raw
    // output is by; the stats rows get (sum dz, sum dz*xhat) of it, dz = da where by*scale+shift > 0,
    // xhat = (by-mean)*invstd (what sd_bn_bwd_reduce computes in a pass of its own)
    const __bf16* by;
    const float *bsc, *bsh, *bmu, *bis;
    // split-K (eval STORE launches whose items leave most CUs idle: the batch-1 forwards of the deep layers): ksplit
    // groups of gblk = gper * nblk blocks, group ks runs chunks [ks*cps, ks*cps + cps) of every item (wsplit: of the
    // 2 x ncp hi/lo chunks) and stores its raw fp32 sums to part[ks][pixel][N]; k_halo_split_reduce adds the groups'
    // partials, applies the output affine (OAFF) and stores bf16. ksplit = 1: part is null, the epilogue stores out0.
    int ksplit, gblk, cps;
    int npix;  // batch * H * W (partials rows per group)
    float* part;
};

// Cache policy of the conv epilogue stores: nontemporal (2). The outputs (0.1-0.3 GB per launch) are read by the next
// layer's kernel, never again by this one, and allocating them in the XCD's 4 MB L2 evicts the weight rows and halo
// rows the loaders re-read: A/B over the model's 14 layer shapes (tools/conv_micro.py, same box, two rounds) 1894 ->
// 1831 us (-3.3 %). Moving the item epilogue to the loader waves instead (they idle 20-60 % at the barrier) was
// measured too: +1.8 %, the epilogue then delays the next chunk's staging by as much as it saved the MFMA waves.
#ifndef HC_ST_AUX
#define HC_ST_AUX 2
#endif
// weight images by LDS-DMA in the multi-chunk M16 conv instances (k_halo_conv loaders); HC_WDMA=0 builds: register-staged
#ifndef HC_WDMA
#define HC_WDMA 1
#endif
// the vertical-reuse k-loop of the N = 32 RT = 4 conv instances (k_halo_conv); HC_VR=0 builds: the per-tap loop
#ifndef HC_VR
#define HC_VR 1
#endif
// BN statistics of one stored 16-B piece (8 bf16 channels; a pixel outside the tile adds zeros): channel pair q's
// (sum, sum) in own[4q + {0,1}] and (sumsq, sumsq) in own[4q + {2,3}], so each pair is one v_pk_add_f32 and one
// v_pk_fma_f32
__device__ __forceinline__ void stats_add(float* own, const uint4 v, const bool live) {
    const unsigned wv[4] = {live ? v.x : 0u, live ? v.y : 0u, live ? v.z : 0u, live ? v.w : 0u};
#pragma unroll
    for (int q = 0; q < 4; ++q) {
        const f32x2 x = {__uint_as_float(wv[q] << 16), __uint_as_float(wv[q] & 0xffff0000u)};
        f32x2 sm = {own[4 * q], own[4 * q + 1]}, sq = {own[4 * q + 2], own[4 * q + 3]};
        sm += x;
        sq = __builtin_elementwise_fma(x, x, sq);
        own[4 * q] = sm.x;
        own[4 * q + 1] = sm.y;
        own[4 * q + 2] = sq.x;
        own[4 * q + 3] = sq.y;
    }
}
template <bool B> struct BoolC { static constexpr bool v = B; };  // a compile-time flag passed to a generic lambda
constexpr int PERSIST_BLOCKS = 256;                 // one block per CU on MI355X
constexpr int SBN_MAX = 1024;                       // input channels of the forward/dgrad kernel (LDS BN affine)
constexpr int HMAX = 384;                           // wgrad halo pixels (>= 17 x 22 for a whole 15x20 image)
// halo pixels per LDS buffer: 384 (RT 2, and RT 3 at CK 32: 17 x 22 for a whole 15x20 image), 512, 640
__host__ __device__ constexpr int halo_px_cap(int RT, int CK) { return RT == 4 ? 640 : (RT == 3 && CK == 16 ? 512 : 384); }
// CK = 8 (the 8-channel network input, enc1.0): one 16-B slot per halo pixel (consecutive pixels are
// consecutive slots), 176-B weight rows
__host__ __device__ constexpr int halo_ld(int CK) { return CK == 8 ? 8 : CK + 8; }       // 48 / 80 B: odd # of 16-B slots
__host__ __device__ constexpr int wrow_ld(int CK) { return CK == 8 ? 88 : 9 * CK + 8; }  // 304 / 592 B: odd # of 16-B slots
// M16 weight rows: piece p of a tap stored at p ^ wswz(row) (see k_halo_conv)
__device__ __forceinline__ int wswz(int row) { return ((row >> 2) & 1) * 2; }

// Loader piece `item` -> (halo pixel, 16-B piece within the pixel). ds_write_b128 is banked per 8-lane
// group over 8 slots ((a/4) mod 32): 8 lanes on 8 consecutive pixels at one piece land on 8 distinct
// slots at the odd pixel stride (5 or 3 slots); pixel-major order (2 pixels x 4 pieces per group) put
// slots 5p and 5p+8 on one bank in every group. The piece is fixed per thread (item = ltid + 256*i).
template <int PPX>
__device__ __forceinline__ int ld_pixel(int item) { return (item / (8 * PPX)) * 8 + (item & 7); }
template <int PPX>
__device__ __forceinline__ int ld_piece(int item) { return (item >> 3) % PPX; }

// IT items (spatial tiles of the same N-block) per pass: every chunk's weights are staged once for IT halos and
// the MFMA waves keep IT accumulator sets (IT = 2 with CK = 16 halves the weight staging per MFMA)
// OAFF (eval forwards, sd_conv3x3_ex): the epilogue applies the layer's eval-mode BatchNorm affine before the bf16
// rounding, so the stored tensor is z = scale*y + shift and its consumers apply only the ReLU. Rounding z instead of y
// keeps bf16's relative precision on the normalised activation: where a channel's |mean| / std is large (enc1.0: ~4.6
// on a trained checkpoint) the rounding of y, magnified by scale, was the largest activation error of the bf16 path
// (tools/precision_study.py: per-batch EPE noise 1.5e-3 -> 5.4e-4 px, as much as fp32 storage would give).
// (Weights in registers for the N % 64 layers, each MFMA wave owning 16 output channels over a whole 256-pixel tile
// with its A fragments read from L2 one chunk ahead, was built in r04 and measured 5-28 % slower than these LDS-weight
// instances at every N % 64 shape: DESIGN.md §3 r04. Removed in r05.)
template <int NT, int RT, int CK, bool STATS, bool WCONST, int IT, bool BNS, bool OAFF, bool RAW>
__device__ __forceinline__ void halo_conv_body(const HFwdArgs& p) {
    static_assert(!(OAFF && (STATS || BNS)), "the affine epilogue stores eval-mode outputs (no statistics)");
    constexpr int BN = 32 * NT;
    constexpr int PPX = CK / 8;                          // 16-B pieces per pixel (and per tap of a weight row)
    // M16 (every CK = 32 instance but the BNS dgrads): v_mfma_f32_16x16x32_bf16, one k-step per tap. Same LDS bytes and
    // MFMA cycles per FLOP as 32x32x16 at the same wave tile, but the chip holds a higher clock under it
    // (MI355X_MICROARCH.md, DVFS give-back item 7: 1.12-1.14x the FLOP/s with operands from LDS; measured here 3-6 %
    // per layer). Its fragments are 16 rows x 4 pieces, so the halo is stored piece-major ([piece][pixel], 16 B per
    // pixel: the 16 consecutive pixels of one ds_read_b128 lane group hit 16 distinct bank slots) and the weight rows
    // (36 slots, unpadded) swap their pieces by row, piece ^ wswz(row): rows r (piece p) and r' (piece p + 1) of one lane
    // group land on 16 distinct slots (the 4-row classes r mod 16 in {0-3, 12-15} / {4-11} map to slot residues
    // {0,2} / {1,3} mod 4).
    // Not the BNS dgrads: their y prefetch and BatchNorm-backward constants beside the 16x16 fragment ring spill at
    // RT 4 (461 vs 236 us per launch); they are HBM-bound full-resolution layers, where the shape buys nothing.
    // (Tried: 512-pixel items, NT = 2 x RT = 4 at 12x32 / 10x40 tiles with a 512-pixel halo, to halve the weight
    // staging per MFMA: 10-30 % slower per layer. Those tiles hold 384-400 pixels, so a quarter of the MFMA columns
    // idle, and the 128 accumulators leave no room for a fragment ring.)
    // (Also with the vertical-reuse k-loop's smaller fragment ring, 48 VGPRs instead of 80, the N = 32 RT = 4 BNS dgrad
    // spills 75-122 VGPRs in this form: its y pieces, BatchNorm constants and sums sit beside the accumulators.)
    constexpr bool M16 = CK == 32 && IT == 1 && !BNS;
    constexpr int HX_LD = halo_ld(CK), W_LD = M16 ? 9 * CK : wrow_ld(CK);
    // IT = 2: the CK = 32 tilings (halo <= 384 px)
    constexpr int HPX = IT == 2 ? 384 : halo_px_cap(RT, CK);
    constexpr int HP = (HPX * PPX + 255) / 256;          // halo pieces per loader thread
    constexpr int WPIECES = BN * 9 * PPX;                // weight pieces per chunk
    constexpr int W_PER_THREAD = (WPIECES + 255) / 256;
    static_assert(!M16 || (HP * 256 == HPX * PPX && HPX % 16 == 0), "M16: the loader pieces tile the halo exactly");
    constexpr int HALO_ITEM = M16 ? HPX * CK : HP * 256 / PPX * HX_LD;  // one item's halo region
    constexpr int HALO_ELEMS = IT * HALO_ITEM, W_ELEMS = BN * W_LD, BUF = HALO_ELEMS + W_ELEMS;
    static_assert(IT == 1 || (IT == 2 && HP * IT <= 16), "item masks fit 16 bits");
    constexpr int KS = (9 * CK + 15) / 16;               // 16-deep k-steps per chunk (CK 8: 5, the last half padding)
    __shared__ __attribute__((aligned(16))) __bf16 smem[2 * BUF];
    // epilogue transpose scratch: 32 (M16: 16) pixels x BN channels per MFMA wave (its own region, no block sync)
    constexpr int SCR_PX = M16 ? 16 : 32;
    __shared__ __attribute__((aligned(16))) __bf16 scr[4 * SCR_PX * BN];

    // waves 0-3 land on the 4 different SIMDs (dispatch order 0->2->1->3, measured), and so do 4-7:
    // one MFMA wave and one loader wave per SIMD
    const int tid = threadIdx.x, lane = tid & 63;
    const bool is_loader = (tid >> 6) >= 4;
    const int wid = (tid >> 6) & 3;  // role-local wave index
    // Workgroups are dealt round-robin to the 8 XCDs (workgroup i -> XCD i % 8), each with its own L2.
    // Renumbered so that each XCD owns a contiguous range of block ids, the tiles a wave of items covers
    // on one XCD are neighbours (shared halo rows, and the N-blocks of one tile) and meet in that L2.
    const int bid = p.xcd ? (blockIdx.x & 7) * (gridDim.x >> 3) + (blockIdx.x >> 3) : blockIdx.x;
    const int ks = bid / p.gblk, bb = bid - ks * p.gblk;  // split-K group, block within the group
    const int nb = bb % p.nblk, slot = bb / p.nblk;
    const int n0 = nb * BN;
    // chunks never straddle the two sources (a source's last chunk may be partial): every chunk has one
    // source, one channel stride and one BN affine
    const int nc0 = (p.a.c0 + CK - 1) / CK;
    const int ncp = nc0 + (p.a.c1 + CK - 1) / CK;  // chunks of the input channels
    // wsplit: an item runs its ncp chunks twice, against the hi then the lo bf16 halves of fp32 weights (w = hi + lo
    // to ~2^-17 relative), so the sum over both passes is the product with the fp32 weights: the full-resolution
    // layers' weight rounding is what moved the bf16 path's EPE (tools/precision_study.py). The MFMA waves see
    // 2 x ncp chunks per item; only the loaders know which pass a chunk belongs to.
    const int nch_v = p.wsplit ? 2 * ncp : ncp;
    const int c_lo = ks * p.cps;  // split-K: this group's chunks [c_lo, c_lo + nchunks)
    const int nchunks = (c_lo + p.cps < nch_v ? c_lo + p.cps : nch_v) - c_lo;
    const int wct = p.wsplit ? 2 * p.a.ctot : p.a.ctot;  // packed weight channels per tap
    const int mvalid = p.th * p.tw;
    const int my_items = slot < p.nsp ? (p.nsp - 1 - slot) / p.gper + 1 : 0;
    const int total = (my_items + IT - 1) / IT * nchunks;  // chunk iterations (block-uniform), IT items each
#ifndef HC_LS_N32
#define HC_LS_N32 2
#endif
    // loader register sets (chunks in flight); HC_LS_N32: for the 32-channel-chunk N = 32 instances (A/B builds)
    constexpr int LS = NT == 1 && CK == 8 ? 4 : (NT == 1 && CK == 32 ? HC_LS_N32 : 2);
    const int padded = (total + LS - 1) / LS * LS;   // loader iterations

    // the BN affine of every input channel (identity for raw sources), read by the loaders per chunk from LDS
    __shared__ __attribute__((aligned(16))) float sbn[2 * SBN_MAX + 2 * CK];  // + the tail of a partial chunk
    __shared__ __attribute__((aligned(16))) float oaff[OAFF ? 2 * BN : 4];      // OAFF: [scale | shift] of this N-block
    // The tables are filled by both roles, each before the launch's first barrier; the loaders issue their first
    // chunks' loads before their share (VMEM loads complete in order, so one memory latency covers the tables, the
    // weights and the first halos instead of one each: the serial latencies are what a batch-1 launch costs)
    auto fill_tables = [&]() __attribute__((always_inline)) {
        if constexpr (OAFF) {
            for (int c = tid; c < 2 * BN; c += 512) {
                const int ch = n0 + (c < BN ? c : c - BN);
                oaff[c] = ch < p.N ? (c < BN ? p.osc : p.osh)[ch] : 0.f;
            }
        }
        for (int c = tid; c < p.a.ctot; c += 512) {
            const bool first = c < p.a.c0;
            const int cl = first ? c : c - p.a.c0;
            const bool bn = (first ? p.a.x0 : p.a.x1) == SD_BNRELU;
            sbn[c] = bn ? (first ? p.a.sc0 : p.a.sc1)[cl] : 1.f;
            sbn[SBN_MAX + c] = bn ? (first ? p.a.sh0 : p.a.sh1)[cl] : 0.f;
        }
    };
    float* const redf = sbn;  // [4][BN][2] BN statistics after the last item (the loaders no longer read sbn)
    static_assert(4 * BN * 2 <= 2 * SBN_MAX, "redf fits in sbn");

    // p.prio: 1 = MFMA waves, 2 = loader waves at s_setprio 1 for the whole launch. The loader waves are the younger
    // half of the workgroup and lose issue arbitration to the MFMA waves on every SIMD they share; when they also run
    // the BN+ReLU transform the MFMA waves then wait for them at the chunk barriers (diagnostic build, 30x40 512->256:
    // 23 % of MFMA-wave cycles). Loader priority: 30x40 forwards 9 % faster, 60x80 5 %; dgrads (raw dy) lose 1-3 %.
    if (p.prio != 0 && (__builtin_amdgcn_readfirstlane(threadIdx.x) >= 256) == (p.prio == 2))
        __builtin_amdgcn_s_setprio(1);
    if (is_loader) {
        // =========================================================== loader waves
        // Per-chunk work is kept to the loads and LDS stores themselves (the loader VALU count per chunk, not
        // the memory system, bounded the deep layers: ~450 VALU per chunk with per-piece 64-bit address math
        // and zero-selects). Offsets are 32-bit and precomputed: weights once per block (a chunk adds a scalar
        // soffset), halo pixels once per item; loads are buffer loads whose out-of-range offset (OOB) returns
        // zeros without memory traffic, so invalid pieces need no select unless the BN transform follows.
        const int ltid = wid * 64 + lane;
        constexpr unsigned OOB = 0x80000000u;
        const int hw_img = p.H * p.W;
        const int lpiece = ld_piece<PPX>(ltid);  // this thread's 8-channel piece of every halo pixel
        unsigned pgeo[HP];                       // (halo row << 16 | halo col) of each piece, ~0 past the halo
#pragma unroll
        for (int i = 0; i < HP; ++i) {
            const int px = ld_pixel<PPX>(ltid + i * 256);
            const int hy = px / p.hw;
            pgeo[i] = px < p.nhalo ? ((unsigned)hy << 16) | (unsigned)(px - hy * p.hw) : 0xffffffffu;
        }
        int hpx[IT][HP];  // image-local pixel of each piece for the items of pass ld_pass, -1 outside the image
        const __bf16* ib0[IT];  // the items' images in source 0 / source 1
        const __bf16* ib1[IT];
        int ld_pass = 0, ld_cc = 0;
        auto geometry = [&]() __attribute__((always_inline)) {
#pragma unroll
            for (int u = 0; u < IT; ++u) {
                // past the block's last item (unconditional loads): every piece out of range, no traffic
                const int itm = ld_pass * IT + u;
                const bool live = itm < my_items;
                const int sp = slot + (live ? itm : 0) * p.gper;
                const int b = sp / p.tiles, tl = sp - b * p.tiles;
                const int ty = tl / p.tiles_x;
                const int h0 = ty * p.th - 1, w0 = (tl - ty * p.tiles_x) * p.tw - 1;
                ib0[u] = p.a.p0 + (size_t)b * hw_img * p.a.c0;
                ib1[u] = p.a.c1 ? p.a.p1 + (size_t)b * hw_img * p.a.c1 : p.a.p0;
#pragma unroll
                for (int i = 0; i < HP; ++i) {
                    const int h = h0 + (int)(pgeo[i] >> 16), w = w0 + (int)(pgeo[i] & 0xffffu);
                    const bool in = live & (pgeo[i] != 0xffffffffu) & (h >= 0) & (w >= 0) & (h < p.H) & (w < p.W);
                    hpx[u][i] = in ? h * p.W + w : -1;
                }
            }
        };
        // weights: byte offset of each piece in chunk 0 (OOB: past the weight rows of this N-block)
        const __amdgpu_buffer_rsrc_t wrs =
            __builtin_amdgcn_make_buffer_rsrc((void*)p.wp, (short)0, p.N * p.kpad * 2, 0x00020000);
        constexpr bool WDMA = HC_WDMA && M16 && IT == 1 && (!WCONST || RAW);  // weights by LDS-DMA (below)
        unsigned woff[W_PER_THREAD];
#pragma unroll
        for (int i = 0; i < W_PER_THREAD; ++i) {
            const int item = ltid + i * 256;
            const int co = item / (9 * PPX), r = item - co * (9 * PPX), tap = r / PPX, sp = r - tap * PPX;
            woff[i] = ((item < WPIECES) & (n0 + co < p.N)) ? (unsigned)((n0 + co) * p.kpad + tap * wct + sp * 8) * 2u
                                                          : OOB;
            if constexpr (!WDMA) asm volatile("" : "+v"(woff[i]));  // kept in registers, not recomputed per chunk
        }
        // WDMA (the multi-chunk M16 instances): the chunk's weight image goes global -> LDS by LDS-DMA
        // (buffer_load_dwordx4 ... lds: no VGPR destination, no ds_write). The M16 weight image is BN unpadded rows of
        // 36 16-B slots, contiguous, so wave-instruction k of a chunk fills LDS slots 64k .. 64k + 63 (M0 + 16 * lane)
        // and each lane's SOURCE address carries the row's piece swap: slot s = 36 co + rs holds piece rs ^ wswz(co).
        // The DMA of chunk g is issued in loader iteration g after the halo stores, into buffer g & 1 (free since the
        // barrier that ended iteration g - 1), and waited for by a counted vmcnt (the halo loads issued after it may
        // stay in flight) before the iteration's barrier. hipcc does not see the asm loads, so its own counted waits
        // only grow stricter: each one also covers a DMA that the previous iteration's vmcnt already retired.
        // This replaces 9 buffer_load_dwordx4 + 9 ds_write_b128 per loader thread and chunk: the VGPR -> LDS transfer
        // of the stores (13 cycles each) was what the loader waves waited on (SQ_WAIT_INST_LDS).
        constexpr int NWI = WPIECES / 64;                   // wave-instructions per chunk
        constexpr int WDI = WDMA ? (NWI + 3) / 4 : 1;       // per loader wave
        static_assert(!WDMA || (WPIECES % 64 == 0 && (HALO_ELEMS * 2) % 16 == 0 && (BUF * 2) % 16 == 0), "WDMA image");
        const int wid_u = __builtin_amdgcn_readfirstlane(wid);
        unsigned wdoff[WDI];
        if constexpr (WDMA) {
#pragma unroll
            for (int j = 0; j < WDI; ++j) {
                const int k = wid_u * WDI + j, s = k * 64 + lane;
                const int co = s / (9 * PPX), rs = s - co * (9 * PPX), r = rs ^ wswz(co);
                const int tap = r / PPX, sp = r - tap * PPX;
                wdoff[j] = (k < NWI && n0 + co < p.N) ? (unsigned)((n0 + co) * p.kpad + tap * wct + sp * 8) * 2u : OOB;
                asm volatile("" : "+v"(wdoff[j]));
            }
        }
        const unsigned lds_w0 = (unsigned)(uintptr_t)(smem + HALO_ELEMS) + (unsigned)(wid_u * WDI) * 1024u;
        // Software pipeline, one iteration per chunk g: store chunk g (set g % LS, loaded LS iterations ago) and
        // the weights of chunk g (loaded one iteration ago) into LDS buffer g & 1, load the weights of chunk g+1
        // and the halo of chunk g+LS, barrier; the MFMA waves compute chunk g-1 meanwhile. Every iteration
        // issues the same loads and waits on every path (chunks past the block's last are out of range, no
        // traffic): a load or a wait on only some paths, or a prologue whose loads differ from an iteration's,
        // makes the compiler's vmcnt bookkeeping merge pessimistically; it then drained every outstanding load
        // before the next loads and left one chunk of latency cover instead of LS. VMEM loads complete in
        // order, so waiting for the weights of chunk g also waits for everything issued before them: they are
        // issued after the halo of chunk g+LS-1 and before that of chunk g+LS.
        // LS register sets: up to LS chunks' halo loads are in flight while the MFMA waves compute another
        // (the 8-channel input, one chunk per item, no weight loads in the loop: LS = 4).
        static_assert(LS == 2 || LS == 4, "set (g % LS) and buffer (g & 1) static per unrolled iteration");
        // one object per set (an array of sets past ~256 B stays in scratch instead of registers)
        struct HSet {
            uint4 hr[IT][HP];
            unsigned m;  // bit u*HP + i: piece i of item u inside the image (and the channels)
            int cb;      // the chunk's first channel (BN affine index)
            bool bn;     // BN+ReLU source
        };
        HSet st0, st1, st2, st3;
        auto set_of = [&](auto S) __attribute__((always_inline)) -> HSet& {
            if constexpr (decltype(S)::value == 0) return st0;
            else if constexpr (decltype(S)::value == 1) return st1;
            else if constexpr (decltype(S)::value == 2) return st2;
            else return st3;
        };
        uint4 wr[W_PER_THREAD];
        // WCONST (one or two chunks per item): the weights of chunk c are the same for every item of this block
        // (fixed N-block), and with at most two chunks chunk c of every item lands in LDS buffer c (g & 1 == g % 2):
        // they are loaded once and stored into the two buffers in the prologue (one chunk: into both). Two-chunk
        // layers (64 input channels: enc2.1, dec2.1, enc3.0, dec1.0, ...) re-staged 36-72 KB of weights per item
        int w_cc = 0;  // chunk (within the item) of the next weights to load
        auto load_w_into = [&](uint4 (&wdst)[W_PER_THREAD]) __attribute__((always_inline)) {  // chunk w_cc, advance
            const int wv = c_lo + w_cc;
            const bool lo = wv >= ncp;  // wsplit: the second pass reads the lo halves
            const int wc = lo ? wv - ncp : wv;
            const bool s1 = wc >= nc0;
            const int C = s1 ? p.a.c1 : p.a.c0;
            const int cl = (s1 ? wc - nc0 : wc) * CK;
            if (++w_cc == nchunks) w_cc = 0;
            unsigned v[W_PER_THREAD];
#pragma unroll
            for (int i = 0; i < W_PER_THREAD; ++i) v[i] = woff[i];
            if (cl + CK > C) {  // partial chunk: pieces past the source's channels read zeros
#pragma unroll
                for (int i = 0; i < W_PER_THREAD; ++i) {
                    const int sp = ((ltid + i * 256) % (9 * PPX)) % PPX;
                    if (cl + sp * 8 >= C) v[i] = OOB;
                }
            }
            // first channel of the chunk in the packed k = tap*wct + c (+ ctot for the lo halves)
            const int cbg = (s1 ? p.a.c0 : 0) + cl + (lo ? p.a.ctot : 0);
#pragma unroll
            for (int i = 0; i < W_PER_THREAD; ++i) {
                const auto x = __builtin_amdgcn_raw_buffer_load_b128(wrs, v[i], cbg * 2, 0);
                wdst[i] = make_uint4(x[0], x[1], x[2], x[3]);
            }
        };
        auto load_w = [&]() __attribute__((always_inline)) { load_w_into(wr); };
        // WDMA: chunk w_cc's weight image -> LDS buffer buf (this wave's WDI KiB of it), advance. No per-piece masks of
        // a partial chunk: its pieces past the source's channels read other (finite) weights of the layer, which meet
        // the zero halo pieces of those channels.
        auto dma_w = [&](int buf) __attribute__((always_inline)) {
            const int wv = c_lo + w_cc;
            const bool lo = wv >= ncp;
            const int wc = lo ? wv - ncp : wv;
            const bool s1 = wc >= nc0;
            const int cl = (s1 ? wc - nc0 : wc) * CK;
            if (++w_cc == nchunks) w_cc = 0;
            const unsigned soff = __builtin_amdgcn_readfirstlane(((s1 ? p.a.c0 : 0) + cl + (lo ? p.a.ctot : 0)) * 2);
            const unsigned m0b = __builtin_amdgcn_readfirstlane(lds_w0 + (unsigned)(buf * BUF * 2));
#pragma unroll
            for (int j = 0; j < WDI; ++j) {
                if (NWI % 4 != 0 && wid_u * WDI + j >= NWI) break;  // wave-uniform
                unsigned keep;
                asm volatile(
                    "s_mov_b32 %0, m0\n\t"
                    "s_mov_b32 m0, %2\n\t"
                    "s_nop 0\n\t"
                    "buffer_load_dwordx4 %1, %3, %4 offen lds\n\t"
                    "s_mov_b32 m0, %0"
                    : "=&s"(keep)
                    : "v"(wdoff[j]), "s"(m0b + (unsigned)j * 1024u), "s"(wrs), "s"(soff)
                    : "memory");
            }
        };
        if constexpr (RAW) {
            // ------------------------------------------------- RAW: every source is a raw tensor (the dgrads, the
            // pooled encoder inputs): the halo goes global -> LDS by LDS-DMA as well, so these loader waves issue
            // nothing but LDS-DMA (no VGPR loads, no ds_write, no VALU on the data). The M16 halo is piece-major,
            // [4 pieces][HPX pixels] of 16 B: loader wave w fills piece w, one wave-instruction per 64 consecutive
            // halo pixels (lane l: pixel 64 i + l), each lane's source the pixel's 16-B piece in the image (out of the
            // image or past the source's channels: out of range, zeros written, no traffic). Chunk g's halo and
            // weights are issued at the start of iteration g into buffer g & 1 and waited for (vmcnt(0)) before the
            // iteration's barrier.
            static_assert(M16 && PPX == 4 && HPX % 64 == 0 && WDMA, "RAW: the M16 piece-major halo, weights by DMA");
            constexpr int HI = HPX / 64;  // halo wave-instructions per loader wave and chunk
            unsigned hg[HI];              // (halo row << 16 | halo col) of this lane's pixels, ~0 past the halo
#pragma unroll
            for (int i = 0; i < HI; ++i) {
                const int px = i * 64 + lane;
                const int hy = px / p.hw;
                hg[i] = px < p.nhalo ? ((unsigned)hy << 16) | (unsigned)(px - hy * p.hw) : 0xffffffffu;
            }
            int hp[HI];  // image-local pixel of each, -1 outside the image
            const __bf16 *rb0 = p.a.p0, *rb1 = p.a.p0;
            int r_pass = 0, r_cc = 0;
            auto rgeo = [&]() __attribute__((always_inline)) {
                const bool live = r_pass < my_items;
                const int sp = slot + (live ? r_pass : 0) * p.gper;
                const int b = sp / p.tiles, tl = sp - b * p.tiles;
                const int ty = tl / p.tiles_x;
                const int h0 = ty * p.th - 1, w0 = (tl - ty * p.tiles_x) * p.tw - 1;
                rb0 = p.a.p0 + (size_t)b * hw_img * p.a.c0;
                rb1 = p.a.c1 ? p.a.p1 + (size_t)b * hw_img * p.a.c1 : p.a.p0;
#pragma unroll
                for (int i = 0; i < HI; ++i) {
                    const int h = h0 + (int)(hg[i] >> 16), w = w0 + (int)(hg[i] & 0xffffu);
                    const bool in = live & (hg[i] != 0xffffffffu) & (h >= 0) & (w >= 0) & (h < p.H) & (w < p.W);
                    hp[i] = in ? h * p.W + w : -1;
                }
            };
            rgeo();
            const unsigned lds_h0 = (unsigned)(uintptr_t)smem + (unsigned)(wid_u * HPX * 16);
            fill_tables();
            __syncthreads();  // the tables (the MFMA waves meet it before their first chunk)
            if constexpr (WCONST) {  // chunk c of every item in buffer c (one chunk: in both)
                dma_w(0);
                dma_w(1);
            }
            for (int g = 0; g < padded; ++g) {
                if (g < total) {
                    const int hv = c_lo + r_cc;
                    const int hc = hv >= ncp ? hv - ncp : hv;  // wsplit: the second pass re-reads the same halo
                    const bool s1 = hc >= nc0;
                    const int C = s1 ? p.a.c1 : p.a.c0;
                    const int cl = (s1 ? hc - nc0 : hc) * CK;
                    const __amdgpu_buffer_rsrc_t hrs =
                        __builtin_amdgcn_make_buffer_rsrc((void*)(s1 ? rb1 : rb0), (short)0, hw_img * C * 2, 0x00020000);
                    const bool cok = cl + wid_u * 8 < C;
                    const unsigned soff = __builtin_amdgcn_readfirstlane(cl * 2);
                    const unsigned m0b = __builtin_amdgcn_readfirstlane(lds_h0 + (unsigned)((g & 1) * BUF * 2));
#pragma unroll
                    for (int i = 0; i < HI; ++i) {
                        const unsigned off = (cok & (hp[i] >= 0)) ? (unsigned)(hp[i] * C + wid_u * 8) * 2u : OOB;
                        unsigned keep;
                        asm volatile(
                            "s_mov_b32 %0, m0\n\t"
                            "s_mov_b32 m0, %2\n\t"
                            "s_nop 0\n\t"
                            "buffer_load_dwordx4 %1, %3, %4 offen lds\n\t"
                            "s_mov_b32 m0, %0"
                            : "=&s"(keep)
                            : "v"(off), "s"(m0b + (unsigned)i * 1024u), "s"(hrs), "s"(soff)
                            : "memory");
                    }
                    if constexpr (!WCONST) dma_w(g & 1);
                    if (++r_cc == nchunks) {
                        r_cc = 0;
                        ++r_pass;
                        rgeo();
                    }
                }
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __syncthreads();
            }
            __syncthreads();  // stats reduction barrier (MFMA waves)
            return;
        }
        auto store_w_from = [&](int buf, const uint4 (&wsrc)[W_PER_THREAD]) __attribute__((always_inline)) {
            __bf16* wl = smem + buf * BUF + HALO_ELEMS;
#pragma unroll
            for (int i = 0; i < W_PER_THREAD; ++i) {
                const int item = ltid + i * 256;
                const int co = item / (9 * PPX), r = item - co * (9 * PPX);
                const int rs = M16 ? r ^ wswz(co) : r;  // M16: pieces swapped by row (conflict-free 16x16 reads)
                if (item < WPIECES) *reinterpret_cast<uint4*>(wl + co * W_LD + rs * 8) = wsrc[i];
            }
        };
        auto store_w = [&](int buf) __attribute__((always_inline)) { store_w_from(buf, wr); };
        auto load = [&](auto S) __attribute__((always_inline)) {  // halo of chunk (ld_item, ld_cc) -> register set S, then advance
            HSet& q = set_of(S);
            const int hv = c_lo + ld_cc;
            const int hc = hv >= ncp ? hv - ncp : hv;  // wsplit: the second pass re-reads the same halo
            const bool s1 = hc >= nc0;
            const int C = s1 ? p.a.c1 : p.a.c0;
            const int cl = (s1 ? hc - nc0 : hc) * CK;
            q.cb = (s1 ? p.a.c0 : 0) + cl;
            q.bn = (s1 ? p.a.x1 : p.a.x0) == SD_BNRELU;
            const bool cok = cl + lpiece * 8 < C;
            // one buffer load per piece on the source's image; pieces outside the image or past the source's
            // channels are out of range (zeros; masked again after a BN transform)
            unsigned m = 0;
#pragma unroll
            for (int u = 0; u < IT; ++u) {
                const __amdgpu_buffer_rsrc_t hrs =
                    __builtin_amdgcn_make_buffer_rsrc((void*)(s1 ? ib1[u] : ib0[u]), (short)0, hw_img * C * 2, 0x00020000);
#pragma unroll
                for (int i = 0; i < HP; ++i) {
                    const bool ok = (hpx[u][i] >= 0) & cok;
                    m |= (unsigned)ok << (u * HP + i);
                    unsigned off;
                    asm("v_mad_u32_u24 %0, %1, %2, %3" : "=v"(off) : "v"(hpx[u][i]), "s"(C * 2), "v"(lpiece * 16));
                    off = ok ? off : OOB;
                    if (WG_EXP & 262144) {
                        q.hr[u][i] = make_uint4(off, off, off, off);
                        continue;
                    }
                    const auto x = __builtin_amdgcn_raw_buffer_load_b128(hrs, off, cl * 2, 0);
                    q.hr[u][i] = make_uint4(x[0], x[1], x[2], x[3]);
                }
            }
            q.m = m;
            if (++ld_cc == nchunks) {
                ld_cc = 0;
                ++ld_pass;
                geometry();
            }
        };
        auto store = [&](auto S, int buf) __attribute__((always_inline)) {  // halo set S and the weights in wr -> LDS buffer buf
            HSet& q = set_of(S);
            __bf16* hx = smem + buf * BUF;
            float4 s0, s1, h0, h1;
            if (q.bn) {
                const float* sc = sbn + q.cb + lpiece * 8;
                s0 = *reinterpret_cast<const float4*>(sc);
                s1 = *reinterpret_cast<const float4*>(sc + 4);
                h0 = *reinterpret_cast<const float4*>(sc + SBN_MAX);
                h1 = *reinterpret_cast<const float4*>(sc + SBN_MAX + 4);
            }
            if (!(WG_EXP & 32))
#pragma unroll
            for (int u = 0; u < IT; ++u)
#pragma unroll
            for (int i = 0; i < HP; ++i) {  // every piece lands inside the item's halo region
                const int item = ltid + i * 256;
                uint4 v = q.hr[u][i];
                const bool ok = (q.m >> (u * HP + i)) & 1u;
                if (q.bn && !(WG_EXP & 2048)) {
                    v = bnrelu_pk(v, s0, s1, h0, h1);
                    v = ok ? v : make_uint4(0, 0, 0, 0);  // zero padding after the activation
                }
                const int hoff = M16 ? ld_piece<PPX>(item) * HPX * 8 + ld_pixel<PPX>(item) * 8
                                     : ld_pixel<PPX>(item) * HX_LD + ld_piece<PPX>(item) * 8;
                *reinterpret_cast<uint4*>(hx + u * HALO_ITEM + hoff) = v;
            }
            if constexpr (!WCONST && !WDMA) if (!(WG_EXP & 131072)) store_w(buf);
        };
        constexpr std::integral_constant<int, 0> S0{};
        constexpr std::integral_constant<int, 1> S1{};
        constexpr std::integral_constant<int, 2> S2{};
        constexpr std::integral_constant<int, 3> S3{};
        constexpr bool DG = (WG_EXP & 1024) != 0;
        unsigned long long t_st = 0, t_ld = 0, t_br = 0, t0 = 0, t_all = DG ? __builtin_amdgcn_s_memtime() : 0;
        auto stamp = [&](unsigned long long& acc_) __attribute__((always_inline)) {
            if (DG) {
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
                const unsigned long long t1 = __builtin_amdgcn_s_memtime();
                acc_ += t1 - t0;
                t0 = t1;
            } else if (WG_EXP & 8192) {
                asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            }
        };
        auto iter = [&](auto U) __attribute__((always_inline)) {
            if (DG) t0 = __builtin_amdgcn_s_memtime();
            if (!(WG_EXP & 65536)) store(U, decltype(U)::value & 1);
            stamp(t_st);
            if constexpr (WDMA) {
                __builtin_amdgcn_sched_barrier(0);
                dma_w(decltype(U)::value & 1);
                __builtin_amdgcn_sched_barrier(0);
            } else if constexpr (!WCONST) {
                if (!(WG_EXP & 65536)) load_w();
            }
            if (!(WG_EXP & 65536)) load(U);
            stamp(t_ld);
            if constexpr (WDMA && !(WG_EXP & 4194304)) {  // this chunk's weight DMA landed; the halo loads just issued
                __builtin_amdgcn_sched_barrier(0);                // stay in flight (WG_EXP bit 22: no wait, timing only)
                asm volatile("s_waitcnt vmcnt(%0)" ::"i"(IT * HP) : "memory");
            }
            __syncthreads();
            stamp(t_br);
        };
        // WCONST: the second chunk's weights (two chunks per item) in registers of their own, so both loads are in
        // flight with the first halos
        uint4 wr2[WCONST ? W_PER_THREAD : 1];
        if (total > 0) {
            // the loads an iteration would have issued before chunk 0: the halo of chunks 0 .. LS-2, the weights
            // of chunk 0, the halo of chunk LS-1 (WCONST: the weights of both chunks first, stored after the tables)
            // sched barriers: the issue order must be an iteration's (the scheduler may swap independent sets)
            geometry();
            if constexpr (WCONST) {
                load_w();  // chunk 0
                if (nchunks > 1) load_w_into(wr2);  // chunk 1
                __builtin_amdgcn_sched_barrier(0);
            }
            load(S0);
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (LS == 4) {
                load(S1);
                __builtin_amdgcn_sched_barrier(0);
                load(S2);
                __builtin_amdgcn_sched_barrier(0);
            }
            if constexpr (!WCONST && !WDMA) load_w();
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (LS == 4) load(S3);
            else load(S1);
        }
        fill_tables();
        __syncthreads();  // the tables (the MFMA waves meet it before their first chunk)
        if (total > 0) {
            if constexpr (WCONST) {
                store_w(0);
                if (nchunks > 1) store_w_from(1, wr2);
                else store_w(1);  // one chunk per item: chunk 0 in both buffers
            }
            // a multiple of LS iterations, no exit between them (an exit between the sets made the compiler's
            // vmcnt bookkeeping drain every load in half of them); the iterations past the last chunk store
            // zeros into buffers the MFMA waves no longer read, and they meet them with extra barriers
            for (int gi = 0; gi < total; gi += LS) {
                iter(S0);
                iter(S1);
                if constexpr (LS == 4) {
                    iter(S2);
                    iter(S3);
                }
            }
        }
        if (DG && p.dbg && lane == 0) {
            unsigned long long* d = p.dbg + ((size_t)blockIdx.x * 8 + 4 + wid) * 4;
            d[0] = t_st;
            d[1] = t_ld;
            d[2] = t_br;
            d[3] = __builtin_amdgcn_s_memtime() - t_all;
        }
        __syncthreads();  // stats reduction barrier (MFMA waves)
        return;
    }

    // =============================================================== MFMA waves
    fill_tables();
    __syncthreads();  // the tables
    // BN statistics of the stored values, taken from the transposed pieces: a lane always reads channels
    // n0 + 8*(lane % PPP) + 0..7, so it keeps 8 (sum, sumsq) pairs across all of the block's items and the
    // lanes sharing channels are reduced once at the end.
    static_assert(!(STATS && BNS), "one kind of stats rows");
    constexpr int NOWN = STATS || BNS ? 16 : 1;
    // channels n0 + 8*(lane % PPP) + 2q, 2q + 1: own[4q + {0,1}] their sums (STATS, stats_add) or sums of dz (BNS,
    // bns_add), own[4q + {2,3}] their sums of squares or of dz*xhat
    float own[NOWN];
#pragma unroll
    for (int j = 0; j < NOWN; ++j) own[j] = 0.f;
    constexpr int PPP = NT * 4;      // 16-B pieces per pixel row
    // 32-pixel column tile i of this MFMA wave: the M16 instances own RT consecutive ones (in 32-pixel-wide tiles, RT
    // consecutive rows: what the vertical-reuse k-loop below needs), the others every fourth
    // The N = 32 RT = 4 BNS dgrads (32x32x16 MFMAs, VR32) run the same vertical reuse on 32-pixel fragments (one tile row
    // each) and channel halves, in the tap order of the 16x16x32 loop (so their stores equal the STORE instance's)
    constexpr bool VR32 = HC_VR && !M16 && NT == 1 && RT == 4 && CK == 32 && IT == 1;
    auto tile_T = [&](int i) { return M16 || VR32 ? wid * RT + i : wid + 4 * i; };
    // Vertical reuse (the N = 32 RT = 4 instances: full-resolution 16x32 tiles, 4 rows per wave): the taps of one kernel
    // column kw meet the same halo fragments one row apart, so each 16-pixel halo fragment (row hr, half h, shifted by
    // kw) is read once and feeds the up-to-3 output rows hr - kh: (RT + 2) x 2 reads per kw instead of 3 x 2RT, 40 %
    // fewer of the LDS fragment reads that paced the full-resolution layers' MFMA phase. HC_VR=0 builds: the per-tap loop.
    constexpr bool VR = HC_VR && M16 && NT == 1 && RT == 4;
    // B-fragment (pixel) halo offsets of this lane's columns (tap (0,0)), the same for every tile;
    // columns past the tile read pixel 0 and are masked in the epilogue
    int abase[RT];
#pragma unroll
    for (int i = 0; i < RT; ++i) {
        const int m = tile_T(i) * 32 + (lane & 31);
        const int hm = m / p.tw, wm = m - hm * p.tw;
        abase[i] = m < mvalid ? hm * p.hw + wm : 0;
    }
    // M16: 16-pixel column blocks (two per 32-pixel tile); lane l reads pixel l & 15 of its block, piece l >> 4
    int abase16[M16 ? 2 * RT : 1];
    if constexpr (M16) {
#pragma unroll
        for (int i = 0; i < 2 * RT; ++i) {
            const int m = tile_T(i >> 1) * 32 + (i & 1) * 16 + (lane & 15);
            const int hm = m / p.tw, wm = m - hm * p.tw;
            abase16[i] = (lane >> 4) * HPX * 8 + (m < mvalid ? hm * p.hw + wm : 0) * 8;
        }
    }
    f32x16 acc[M16 ? 1 : IT][M16 ? 1 : RT][M16 ? 1 : NT];
    f32x4 acc4[M16 ? 2 * RT : 1][M16 ? 2 * NT : 1];  // M16: [16-pixel block][16-channel block]
    // Epilogue: the bf16 results go through this wave's LDS scratch (pixel rows of BN channels, 16-B pieces
    // XOR-swizzled by pixel so both the row-per-lane writes and the piece-per-lane reads are conflict-free)
    // and leave as stores of EPR whole pixels per instruction (1 KiB contiguous, 8 or 16 full 128-B lines)
    // instead of 32 pixels x 32 B: the scattered form made the MFMA waves wait on store issue for ~20 % of
    // the kernel at full resolution. Buffer stores: pixels outside the image are out of range (dropped).
    constexpr int EPR = 64 / PPP;    // pixels per store instruction
    constexpr int ER = 32 / EPR;     // store instructions per 32-pixel tile
    auto swz = [](int j, int px) { return NT == 2 ? j ^ (px & 7) : j ^ ((px >> 1) & 3); };
    // tile-relative (row << 9 | col) of the pixel this lane stores, 0xffff past the tile; two per register
    // (tiles are < 64 rows and < 512 columns, halo_tile)
    unsigned erel[(RT * ER + 1) / 2];
#pragma unroll
    for (int k = 0; k < (RT * ER + 1) / 2; ++k) erel[k] = 0xffffffffu;
#pragma unroll
    for (int i = 0; i < RT; ++i)
#pragma unroll
        for (int r = 0; r < ER; ++r) {
            const int m = tile_T(i) * 32 + r * EPR + lane / PPP;
            const int hm = m / p.tw, wm = m - hm * p.tw;
            const unsigned v = m < mvalid ? (unsigned)((hm << 9) | wm) : 0xffffu;
            const int k = i * ER + r;
            erel[k / 2] = (erel[k / 2] & ~(0xffffu << (16 * (k & 1)))) | (v << (16 * (k & 1)));
        }
    // M16: the same pixels as offsets from the tile origin in the image (hm * W + wm, -1 past the tile), for the
    // epilogue of items whose tile lies inside the image (no per-row bounds or (row, col) arithmetic)
    constexpr bool EFAST = M16 && !(NT == 2 && RT == 3);  // (2 x 3 tiles: the offsets spill beside the accumulators)
    constexpr int NEO = EFAST ? RT * ER : 1;
    int eoff[NEO];
#pragma unroll
    for (int k = 0; k < NEO; ++k) {
        const int m = tile_T(k / ER) * 32 + (k % ER) * EPR + lane / PPP;
        const int hm = m / p.tw, wm = m - hm * p.tw;
        eoff[k] = m < mvalid ? hm * p.W + wm : -1;
    }
    __bf16* const scw = scr + wid * SCR_PX * BN;
    // BNS: the lane's 8 channels are fixed (piece lane % PPP): their BatchNorm constants in registers, and the y
    // pieces of an item's stores prefetched while its last chunk is in the matrix core
    constexpr int NBK = BNS ? 8 : 1, NYQ = BNS ? RT * ER : 1;
    BnsK bk[NBK / 2 > 0 ? NBK / 2 : 1];  // channel pairs (2q, 2q+1)
    uint4 yq[NYQ];
    if constexpr (BNS) {
        const int c = n0 + (lane % PPP) * 8;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            float v[4][2];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int ch = c + 2 * q + h;
                const bool cin = ch < p.N;
                v[0][h] = cin ? p.bsc[ch] : 0.f;
                v[1][h] = cin ? p.bsh[ch] : 0.f;
                v[2][h] = cin ? p.bis[ch] : 0.f;
                v[3][h] = cin ? -p.bmu[ch] * p.bis[ch] : 0.f;
            }
            bk[q].sc = f32x2{v[0][0], v[0][1]};
            bk[q].sh = f32x2{v[1][0], v[1][1]};
            bk[q].is = f32x2{v[2][0], v[2][1]};
            bk[q].nmi = f32x2{v[3][0], v[3][1]};
        }
    }
    auto prefetch_y = [&](int itm) __attribute__((always_inline)) {  // the y pieces this lane stores for item itm
        const int sp = slot + itm * p.gper;
        const int b = sp / p.tiles, tl = sp - b * p.tiles;
        const int ty = tl / p.tiles_x;
        const int h0 = ty * p.th, w0 = (tl - ty * p.tiles_x) * p.tw;
        const int hw_img = p.H * p.W;
        const __amdgpu_buffer_rsrc_t ry = __builtin_amdgcn_make_buffer_rsrc(
            (void*)(p.by + (size_t)b * hw_img * p.N), (short)0, hw_img * p.N * 2, 0x00020000);
#pragma unroll
        for (int k = 0; k < RT * ER; ++k) {
            const unsigned rel = (erel[k / 2] >> (16 * (k & 1))) & 0xffffu;
            const int h = h0 + (int)(rel >> 9), w = w0 + (int)(rel & 511u);
            const int c = n0 + (lane % PPP) * 8;
            const bool in = (rel != 0xffffu) & (h < p.H) & (w < p.W) & (c < p.N);
            const unsigned off = in ? (unsigned)((h * p.W + w) * p.N + c) * 2u : 0x80000000u;
            const auto v = __builtin_amdgcn_raw_buffer_load_b128(ry, off, 0, 0);
            yq[k] = make_uint4(v[0], v[1], v[2], v[3]);
        }
    };

    constexpr bool DG = (WG_EXP & 1024) != 0;
    unsigned long long t_cp = 0, t_ep = 0, t_br = 0, t0 = 0, t_all = DG ? __builtin_amdgcn_s_memtime() : 0;
    int cc = 0, pass = 0;
    for (int gi = 0; gi < total; ++gi) {
        if (DG) t0 = __builtin_amdgcn_s_memtime();
        if (WG_EXP & 16384) {
            asm volatile("" ::: "memory");
            __builtin_amdgcn_sched_barrier(0);
        }
        __syncthreads();  // chunk gi is in buffer gi & 1 (and the loaders may overwrite the other one)
        if (DG) {
            const unsigned long long t1 = __builtin_amdgcn_s_memtime();
            t_br += t1 - t0;
            t0 = t1;
        }
        if (WG_EXP & 16384) {
            asm volatile("" ::: "memory");
            __builtin_amdgcn_sched_barrier(0);
        }
        if (cc == 0) {
            if constexpr (M16) {
#pragma unroll
                for (int i = 0; i < 2 * RT; ++i)
#pragma unroll
                    for (int t = 0; t < 2 * NT; ++t) acc4[i][t] = f32x4{0.f, 0.f, 0.f, 0.f};
            } else {
#pragma unroll
            for (int u = 0; u < IT; ++u)
#pragma unroll
            for (int i = 0; i < RT; ++i)
#pragma unroll
                for (int t = 0; t < NT; ++t)
#pragma unroll
                    for (int r = 0; r < 16; ++r) acc[u][i][t][r] = 0.f;
            }
        }
        if constexpr (BNS) {
            if (cc == nchunks - 1) prefetch_y(pass);  // IT == 1: the pass is the item
        }
        const __bf16* hx = smem + (gi & 1) * BUF;
        const __bf16* wl = hx + HALO_ELEMS;
        // KS k-steps (tap, 16-channel part); fragments are read one step ahead of the MFMAs
        // (register ring) so LDS latency stays behind the matrix core (2 steps measured no faster)
#ifndef HC_PF
#define HC_PF 1
#endif
        constexpr int PF = HC_PF;
        bf16x8 af[PF + 1][IT][RT], bfr[PF + 1][NT];
        auto read_frags = [&](int step) {
            const int slot_ = step % (PF + 1);
            // CK 8: a k-step is two taps of 8 channels (lane half = tap parity); tap 9 is padding
            const int tapv = CK == 8 ? 2 * step + (lane >> 5) : step / (CK >= 16 ? CK / 16 : 1);
            const int tap = tapv < 9 ? tapv : 8;
            const int c8 = CK == 8 ? 0 : (step % (CK >= 16 ? CK / 16 : 1)) * 2 + (lane >> 5);  // 8-channel piece
            const int toff = (tap / 3) * p.hw + tap % 3;
#pragma unroll
            for (int t = 0; t < NT; ++t) {
                bfr[slot_][t] = *reinterpret_cast<const bf16x8*>(wl + (t * 32 + (lane & 31)) * W_LD + tap * CK + c8 * 8);
                if (CK == 8 && tapv > 8) bfr[slot_][t] = bf16x8{};  // zero weights for the padding tap
            }
#pragma unroll
            for (int u = 0; u < IT; ++u)
#pragma unroll
            for (int i = 0; i < RT; ++i)
                af[slot_][u][i] = *reinterpret_cast<const bf16x8*>(hx + u * HALO_ITEM + (abase[i] + toff) * HX_LD + c8 * 8);
        };
        if constexpr (VR) {
          if (!(WG_EXP & 8)) {
            constexpr int R = RT, NH = R + 2, NS = 3 * NH, PV = 2;  // rows, halo rows, steps (kw, hr), read-ahead
            constexpr int HWV = 34;                                 // halo width of a 32-pixel-wide tile
            // weights of taps (kh, kw), 16-channel blocks t: one set; column kw+1's kh = 0, 1 are read during column
            // kw's last row step (which uses kh = 2 only), its kh = 2 during column kw+1's first (kh = 0 only)
            bf16x8 av[3][2];
            bf16x8 xv[PV + 1][2];    // halo fragments of step s (halves h), ring
            const __bf16* const xb = hx + (lane >> 4) * HPX * 8 + (wid * RT * HWV + (lane & 15)) * 8;
            auto readA = [&](int kw, int kh) __attribute__((always_inline)) {
#pragma unroll
                for (int t = 0; t < 2; ++t)
                    av[kh][t] = *reinterpret_cast<const bf16x8*>(
                        wl + (t * 16 + (lane & 15)) * W_LD + (kh * 3 + kw) * CK + ((lane >> 4) ^ wswz(lane & 15)) * 8);
            };
            auto readX = [&](int st) __attribute__((always_inline)) {
                const int kw = st / NH, hr = st % NH;
#pragma unroll
                for (int h = 0; h < 2; ++h)
                    xv[st % (PV + 1)][h] = *reinterpret_cast<const bf16x8*>(xb + (hr * HWV + h * 16 + kw) * 8);
            };
#pragma unroll
            for (int kh = 0; kh < 3; ++kh) readA(0, kh);
#pragma unroll
            for (int st = 0; st < PV; ++st) readX(st);
#pragma unroll
            for (int st = 0; st < NS; ++st) {
                const int kw = st / NH, hr = st % NH;
                if (hr == NH - 1 && kw < 2) {  // this step uses kh = 2 only
                    readA(kw + 1, 0);
                    readA(kw + 1, 1);
                }
                if (hr == 0 && kw > 0) readA(kw, 2);  // this step uses kh = 0 only
                if (st + PV < NS) readX(st + PV);
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int kh = 0; kh < 3; ++kh) {
                    const int r = hr - kh;  // output row of this (halo row, kernel row) pair
                    if (r < 0 || r >= R) continue;
#pragma unroll
                    for (int h = 0; h < 2; ++h)
#pragma unroll
                        for (int t = 0; t < 2; ++t)
                            acc4[2 * r + h][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(
                                av[kh][t], xv[st % (PV + 1)][h], acc4[2 * r + h][t], 0, 0, 0);
                }
                __builtin_amdgcn_sched_barrier(0);
            }
          }
        }
        if constexpr (M16) {
          if (!VR && !(WG_EXP & 8)) {
            // one k-step per tap: A = 16 weight rows x 32 channels, B = 32 channels x 16 halo pixels
            bf16x8 a16[PF + 1][2 * NT], b16[PF + 1][2 * RT];
            auto read16 = [&](int tap) {
                const int sl = tap % (PF + 1);
                const int toff = ((tap / 3) * p.hw + tap % 3) * 8;
#pragma unroll
                for (int t = 0; t < 2 * NT; ++t)
                    a16[sl][t] = *reinterpret_cast<const bf16x8*>(wl + (t * 16 + (lane & 15)) * W_LD + tap * CK +
                                                                  ((lane >> 4) ^ wswz(lane & 15)) * 8);
#pragma unroll
                for (int i = 0; i < 2 * RT; ++i) b16[sl][i] = *reinterpret_cast<const bf16x8*>(hx + abase16[i] + toff);
            };
#pragma unroll
            for (int tap = 0; tap < PF; ++tap) read16(tap);
#pragma unroll
            for (int tap = 0; tap < 9; ++tap) {
                if (tap + PF < 9) read16(tap + PF);
                __builtin_amdgcn_sched_barrier(0);
                const int sl = tap % (PF + 1);
#pragma unroll
                for (int i = 0; i < 2 * RT; ++i)
#pragma unroll
                    for (int t = 0; t < 2 * NT; ++t)
                        acc4[i][t] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a16[sl][t], b16[sl][i], acc4[i][t], 0, 0, 0);
                __builtin_amdgcn_sched_barrier(0);
            }
          }
        } else if (VR32 && !(WG_EXP & 8)) {
            // steps (kw, halo row hr, channel half ch); weights of (kh, kw, ch) in one set: column kw+1's kh = 0, 1 are
            // read during column kw's last row (kh = 2 only), its kh = 2 during its own first row (kh = 0 only)
            constexpr int R = RT, NH = R + 2, NS = 3 * NH * 2, PV = 2, HWV = 34;
            bf16x8 av[3][2];
            bf16x8 xv[PV + 1];
            const __bf16* const xb = hx + (wid * RT * HWV + (lane & 31)) * HX_LD + (lane >> 5) * 8;
            auto readA = [&](int kw, int kh) __attribute__((always_inline)) {
#pragma unroll
                for (int ch = 0; ch < 2; ++ch)
                    av[kh][ch] = *reinterpret_cast<const bf16x8*>(wl + (lane & 31) * W_LD + (kh * 3 + kw) * CK +
                                                                  (ch * 2 + (lane >> 5)) * 8);
            };
            auto readX = [&](int st) __attribute__((always_inline)) {
                const int kw = st / (2 * NH), hr = (st >> 1) % NH, ch = st & 1;
                xv[st % (PV + 1)] = *reinterpret_cast<const bf16x8*>(xb + (hr * HWV + kw) * HX_LD + ch * 16);
            };
#pragma unroll
            for (int kh = 0; kh < 3; ++kh) readA(0, kh);
#pragma unroll
            for (int st = 0; st < PV; ++st) readX(st);
#pragma unroll
            for (int st = 0; st < NS; ++st) {
                const int kw = st / (2 * NH), hr = (st >> 1) % NH, ch = st & 1;
                if (hr == NH - 1 && ch == 0 && kw < 2) {
                    readA(kw + 1, 0);
                    readA(kw + 1, 1);
                }
                if (hr == 0 && ch == 0 && kw > 0) readA(kw, 2);
                if (st + PV < NS) readX(st + PV);
                __builtin_amdgcn_sched_barrier(0);
#pragma unroll
                for (int kh = 0; kh < 3; ++kh) {
                    const int r = hr - kh;
                    if (r < 0 || r >= R) continue;
                    acc[0][r][0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(av[kh][ch], xv[st % (PV + 1)], acc[0][r][0], 0,
                                                                           0, 0);
                }
                __builtin_amdgcn_sched_barrier(0);
            }
        } else if (!(WG_EXP & 8)) {
#pragma unroll
        for (int step = 0; step < PF; ++step) read_frags(step);
#pragma unroll
        for (int step = 0; step < KS; ++step) {
            if (step + PF < KS) read_frags(step + PF);
            __builtin_amdgcn_sched_barrier(0);
            const int sl = step % (PF + 1);
#pragma unroll
            for (int u = 0; u < IT; ++u)
#pragma unroll
            for (int i = 0; i < RT; ++i)
#pragma unroll
                for (int t = 0; t < NT; ++t)
                    acc[u][i][t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(bfr[sl][t], af[sl][u][i], acc[u][i][t], 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
        }
        }

        if (DG) {
            const unsigned long long t1 = __builtin_amdgcn_s_memtime();
            t_cp += t1 - t0;
            t0 = t1;
        }
        if (WG_EXP & 16384) {
            asm volatile("" ::: "memory");
            __builtin_amdgcn_sched_barrier(0);
        }
        if (++cc == nchunks) {
#pragma unroll
          for (int u = 0; u < IT; ++u) {
            // ---------------------------------------------------- epilogue of the pass's item u
            const int item = pass * IT + u;
            if (IT > 1 && item >= my_items) break;  // the last pass's missing item (block-uniform)
            const int sp = slot + item * p.gper;
            const int b = sp / p.tiles, tl = sp - b * p.tiles;
            const int ty = tl / p.tiles_x;
            const int h0 = ty * p.th, w0 = (tl - ty * p.tiles_x) * p.tw;
            const int hw_img = p.H * p.W;
            if constexpr (!STATS && !BNS) {
                if (p.part) {
                    // split-K partials straight from the accumulators (4 consecutive channels of one pixel per 16-B
                    // store; batch-1 sizes, a few MB per launch)
                    float* const pk = p.part + ((size_t)ks * p.npix + (size_t)b * hw_img) * p.N;
                    auto put = [&](int m, int c, float a0, float a1, float a2, float a3) __attribute__((always_inline)) {
                        const int hm = m / p.tw, wm = m - hm * p.tw;
                        if ((m < mvalid) & (h0 + hm < p.H) & (w0 + wm < p.W) & (n0 + c < p.N))
                            *reinterpret_cast<float4*>(pk + ((size_t)(h0 + hm) * p.W + w0 + wm) * p.N + n0 + c) =
                                make_float4(a0, a1, a2, a3);
                    };
                    if constexpr (M16) {
#pragma unroll
                        for (int i2 = 0; i2 < 2 * RT; ++i2)
#pragma unroll
                            for (int t = 0; t < 2 * NT; ++t)
                                put(tile_T(i2 >> 1) * 32 + (i2 & 1) * 16 + (lane & 15), t * 16 + 4 * (lane >> 4),
                                    acc4[i2][t][0], acc4[i2][t][1], acc4[i2][t][2], acc4[i2][t][3]);
                    } else {
#pragma unroll
                        for (int i = 0; i < RT; ++i)
#pragma unroll
                            for (int t = 0; t < NT; ++t)
#pragma unroll
                                for (int g4 = 0; g4 < 4; ++g4)
                                    put(tile_T(i) * 32 + (lane & 31), t * 32 + 8 * g4 + 4 * (lane >> 5),
                                        acc[u][i][t][4 * g4], acc[u][i][t][4 * g4 + 1], acc[u][i][t][4 * g4 + 2],
                                        acc[u][i][t][4 * g4 + 3]);
                    }
                    continue;
                }
            }
            const bool split = p.epi == SD_EPI_SPLIT || p.epi == SD_EPI_SPLIT_STATS;
            const int ns = split ? p.n_split : p.N;
            const __amdgpu_buffer_rsrc_t rs0 = __builtin_amdgcn_make_buffer_rsrc(
                (void*)(p.out0 + (size_t)b * hw_img * ns), (short)0, hw_img * ns * 2, 0x00020000);
            const __amdgpu_buffer_rsrc_t rs1 = __builtin_amdgcn_make_buffer_rsrc(
                (void*)(split ? p.out1 + (size_t)b * hw_img * (p.N - ns) : p.out0), (short)0,
                split ? hw_img * (p.N - ns) * 2 : 0, 0x00020000);
            constexpr int NPART = M16 ? 2 * RT : RT;  // epilogue passes: 16-pixel halves (M16) or 32-pixel tiles
            constexpr int RPP = M16 ? ER / 2 : ER;     // store instructions per pass
            // one store row: BN statistics of piece v and its 16-B store(s) (32-pixel tile i, store row r)
            const bool inside = h0 + p.th <= p.H && w0 + p.tw <= p.W;  // the whole tile is in the image
            const int pix0 = h0 * p.W + w0;
            auto row_out = [&](const uint4 v, const int i, const int r, auto SPL, auto INS) {
                const int j = lane % PPP;
                bool live;
                int pix;
                if constexpr (decltype(INS)::v) {
                    live = eoff[i * ER + r] >= 0;
                    pix = pix0 + eoff[i * ER + r];
                } else {
                    const unsigned rel = (erel[(i * ER + r) / 2] >> (16 * ((i * ER + r) & 1))) & 0xffffu;
                    const int h = h0 + (int)(rel >> 9), w = w0 + (int)(rel & 511u);
                    live = (rel != 0xffffu) & (h < p.H) & (w < p.W);
                    pix = h * p.W + w;
                }
                const bool in = live & !(WG_EXP & 4096);
                const int c = n0 + j * 8;
                if constexpr (BNS) {
                    bns_add(own, v, yq[i * ER + r], live, bk);
                }
                if constexpr (STATS) {
                    stats_add(own, v, live);
                }
                __attribute__((ext_vector_type(4))) unsigned data = {v.x, v.y, v.z, v.w};
                if (!SPL.v) {
                    const unsigned off = (in & (c < p.N)) ? (unsigned)(pix * p.N + c) * 2u : 0x80000000u;
                    __builtin_amdgcn_raw_buffer_store_b128(data, rs0, off, 0, HC_ST_AUX);
                } else {  // dgrad of a concatenation: channels < n_split to out0, the rest to out1
                    const unsigned o0 = (in & (c < ns)) ? (unsigned)(pix * ns + c) * 2u : 0x80000000u;
                    const unsigned o1 = (in & (c >= ns) & (c < p.N)) ? (unsigned)(pix * (p.N - ns) + c - ns) * 2u
                                                                   : 0x80000000u;
                    __builtin_amdgcn_raw_buffer_store_b128(data, rs0, o0, 0, HC_ST_AUX);
                    __builtin_amdgcn_raw_buffer_store_b128(data, rs1, o1, 0, HC_ST_AUX);
                }
            };
            if constexpr (M16) {
                // All halves' scratch writes and read-backs issue back to back, then the item's stores: one LDS
                // round trip per item instead of one per half (LDS is in order per wave, so a half's writes land
                // after the previous half's reads of the same scratch rows).
                // (in groups of EG halves where all of them would not fit beside the accumulators)
                constexpr int EG = (NT == 2 && RT >= 3) ? 2 : NPART;
                static_assert(NPART % EG == 0, "whole groups of halves");
                auto epi16 = [&](auto SPL, auto INS) {
#pragma unroll
                  for (int g0 = 0; g0 < NPART; g0 += EG) {
                    uint4 vv[EG][RPP];
#pragma unroll
                    for (int e = 0; e < EG; ++e) {
                        const int i2 = g0 + e;
                        // lane l holds channels 4 * (l >> 4) + 0..3 of each 16-channel block for pixel l & 15 of
                        // the half: 8-B pieces into the pixel rows of the scratch, read back as whole 16-B pieces
#pragma unroll
                        for (int t = 0; t < 2 * NT; ++t) {
                            bf16x4 v;
                            const int px = lane & 15, c = t * 16 + 4 * (lane >> 4);
                            if constexpr (OAFF) {
                                const float4 sc = *reinterpret_cast<const float4*>(oaff + c);
                                const float4 sh = *reinterpret_cast<const float4*>(oaff + BN + c);
                                v[0] = (__bf16)fmaf(acc4[i2][t][0], sc.x, sh.x);
                                v[1] = (__bf16)fmaf(acc4[i2][t][1], sc.y, sh.y);
                                v[2] = (__bf16)fmaf(acc4[i2][t][2], sc.z, sh.z);
                                v[3] = (__bf16)fmaf(acc4[i2][t][3], sc.w, sh.w);
                            } else {
#pragma unroll
                                for (int q = 0; q < 4; ++q) v[q] = (__bf16)acc4[i2][t][q];
                            }
                            *reinterpret_cast<uint2*>(scw + px * BN + swz(c >> 3, px) * 8 + (c & 4)) = *reinterpret_cast<uint2*>(&v);
                        }
                        asm volatile("" ::: "memory");  // the reads below after the writes above
#pragma unroll
                        for (int rr = 0; rr < RPP; ++rr) {
                            const int px = rr * EPR + lane / PPP, j = lane % PPP;
                            vv[e][rr] = *reinterpret_cast<const uint4*>(scw + px * BN + swz(j, px) * 8);
                        }
                        asm volatile("" ::: "memory");  // the next half's writes after these reads
                    }
#pragma unroll
                    for (int e = 0; e < EG; ++e)
#pragma unroll
                        for (int rr = 0; rr < RPP; ++rr)
                            row_out(vv[e][rr], (g0 + e) >> 1, ((g0 + e) & 1) * RPP + rr, SPL, INS);
                  }
                };
                if (split) {
                    epi16(BoolC<true>{}, BoolC<false>{});
                } else if constexpr (EFAST) {
                    if (inside) epi16(BoolC<false>{}, BoolC<true>{});
                    else epi16(BoolC<false>{}, BoolC<false>{});
                } else {
                    epi16(BoolC<false>{}, BoolC<false>{});
                }
            } else {  // 32x32 tiles: the scratch round trips of TG tiles back to back, then their stores
                constexpr int TG = BNS ? 1 : (NT == 2 && RT == 4) ? 2 : RT;  // BNS and 4 tiles x 4 rows spill
#pragma unroll
            for (int i0 = 0; i0 < RT; i0 += TG) {
              uint4 rows[TG][RPP];
#pragma unroll
              for (int e = 0; e < TG; ++e) {
                const int i = i0 + e;
#pragma unroll
                for (int t = 0; t < NT; ++t) {
                    uint2 pk[4];  // this lane's 4 channels of each 8-channel group g4, packed bf16
#pragma unroll
                    for (int g4 = 0; g4 < 4; ++g4) {
                        bf16x4 v;
                        if constexpr (OAFF) {  // rows 8*g4 + 4*(lane >> 5) + q of the 32-channel tile t
                            const int c = t * 32 + 8 * g4 + 4 * (lane >> 5);
                            const float4 sc = *reinterpret_cast<const float4*>(oaff + c);
                            const float4 sh = *reinterpret_cast<const float4*>(oaff + BN + c);
                            v[0] = (__bf16)fmaf(acc[u][i][t][4 * g4 + 0], sc.x, sh.x);
                            v[1] = (__bf16)fmaf(acc[u][i][t][4 * g4 + 1], sc.y, sh.y);
                            v[2] = (__bf16)fmaf(acc[u][i][t][4 * g4 + 2], sc.z, sh.z);
                            v[3] = (__bf16)fmaf(acc[u][i][t][4 * g4 + 3], sc.w, sh.w);
                        } else {
#pragma unroll
                            for (int q = 0; q < 4; ++q) v[q] = (__bf16)acc[u][i][t][4 * g4 + q];
                        }
                        pk[g4] = *reinterpret_cast<uint2*>(&v);
                    }
                    // lanes l and l+32 hold the two 4-channel halves of each 8-channel group of one pixel:
                    // v_permlane32_swap on groups (k, k+1) leaves group k whole in lane l and group k+1 in l+32
#pragma unroll
                    for (int k = 0; k < 4; k += 2) {
                        const auto rx = __builtin_amdgcn_permlane32_swap(pk[k].x, pk[k + 1].x, false, false);
                        const auto ry = __builtin_amdgcn_permlane32_swap(pk[k].y, pk[k + 1].y, false, false);
                        const int px = lane & 31, j = t * 4 + k + (lane >> 5);
                        *reinterpret_cast<uint4*>(scw + px * BN + swz(j, px) * 8) = make_uint4(rx[0], ry[0], rx[1], ry[1]);
                    }
                }
                asm volatile("" ::: "memory");  // LDS is in order per wave: the reads below see the writes above
#pragma unroll
                for (int r = 0; r < RPP; ++r) {
                    const int px = r * EPR + lane / PPP, j = lane % PPP;  // pixel within the tile's scratch rows
                    rows[e][r] = *reinterpret_cast<const uint4*>(scw + px * BN + swz(j, px) * 8);
                }
                asm volatile("" ::: "memory");  // the next tile's writes after these reads
              }
#pragma unroll
              for (int e = 0; e < TG; ++e) {
                const int i = i0 + e;
#pragma unroll
                for (int r = 0; r < RPP; ++r) {
                    const int j = lane % PPP;
                    const uint4 v = rows[e][r];
                    const unsigned rel = (erel[(i * ER + r) / 2] >> (16 * ((i * ER + r) & 1))) & 0xffffu;
                    const int h = h0 + (int)(rel >> 9), w = w0 + (int)(rel & 511u);
                    const bool live = (rel != 0xffffu) & (h < p.H) & (w < p.W);
                    const bool in = live & !(WG_EXP & 4096);
                    const int pix = h * p.W + w, c = n0 + j * 8;
                    if constexpr (BNS) {
                        bns_add(own, v, yq[i * ER + r], live, bk);
                    }
                    if constexpr (STATS) {
                        stats_add(own, v, live);
                    }
                    __attribute__((ext_vector_type(4))) unsigned data = {v.x, v.y, v.z, v.w};
                    if (!split) {
                        const unsigned off = (in & (c < p.N)) ? (unsigned)(pix * p.N + c) * 2u : 0x80000000u;
                        __builtin_amdgcn_raw_buffer_store_b128(data, rs0, off, 0, HC_ST_AUX);
                    } else {  // dgrad of a concatenation: channels < n_split to out0, the rest to out1
                        const unsigned o0 = (in & (c < ns)) ? (unsigned)(pix * ns + c) * 2u : 0x80000000u;
                        const unsigned o1 = (in & (c >= ns) & (c < p.N)) ? (unsigned)(pix * (p.N - ns) + c - ns) * 2u
                                                                       : 0x80000000u;
                        __builtin_amdgcn_raw_buffer_store_b128(data, rs0, o0, 0, HC_ST_AUX);
                        __builtin_amdgcn_raw_buffer_store_b128(data, rs1, o1, 0, HC_ST_AUX);
                    }
                }
              }
            }
            }
          }
            cc = 0;
            ++pass;
            if (DG) {
                const unsigned long long t1 = __builtin_amdgcn_s_memtime();
                t_ep += t1 - t0;
                t0 = t1;
            }
        }
    }
    for (int e = total; e < padded; ++e) __syncthreads();  // the loaders' iterations past the last chunk
    if (DG && p.dbg && lane == 0) {
        unsigned long long* d = p.dbg + ((size_t)blockIdx.x * 8 + wid) * 4;
        d[0] = t_cp;
        d[1] = t_ep;
        d[2] = t_br;
        d[3] = __builtin_amdgcn_s_memtime() - t_all;
    }

    // ---------------------------------------------------------------- BN statistics row
    if constexpr (STATS || BNS) {
        // lanes l, l + PPP, l + 2*PPP, ... hold the same 8 channels (of different pixels)
#pragma unroll
        for (int k = 0; k < NOWN; ++k) {
#pragma unroll
            for (int o = PPP; o < 64; o <<= 1) own[k] += __shfl_xor(own[k], o);
        }
        if (lane < PPP) {
#pragma unroll
            for (int k = 0; k < NOWN; ++k)  // k: channel k / 2, {sum, sumsq} k & 1
                redf[(wid * BN + lane * 8 + k / 2) * 2 + (k & 1)] =
                    own[(k & ~3) | ((k & 1) << 1) | ((k >> 1) & 1)];  // stats_add / bns_add layout
        }
    }
    __syncthreads();
    if ((STATS || BNS) && tid < BN && n0 + tid < p.N) {
        float s = 0.f, ss = 0.f;
#pragma unroll
        for (int w = 0; w < 4; ++w) {
            s += redf[(w * BN + tid) * 2];
            ss += redf[(w * BN + tid) * 2 + 1];
        }
        reinterpret_cast<float2*>(p.stats)[(size_t)slot * p.N + n0 + tid] = make_float2(s, ss);
    }
}

template <int NT, int RT, int CK, bool STATS, bool WCONST, int IT, bool BNS, bool OAFF = false, bool RAW = false>
__global__ __launch_bounds__(512) void k_halo_conv(const HFwdArgs p) {
    halo_conv_body<NT, RT, CK, STATS, WCONST, IT, BNS, OAFF, RAW>(p);
}

// =====================================================================================
// wgrad: any 3x3 weight gradient with M = 32 or a multiple of 64 (grid.z = 64-row blocks of dy)
// =====================================================================================
// Tiles are th x tw pixels (th*tw <= 256), flattened into 32-pixel k-steps; LDS tables give each
// flattened pixel its halo offset and (row, col), so every image size tiles with little waste.
struct HWgArgs {
    const __bf16* dy;  // [pixels][M]
    HaloSrc x;
    int H, W, th, tw, hw, nhalo, tiles_x, tiles_y, ntiles, tiles_per_split;
    int M, N;          // N = 9 * ctot
    float* slab;
    int xcd;           // 1: XCD-contiguous block numbering (block count % 8 == 0)
    unsigned long long* dbg;  // timing-diagnostic builds only (WG_EXP & 1024): per-wave cycle counters
    // k_halo_wgrad_ws<..., BNB = true>: the BatchNorm-backward apply (sd_bn_bwd_apply) runs in the dy staging.
    // The loaders read the raw pair (da, y) instead of dy, form dy = k0*(dz - k1 - xhat*k2) (dz = da where
    // y*scale+shift > 0, xhat = (y-mean)*invstd, coef = {k0, k1, k2} per channel), stage it, and write it to
    // `dy` for the dgrad: tile t by the x-channel block t % ncc, so every dy piece is written exactly once.
    const __bf16* bda;
    const __bf16* by;
    const float *bsc, *bsh, *bmu, *bis, *bcoef;
    int ncc;
};

constexpr int XW_LD = CK + 16;  // halo pixel stride for transposed reads (96 B)
// wgrad loader piece `item` -> (halo pixel, piece): an 8-lane ds_write_b128 group covers 4 pixels x 2
// pieces, slots 6j + {0,1} (j < 4) = 8 distinct slots mod 8 at the 6-slot stride (pixel-major order
// had two 2-way conflicts per group). The piece is fixed per thread (bits 0 and 4 of tid).
__device__ __forceinline__ int wg_pixel(int item) { return (item >> 5) * 8 + ((item >> 3) & 1) * 4 + ((item >> 1) & 3); }
__device__ __forceinline__ int wg_piece(int item) { return (item & 1) + ((item >> 4) & 1) * 2; }
constexpr int HP_PER_THREAD = HMAX * (CK / 8) / 256;  // wgrad halo pieces per thread (6)
constexpr int WG_MAXPX = 256;   // pixels per wgrad tile (8 k-steps)



// BNB: BatchNorm-backward apply in the dy staging (no dy written: enc1.0 has no dgrad). X8: an x source of at most 8
// channels (enc1.0's padded input): one 8-channel piece per halo pixel, 2 per thread instead of 6 pieces of which 3 in 4
// were past the channels (loaded from a clamped address and discarded). The chunk's other pieces are never written:
// they only feed the dW columns of channels >= 8, which the slab write skips. The freed registers hold a second tile
// in flight (BNB, one (da, y) set: latency-bound at 3.9 TB/s, r06).
template <int COUT, bool BNB, bool X8 = false>
__global__ __launch_bounds__(256, 2) void k_halo_wgrad(const HWgArgs p) {  // two blocks per CU (LDS: 63-80 KB)
    constexpr int DY_LD = COUT + 16;             // 96 B / 160 B rows: conflict-free transposed reads
    constexpr int RM = COUT / 32;                // 16-row tiles of output channels per wave
    constexpr int DY_PIECES = WG_MAXPX * (COUT / 8);
    constexpr int DY_PER_THREAD = DY_PIECES / 256;
    constexpr int DY_ELEMS = WG_MAXPX * DY_LD, HX_ELEMS = HMAX * XW_LD;
    __shared__ __attribute__((aligned(16))) __bf16 smem[DY_ELEMS + HX_ELEMS];
    __shared__ int hoff[WG_MAXPX + 8];           // halo offset of flattened pixel m (tap (0,0))
    __shared__ int prc[WG_MAXPX];                // (row << 16 | col) of pixel m, -1 past the tile
    // BNB: the folded BatchNorm-backward constants of the block's dy channels (scale, shift, Bz, Cz; bn_bwd_pk),
    // read per tile (in registers they would cost the kernel its second wave per SIMD)
    __shared__ __attribute__((aligned(16))) float kbn[BNB ? 4 * COUT : 4];
    __bf16* dys = smem;
    __bf16* hxs = smem + DY_ELEMS;

    const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
    // block -> (chunk, dy block, split). With p.xcd the hardware order (x fastest, dealt round-robin to
    // the 8 XCDs) is renumbered so each XCD owns a contiguous range of splits with all their chunks and
    // dy blocks: the blocks that read the same dy tile (every chunk) and the same x halo (every dy
    // block) share that XCD's L2 instead of fetching it once per XCD.
    int cc = blockIdx.x, zb = blockIdx.z, split = blockIdx.y;
    if (p.xcd) {
        const int G = gridDim.x * gridDim.y * gridDim.z;
        const int L = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
        const int lg = (L & 7) * (G >> 3) + (L >> 3);
        cc = lg % gridDim.x;
        const int r = lg / gridDim.x;
        zb = r % gridDim.z;
        split = r / gridDim.z;
    }
    const int mb = zb * COUT;                    // this block's dy channels
    const int t_begin = split * p.tiles_per_split;
    const int t_end = min(p.ntiles, t_begin + p.tiles_per_split);
    const int co0 = (wid >> 1) * (COUT / 2);     // this wave's output-channel rows
    const int ci0 = (wid & 1) * 16;              // this wave's 16 input channels of the chunk
    const int mvalid = p.th * p.tw;
    const int ksteps = (mvalid + 31) >> 5;

    for (int m = tid; m < WG_MAXPX + 8; m += 256) {
        const int hm = m / p.tw, wm = m - hm * p.tw;
        const bool in = m < mvalid;
        hoff[m] = in ? hm * p.hw + wm : 0;
        if (m < WG_MAXPX) prc[m] = in ? (hm << 16 | wm) : -1;
    }
    if constexpr (BNB) {
        for (int j = tid; j < COUT; j += 256) {
            const int c = mb + j;
            const float k1 = p.bcoef[3 * c + 1], k2 = p.bcoef[3 * c + 2];
            const float is = p.bis[c], sc = p.bsc[c], sh = p.bsh[c];
            kbn[j] = sc;
            kbn[COUT + j] = sh;
            kbn[2 * COUT + j] = -is * k2;
            kbn[3 * COUT + j] = is * k2 * sh + sc * (p.bmu[c] * is * k2 - k1);
        }
    }
    constexpr int HPT = X8 ? (HMAX + 255) / 256 : HP_PER_THREAD;  // halo pieces per thread
    int hgeo[HPT];                               // (row << 16 | col) of this thread's halo pieces
#pragma unroll
    for (int i = 0; i < HPT; ++i) {
        const int px = X8 ? tid + i * 256 : wg_pixel(tid + i * 256);
        const int hy = px / p.hw;
        hgeo[i] = px < p.nhalo ? (hy << 16 | (px - hy * p.hw)) : -1;
    }
    __syncthreads();

    f32x4 acc[9][RM];
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
        for (int i = 0; i < RM; ++i) acc[t][i] = f32x4{0.f, 0.f, 0.f, 0.f};

    // Register sets for the tiles in flight (global -> registers) while a tile is in the matrix core:
    // two for M = 32 (one tile of cover was shorter than an HBM round trip at full resolution; three
    // measured no faster)
    // (BNB: one, the raw (da, y) pair of a second set does not fit beside the halo in two waves per SIMD)
    constexpr int WS = COUT == 32 && (!BNB || X8) ? 2 : 1;
    uint4 dr[WS][DY_PER_THREAD], xr[WS][HPT];
    uint4 yr[BNB ? WS : 1][BNB ? DY_PER_THREAD : 1];  // BNB: the raw y pieces beside da in dr
    unsigned dmask[WS], xmask[WS];  // bit i: piece i valid (else stored as zeros)
    // fixed for the whole block (slab: any valid address)
    const HaloCol hc = halo_col(p.x, cc * CK + (X8 ? 0 : wg_piece(tid)) * 8, p.slab);
    auto load_tile = [&](auto S, int tile) __attribute__((always_inline)) {
        const int tx = tile % p.tiles_x;
        const int rest = tile / p.tiles_x;
        const int ty = rest % p.tiles_y, b = rest / p.tiles_y;
        const int h0 = ty * p.th, w0 = tx * p.tw;
        unsigned dm = 0, xm = 0;
#pragma unroll
        for (int i = 0; i < DY_PER_THREAD; ++i) {
            const int item = tid + i * 256;
            const int m = item / (COUT / 8), s = item - m * (COUT / 8);
            const int rc = prc[m];
            const int h = h0 + (rc >> 16), w = w0 + (rc & 0xffff);
            const bool ok = (rc >= 0) & (h < p.H) & (w < p.W);
            dm |= (unsigned)ok << i;
            const size_t off = ok ? (((size_t)b * p.H + h) * p.W + w) * p.M + mb + s * 8 : 0;
            dr[S][i] = *reinterpret_cast<const uint4*>((BNB ? p.bda : p.dy) + off);
            if constexpr (BNB) yr[S][i] = *reinterpret_cast<const uint4*>(p.by + off);
        }
#pragma unroll
        for (int i = 0; i < HPT; ++i) {
            const int g = hgeo[i];
            const int h = h0 - 1 + (g >> 16), w = w0 - 1 + (g & 0xffff);
            const bool ok = (g >= 0) & hc.cok & (h >= 0) & (w >= 0) & (h < p.H) & (w < p.W);
            xm |= (unsigned)ok << i;
            xr[S][i] = halo_load(hc, ok, b, p.H, p.W, h, w);
        }
        dmask[S] = dm;
        xmask[S] = xm;
    };
    auto store_tile = [&](auto S) __attribute__((always_inline)) {
        float ksc[BNB ? 8 : 1], ksh[BNB ? 8 : 1], kB[BNB ? 8 : 1], kC[BNB ? 8 : 1];
        if constexpr (BNB) {  // the thread's dy piece is fixed: channels 8 * (tid % (COUT / 8)) + 0..7
            const int c8 = (tid % (COUT / 8)) * 8;
#pragma unroll
            for (int h = 0; h < 8; h += 4) {
                *reinterpret_cast<float4*>(ksc + h) = *reinterpret_cast<const float4*>(kbn + c8 + h);
                *reinterpret_cast<float4*>(ksh + h) = *reinterpret_cast<const float4*>(kbn + COUT + c8 + h);
                *reinterpret_cast<float4*>(kB + h) = *reinterpret_cast<const float4*>(kbn + 2 * COUT + c8 + h);
                *reinterpret_cast<float4*>(kC + h) = *reinterpret_cast<const float4*>(kbn + 3 * COUT + c8 + h);
            }
        }
#pragma unroll
        for (int i = 0; i < DY_PER_THREAD; ++i) {
            const int item = tid + i * 256;
            const int m = item / (COUT / 8), s = item - m * (COUT / 8);
            uint4 v = dr[S][i];
            if constexpr (BNB) v = bn_bwd_pk(v, yr[S][i], ksc, ksh, kB, kC);
            *reinterpret_cast<uint4*>(dys + m * DY_LD + s * 8) = ((dmask[S] >> i) & 1u) ? v : make_uint4(0, 0, 0, 0);
        }
#pragma unroll
        for (int i = 0; i < HPT; ++i) {  // every piece lands inside the HMAX-pixel region
            const int item = tid + i * 256;
            if constexpr (X8) {
                if (item < HMAX)
                    *reinterpret_cast<uint4*>(hxs + item * XW_LD) = halo_finish_pk(hc, (xmask[S] >> i) & 1u, xr[S][i]);
            } else {
                *reinterpret_cast<uint4*>(hxs + wg_pixel(item) * XW_LD + wg_piece(item) * 8) =
                    halo_finish_pk(hc, (xmask[S] >> i) & 1u, xr[S][i]);
            }
        }
    };
    constexpr std::integral_constant<int, 0> S0{};
    constexpr std::integral_constant<int, 1> S1{};

    // per-lane transposed-read geometry: 16-lane group g, lane 4q+pp of it supplies row q, cols 4pp..4pp+3;
    // the K (pixel) order inside a 32-pixel k-step is permuted consistently for A and B
    const int g = lane >> 4, q = (lane & 15) >> 2, pp = lane & 3;
    const int pc = 16 * (g >> 1) + 4 * (g & 1) + q;  // pixel within the k-step (0..23), +8 for the 2nd read

    auto kstep = [&](int ks) __attribute__((always_inline)) {
        const int m = ks * 32 + pc;
        bf16x8 af[RM];
#pragma unroll
        for (int i = 0; i < RM; ++i) {
            const __bf16* a0 = dys + m * DY_LD + co0 + i * 16 + 4 * pp;
            af[i] = tr_pair(a0, a0 + 8 * DY_LD);
        }
        const __bf16* x0 = hxs + hoff[m] * XW_LD + ci0 + 4 * pp;
        const __bf16* x1 = hxs + hoff[m + 8] * XW_LD + ci0 + 4 * pp;
#pragma unroll
        for (int tap = 0; tap < 9; ++tap) {
            const int toff = ((tap / 3) * p.hw + tap % 3) * XW_LD;
            const bf16x8 bf = tr_pair(x0 + toff, x1 + toff);
#pragma unroll
            for (int i = 0; i < RM; ++i)
                acc[tap][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bf, acc[tap][i], 0, 0, 0);
        }
    };
    auto compute = [&]() __attribute__((always_inline)) {
        if constexpr (COUT == 32) {
            // two k-steps per iteration: the next step's hoff / fragment reads overlap this one's MFMAs
            int ks = 0;
#pragma unroll 1
            for (; ks + 1 < ksteps; ks += 2) {
                kstep(ks);
                kstep(ks + 1);
            }
            if (ks < ksteps) kstep(ks);
        } else {
#pragma unroll 1
            for (int ks = 0; ks < ksteps; ++ks) kstep(ks);
        }
    };
    if constexpr (WS == 2) {
        // M = 32 (full-resolution layers, HBM-bound): two tiles in flight, unrolled by two so the
        // register-set index is static
        auto step = [&](auto S, int tile) __attribute__((always_inline)) {
            store_tile(S);
            __syncthreads();
            if (tile + 2 < t_end) load_tile(S, tile + 2);
            compute();
            __syncthreads();
        };
        if (t_begin < t_end) load_tile(S0, t_begin);
        if (t_begin + 1 < t_end) load_tile(S1, t_begin + 1);
        for (int tile = t_begin; tile < t_end; tile += 2) {
            step(S0, tile);
            if (tile + 1 >= t_end) break;
            step(S1, tile + 1);
        }
    } else {
        // M % 64: one tile in flight (a second register set would halve the waves per SIMD)
        if (t_begin < t_end) load_tile(S0, t_begin);
        for (int tile = t_begin; tile < t_end; ++tile) {
            if (!(WG_EXP & 4)) store_tile(S0);
            __syncthreads();
            if (!(WG_EXP & 2) && tile + 1 < t_end) load_tile(S0, tile + 1);
            if (!(WG_EXP & 1)) compute();
            __syncthreads();
        }
    }

    // slab[z][co][tap*ctot + cc*32 + ci]   (C layout 16x16: row = 4*(lane>>4) + r, col = lane&15)
    float* slab = p.slab + (size_t)split * p.M * p.N;
    const int ci = cc * CK + ci0 + (lane & 15);
    if (ci < p.x.ctot) {
#pragma unroll
        for (int tap = 0; tap < 9; ++tap)
#pragma unroll
            for (int i = 0; i < RM; ++i)
#pragma unroll
                for (int r = 0; r < 4; ++r) {
                    const int co = mb + co0 + i * 16 + 4 * (lane >> 4) + r;
                    slab[(size_t)co * p.N + tap * p.x.ctot + ci] = acc[tap][i][r];
                }
    }
}


// =====================================================================================
// wgrad, warp-specialised: M = 32 or M % 64 == 0, x channels % 32 == 0 (every 3x3 wgrad but enc1.0)
// =====================================================================================
// One 512-thread block per CU. A block owns COUT dy channels (rows of dW) x CIB x channels x 9 taps
// and a range of 128-pixel tiles (split-K). Waves 4-7 stage tile t+1 (the dy rows, and the x halo
// through BN+ReLU) into one LDS buffer while waves 0-3 run tile t's MFMAs from the other, one
// barrier per tile: the one-role-per-wave layout of k_halo_conv. (k_halo_wgrad interleaves both
// roles in every wave at 2 blocks per CU; timing runs with either role removed measured its MFMA
// phase alone at 74 us of 136 us for 120x160x64x64: the staging was not hidden.)
// MFMA waves: CIB/16 x-channel groups of 16 x 4/(CIB/16) dy-channel groups; a wave owns RM 16-row
// dy tiles x 16 x channels x 9 taps of v_mfma_f32_16x16x32_bf16 accumulators (RM = 4 at 64 x 64:
// 144 registers, 26 fragment reads per 36 MFMAs per k-step). The 4 k-steps x 9 taps of a tile run as
// one straight-line stream of tap-steps with the fragment reads WS_PD tap-steps ahead in a register ring.
// The halo is laid out with a fixed row pitch of HP pixels, so the 9 tap offsets of a fragment read
// are compile-time immediates: no address arithmetic per tap-step (a runtime pitch cost 4 VALU per 4
// MFMAs, half the issue slots the 16x16x32 MFMAs leave free). Two layouts, so the staged halo slots
// (each one is BN+ReLU-transformed by the loaders, whose VALU shares the SIMDs with the MFMA waves and
// paces the kernel) stay close to the real halo: HP 34 x 6 rows for 4 x 32 tiles (204 slots), HP 22 x 8
// rows for tiles up to 6 x 20 (176 slots).
constexpr int WS_TPX = 128;                     // pixels per tile (4 k-steps)
// dy tiles by LDS-DMA in the plain (no BatchNorm-backward, single-source-block) instances; WS_DYDMA=0 builds: registers
#ifndef WS_DYDMA
#define WS_DYDMA 1
#endif
constexpr int WS_PD = 5;                        // tap-steps of fragment read-ahead
#ifndef WS_PRIO
// loader waves at s_setprio 1: they run the BN+ReLU (and BatchNorm-backward) transforms and, as the workgroup's younger
// half, otherwise lose issue arbitration to the MFMA waves (tools/conv_micro.py --wgrad: 240x320 M=32 x32 187 -> 158 us,
// 120x160 M=64 x32 57 -> 53 us, the other shapes 1-3 % faster)
#define WS_PRIO 1
#endif
// cache policy of the fused BatchNorm-backward dy stores (nontemporal, as the conv epilogue's HC_ST_AUX)
#ifndef WS_ST_AUX
#define WS_ST_AUX 2
#endif

// blocks per CU: two for the 32 x 32-channel configuration (72 KB of LDS, <= 128 registers), whose
// tiles carry little MFMA work and need more loads in flight; one otherwise
__host__ __device__ constexpr int ws_blocks_per_cu(int cout, int cib) { return cout == 32 && cib == 32 ? 2 : 1; }

// MFMA waves of the MF32 instances (64 dy x 64 x channels per block): v_mfma_f32_32x32x16_bf16, k = 16 pixels.
// The block's output is 4 quadrants (co half, ci half) of 32 x 32 x 9 taps; wave W owns every quadrant of taps W and
// W + 4 and quadrant W of tap 8 (co half W >> 1, ci half W & 1): 9 accumulators of 16 registers, as the 16x16x32 form's
// 36 of 4. Per 16-pixel k-step a wave reads 2 dy fragments (both co halves, shared by its 9 MFMAs) and 5 x fragments
// (taps W, W + 4 x both ci halves, tap 8 x its half): 7 transposed pairs per 9 MFMAs of 32 cycles, against the 16x16x32
// form's 13 pairs per 36 MFMAs of 16 cycles — the same LDS reads per tile, with a third of the MFMA instructions, so
// the matrix pipe holds the SIMD's issue for 8 of every 32 cycles instead of 8 of 16 and the loader wave on the same
// SIMD (BN+ReLU of the halo) gets the rest. The wave's taps are template constants, so every fragment address is a
// per-(k-step, pixel-half) lane base plus an immediate. Fragments (tr_pair, as k_bwd_fused32): 16-lane group g holds
// channels 16 (g & 1) + (lane & 15) of pixels 4 (g >> 1) + {0..3, 8..11} of the k-step. The slab layout is the 16x16
// form's: slab[split][co][tap * ctot + cc * 64 + ci].
template <int HP, int DLD, int XLD, int DY_E, int BUF, int W>
__device__ __forceinline__ void ws_mfma32_tiles(const HWgArgs& p, const __bf16* smem, int lane, int cc, int mb,
                                                int split, int ntile, const unsigned (&xoff)[WS_TPX / 16][2],
                                                unsigned aoff) {
    constexpr int KS = WS_TPX / 16;
    constexpr int T0 = W, T1 = W + 4, C8 = W >> 1, I8 = W & 1;
    constexpr int TO0 = ((T0 / 3) * HP + T0 % 3) * XLD * 2, TO1 = ((T1 / 3) * HP + T1 % 3) * XLD * 2;
    constexpr int TO8 = (2 * HP + 2) * XLD * 2 + I8 * 64;  // bytes
    f32x16 acc[9];
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[t][r] = 0.f;
    const char* lds = reinterpret_cast<const char*>(smem);
    // Fragment reads run PD MFMA steps (step = ks * 9 + k) ahead of their first use: the k-step's two dy fragments and
    // its two halo bases at k = 0 (two sets, by k-step parity), the x fragments at k = 0, 2, 4, 6, 8 into a ring of NB
    // (a slot is rewritten 9 - PD > 1 steps after its first use, past its second)
    constexpr int PD = 6, NB = 5;
    for (int it = 0; it < ntile; ++it) {
        __syncthreads();  // tile it is in buffer it & 1 (and the loaders may overwrite the other one)
        const unsigned bufb = (unsigned)((it & 1) * BUF * 2);
        unsigned abase = aoff + bufb, xbase = bufb + (unsigned)(DY_E * 2);
        asm volatile("" : "+v"(abase), "+s"(xbase));
        bf16x8 fa[2][2], fb[NB];
        unsigned xc[2][2];
        auto xfrag = [&](int ks, int off) __attribute__((always_inline)) {
            return tr_pair(reinterpret_cast<const __bf16*>(lds + xc[ks & 1][0] + off),
                           reinterpret_cast<const __bf16*>(lds + xc[ks & 1][1] + off));
        };
        // the reads first needed by step j
        auto rd = [&](int j) __attribute__((always_inline)) {
            const int ks = j / 9, k = j - ks * 9, s = ks & 1, b = ks * 5 + k / 2;
            if (k == 0) {
#pragma unroll
                for (int h = 0; h < 2; ++h) {
                    const __bf16* a0 = reinterpret_cast<const __bf16*>(lds + abase) + ks * 16 * DLD + h * 32;
                    fa[s][h] = tr_pair(a0, a0 + 8 * DLD);
                    xc[s][h] = xoff[ks][h] + xbase;
                }
                fb[b % NB] = xfrag(ks, TO0);
            } else if (k == 2) {
                fb[b % NB] = xfrag(ks, TO0 + 64);
            } else if (k == 4) {
                fb[b % NB] = xfrag(ks, TO1);
            } else if (k == 6) {
                fb[b % NB] = xfrag(ks, TO1 + 64);
            } else if (k == 8) {
                fb[b % NB] = xfrag(ks, TO8);
            }
        };
        // step k: acc[k] = (tap T0 for k < 4, T1 for k < 8; co half k & 1, ci half (k >> 1) & 1), acc[8] = tap 8
        auto mf = [&](int j) __attribute__((always_inline)) {
            const int ks = j / 9, k = j - ks * 9, s = ks & 1, b = ks * 5 + k / 2;
            if (k < 8) acc[k] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[s][k & 1], fb[b % NB], acc[k], 0, 0, 0);
            else acc[8] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(fa[s][C8], fb[b % NB], acc[8], 0, 0, 0);
        };
#pragma unroll
        for (int j = 0; j < PD; ++j) rd(j);
#pragma unroll
        for (int j = 0; j < KS * 9; ++j) {
            if (j + PD < KS * 9) rd(j + PD);
            __builtin_amdgcn_sched_barrier(0);
            mf(j);
            __builtin_amdgcn_sched_barrier(0);
        }
    }
    if (ntile & 1) __syncthreads();  // the loaders' last (even-count) iteration
    // slab[split][co][tap*ctot + cc*64 + ci]   (32x32 C layout: element i of lane l is row 8 (i / 4) + 4 (l / 32) + i % 4,
    // column l % 32)
    float* slab = p.slab + (size_t)split * p.M * p.N;
    const int ctot = p.x.ctot;
#pragma unroll
    for (int a = 0; a < 9; ++a) {
        const int tap = a < 4 ? T0 : (a < 8 ? T1 : 8);
        const int coh = a < 8 ? (a & 1) : C8, cih = a < 8 ? ((a >> 1) & 1) : I8;
        const int ci = cc * 64 + cih * 32 + (lane & 31);
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            const int co = mb + coh * 32 + 8 * (i / 4) + 4 * (lane >> 5) + i % 4;
            slab[(size_t)co * p.N + tap * ctot + ci] = acc[a][i];
        }
    }
}

template <int HP, int DLD, int XLD, int DY_E, int BUF>
__device__ __forceinline__ void ws_mfma32(const HWgArgs& p, const __bf16* smem, int lane, int wid, int cc, int mb,
                                          int split, int ntile, int mvalid) {
    constexpr int KS = WS_TPX / 16;
    const int g = lane >> 4, q4 = (lane & 15) >> 2, pp = lane & 3;
    const int pk = 4 * (g >> 1) + q4, ch16 = 16 * (g & 1) + 4 * pp;
    // byte offsets (within the halo region) of this lane's two halo pixels of each k-step at tap (0, 0)
    unsigned xoff[KS][2];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int m = ks * 16 + pk + 8 * h;
            const int hm = m / p.tw;
            const int px = m < mvalid ? hm * HP + (m - hm * p.tw) : 0;  // dy is 0 past the tile
            xoff[ks][h] = (unsigned)(px * XLD + ch16) * 2u;
        }
    const unsigned aoff = (unsigned)(pk * DLD + ch16) * 2u;
    switch (__builtin_amdgcn_readfirstlane(wid)) {
    case 0: ws_mfma32_tiles<HP, DLD, XLD, DY_E, BUF, 0>(p, smem, lane, cc, mb, split, ntile, xoff, aoff); break;
    case 1: ws_mfma32_tiles<HP, DLD, XLD, DY_E, BUF, 1>(p, smem, lane, cc, mb, split, ntile, xoff, aoff); break;
    case 2: ws_mfma32_tiles<HP, DLD, XLD, DY_E, BUF, 2>(p, smem, lane, cc, mb, split, ntile, xoff, aoff); break;
    default: ws_mfma32_tiles<HP, DLD, XLD, DY_E, BUF, 3>(p, smem, lane, cc, mb, split, ntile, xoff, aoff); break;
    }
}

// MF32 (64 x 64 blocks only): the MFMA waves run v_mfma_f32_32x32x16_bf16 instead of 16x16x32 (see the MF32 branch
// of the MFMA waves); its fragments read 4 pixels x 32 channels per 32-lane group, so the rows are 96 elements
// (48 dwords: 4 consecutive pixels fall on distinct 16-bank quarters)
template <int COUT, int CIB, int HP, int HR, bool BNB, bool SPAN, bool MF32 = false>  // dy / x channels per block;
                                                       // halo pitch and rows (tw+2 <= HP, th+2 <= HR); BNB:
                                                       // BatchNorm-backward apply in the dy staging; SPAN: a block's x
                                                       // channels may straddle the two sources of a concatenation
__global__ __launch_bounds__(512, 2 * ws_blocks_per_cu(COUT, CIB)) void k_halo_wgrad_ws(const HWgArgs p) {
    constexpr int KS = WS_TPX / 32;
    constexpr int NCI = CIB / 16, NCO = 4 / NCI, RM = COUT / 16 / NCO;  // wave grid and 16-row tiles per wave
    constexpr int DPP = COUT / 8, XPP = CIB / 8;                       // 16-B pieces per pixel (dy, x)
    constexpr int PAD = MF32 ? 32 : 16;
    constexpr int DLD = COUT + PAD, XLD = CIB + PAD;                   // 96 / 160-B rows: conflict-free tr reads
    constexpr int DYP = WS_TPX * DPP / 256;                            // dy pieces per loader thread
    constexpr int HXP = (HP * HR * XPP + 255) / 256;                   // halo pieces per loader thread
    constexpr int DY_E = WS_TPX * DLD, BUF = DY_E + HXP * (256 / XPP) * XLD;  // elements per LDS buffer
    static_assert(RM >= 1 && NCI * NCO == 4, "wave grid");
    static_assert(!MF32 || (COUT == 64 && CIB == 64 && !SPAN), "MF32: 64 x 64 blocks");
    static_assert(2 * BUF * 2 <= 160 * 1024, "LDS");
    __shared__ __attribute__((aligned(16))) __bf16 smem[2 * BUF];

    const int tid = threadIdx.x, lane = tid & 63;
    const bool is_loader = tid >= 256;
    const int wid = (tid >> 6) & 3;
    int cc = blockIdx.x, zb = blockIdx.z, split = blockIdx.y;
    if (p.xcd) {  // XCD-contiguous numbering, as in k_halo_wgrad
        const int G = gridDim.x * gridDim.y * gridDim.z;
        const int L = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
        const int lg = (L & 7) * (G >> 3) + (L >> 3);
        cc = lg % gridDim.x;
        const int r = lg / gridDim.x;
        zb = r % gridDim.z;
        split = r / gridDim.z;
    }
    const int mb = zb * COUT;
    const int t_begin = split * p.tiles_per_split;
    const int ntile = max(0, min(p.ntiles, t_begin + p.tiles_per_split) - t_begin);
    const int mvalid = p.th * p.tw;

    if (is_loader) {
        // =========================================================== loader waves
        // not for the 128 dy x 32 x blocks: their loaders transform half the x halo per tile, and at equal priority the
        // MFMA waves issue first (tools/conv_micro.py --wgrad-step, two rounds: 2-5 % faster at every such shape)
        constexpr int prio = (COUT == 128 && !BNB) ? 0 : WS_PRIO;
        if (prio) __builtin_amdgcn_s_setprio(prio);
        // item = ltid + 256 i -> (pixel item / P, 16-B piece ltid % P) for P pieces per pixel: the piece is
        // fixed per thread; an 8-lane ds_write_b128 group covers one pixel's 8 pieces at the 10-slot row
        // stride (64 channels: conflict-free) or two pixels' 4 at the 6-slot stride
        const int ltid = tid - 256;
        const int dpiece = ltid % DPP, dpix0 = ltid / DPP, xpiece = ltid % XPP, xpix0 = ltid / XPP;
        unsigned dyrc[(DYP + 1) / 2], hgeo[(HXP + 1) / 2];  // (row << 8 | col), 0xffff past the tile / halo
#pragma unroll
        for (int i = 0; i < DYP; i += 2) {
            unsigned e[2];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int m = dpix0 + (256 / DPP) * (i + h);
                const int hm = m / p.tw;
                e[h] = (i + h < DYP && m < mvalid) ? (unsigned)(hm << 8 | (m - hm * p.tw)) : 0xffffu;
            }
            dyrc[i / 2] = e[0] | e[1] << 16;
        }
#pragma unroll
        for (int i = 0; i < HXP; i += 2) {
            unsigned e[2];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int px = xpix0 + (256 / XPP) * (i + h);
                const int hy = px / HP, hx = px - hy * HP;
                e[h] = (i + h < HXP && hy < p.th + 2 && hx < p.hw) ? (unsigned)(hy << 8 | hx) : 0xffffu;
            }
            hgeo[i / 2] = e[0] | e[1] << 16;
        }
        // this thread's 8 x channels (fixed piece): their BN affine (slab: any valid address), channel stride and
        // offset. The buffer resource stays block-uniform (the source of the block's first channel): a per-lane
        // base made hipcc wrap every halo load in a waterfall loop (+8 % on every instance). SPAN (dec1.0: 32 + 32
        // in one 64-channel block, whose dy transform then runs once instead of once per 32-channel block): each
        // lane loads through the resource of its own source, with the other source's load out of range
        const HaloCol hc = halo_col(p.x, cc * CIB + xpiece * 8, p.slab);
        const bool bsrc1 = cc * CIB >= p.x.c0;
        const __bf16* xsrc = bsrc1 ? p.x.p1 : p.x.p0;
        const int xC = SPAN ? hc.C : (bsrc1 ? p.x.c1 : p.x.c0);  // per lane only with SPAN (offsets, not resources)
        const bool lsrc1 = SPAN && cc * CIB + xpiece * 8 >= p.x.c0;
        // Per-piece element offsets from the tile origin (h0, w0), fixed for the launch: a piece's buffer
        // offset is then one add, its bounds test four compares against per-tile scalars, and a piece
        // outside the image / tile gets an offset past the buffer's range, which the buffer load returns
        // as zeros without touching memory (loads of a fixed dummy address made every CU hit one line)
        int dpo[DYP], xpo[HXP];
#pragma unroll
        for (int i = 0; i < DYP; ++i) {
            const unsigned rc = (dyrc[i / 2] >> (16 * (i & 1))) & 0xffffu;
            dpo[i] = ((int)(rc >> 8) * p.W + (int)(rc & 0xff)) * p.M + mb + dpiece * 8;
        }
#pragma unroll
        for (int i = 0; i < HXP; ++i) {
            const unsigned gg = (hgeo[i / 2] >> (16 * (i & 1))) & 0xffffu;
            xpo[i] = (((int)(gg >> 8) - 1) * p.W + (int)(gg & 0xff) - 1) * xC + hc.c;
        }
        // DYDMA (the plain instances: dy is a raw tensor): the dy tile goes global -> LDS by LDS-DMA. The tile image
        // is WS_TPX rows of DLD elements (DPP data pieces + 2 pad slots), contiguous, so wave-instruction k fills
        // slots 64k .. 64k + 63; a lane's slot is (pixel s / RS, piece s % RS), pad slots and pixels past the tile or
        // the image load out of range (zeros). Issued after the iteration's halo stores into buffer i & 1, waited for
        // by a counted vmcnt before the barrier (the x loads issued after it stay in flight); hipcc's own counted
        // waits only grow stricter (it does not see the asm loads). Replaces DYP loads + DYP ds_write_b128 per thread.
        constexpr bool DYDMA = WS_DYDMA && !BNB && !SPAN && (DLD * 2) % 16 == 0;
        constexpr int RS = DLD / 8;                             // 16-B slots per tile row
        constexpr int NDI = (WS_TPX * RS + 63) / 64;            // wave-instructions per tile
        constexpr int DDI = DYDMA ? (NDI + 3) / 4 : 1;          // per loader wave
        const int lw = __builtin_amdgcn_readfirstlane(wid);
        int ddo[DDI];        // element offset from the tile origin in its image, or -1 (pad / past the tile)
        unsigned ddrc[DDI];  // (row << 8 | col) of the slot's pixel
        if constexpr (DYDMA) {
#pragma unroll
            for (int j = 0; j < DDI; ++j) {
                const int k = lw * DDI + j, sl = k * 64 + lane;
                const int m = sl / RS, pc = sl - m * RS;
                const int hm = m / p.tw, wm = m - hm * p.tw;
                const bool ok = k < NDI && pc < DPP && m < mvalid && m < WS_TPX;
                ddo[j] = ok ? (hm * p.W + wm) * p.M + mb + pc * 8 : -1;
                ddrc[j] = ok ? (unsigned)(hm << 8 | wm) : 0xffffu;
            }
        }
        const unsigned lds_dy0 = (unsigned)(uintptr_t)smem + (unsigned)(lw * DDI) * 1024u;
        // BNB: this thread's 8 dy channels (fixed piece) -> the folded BatchNorm-backward constants
        constexpr int NK = BNB ? 8 : 1;
        float ksc[NK], ksh[NK], kB[NK], kC[NK];
        if constexpr (BNB) {
            const int c = mb + dpiece * 8;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const float k1 = p.bcoef[3 * (c + j) + 1], k2 = p.bcoef[3 * (c + j) + 2];
                const float is = p.bis[c + j], sc = p.bsc[c + j], sh = p.bsh[c + j];
                ksc[j] = sc;
                ksh[j] = sh;
                kB[j] = -is * k2;
                kC[j] = is * k2 * sh + sc * (p.bmu[c + j] * is * k2 - k1);
            }
        }
        constexpr int DYY = BNB ? DYP : 1;
        constexpr unsigned OOB = 0x80000000u;
        struct TSet {
            uint4 d[DYP], x[HXP];
            unsigned xm;   // bit i: halo piece i inside the image; BNB: bit 16 + i: dy piece i inside the tile
            uint4 y[DYY];  // BNB: the raw y pieces beside da in d
            int dbase;     // BNB: element offset of the tile origin in its image
            int img;       // BNB: the tile's image
            bool wr;       // BNB: this block writes the tile's dy
        };
        TSet sa, sb;
        auto load = [&](TSet& q, int tile) __attribute__((always_inline)) {
            if (WG_EXP & 256) return;
            const int tx = tile % p.tiles_x;
            const int rest = tile / p.tiles_x;
            const int ty = rest % p.tiles_y, b = rest / p.tiles_y;
            const int h0 = ty * p.th, w0 = tx * p.tw;
            const size_t img = (size_t)b * p.H * p.W;
            const int tpx = h0 * p.W + w0;
            const int nimg = p.H * p.W;
            const __amdgpu_buffer_rsrc_t rdy = __builtin_amdgcn_make_buffer_rsrc(
                (void*)((BNB ? p.bda : p.dy) + img * p.M), (short)0, nimg * p.M * 2, 0x00020000);
            const __amdgpu_buffer_rsrc_t ryr = __builtin_amdgcn_make_buffer_rsrc(
                (void*)((BNB ? p.by : p.dy) + img * p.M), (short)0, BNB ? nimg * p.M * 2 : 0, 0x00020000);
            if constexpr (BNB) {
                q.img = b;
                q.wr = tile % p.ncc == cc;
            }
            const int bxC = bsrc1 ? p.x.c1 : p.x.c0;
            const __amdgpu_buffer_rsrc_t rx =
                __builtin_amdgcn_make_buffer_rsrc((void*)(xsrc + img * bxC), (short)0, nimg * bxC * 2, 0x00020000);
            const __amdgpu_buffer_rsrc_t rx1 = __builtin_amdgcn_make_buffer_rsrc(  // SPAN: source 1 (dual-source calls)
                (void*)(SPAN ? p.x.p1 + img * p.x.c1 : xsrc), (short)0, SPAN ? nimg * p.x.c1 * 2 : 0, 0x00020000);
            // halo piece (hy, hx) is inside the image iff 1 - h0 <= hy < H - h0 + 1 and 1 - w0 <= hx < W - w0 + 1
            int rlo = 1 - h0, rhi = p.H - h0 + 1, clo = 1 - w0, chi = p.W - w0 + 1;
            if (tile >= t_begin + ntile) rhi = rlo;  // past the block's range: every piece out of range, no traffic
            const int dbase = tpx * p.M, xbase = tpx * xC;
            unsigned xm = 0;
#pragma unroll
            for (int i = 0; i < (DYDMA ? 0 : DYP); ++i) {
                const unsigned rc = (dyrc[i / 2] >> (16 * (i & 1))) & 0xffffu;
                const bool ok = (rc != 0xffffu) & ((int)(rc >> 8) < rhi - 1) & ((int)(rc & 0xff) < chi - 1) & (rhi > rlo);
                const unsigned off = ok ? (unsigned)(dbase + dpo[i]) * 2u : OOB;
                const auto v = __builtin_amdgcn_raw_buffer_load_b128(rdy, off, 0, 0);
                q.d[i] = make_uint4(v[0], v[1], v[2], v[3]);
                if constexpr (BNB) {
                    if (WG_EXP & 2097152) {  // timing experiment: no y loads
                        q.y[i] = q.d[i];
                        xm |= (unsigned)ok << (16 + i);
                        continue;
                    }
                    const auto u = __builtin_amdgcn_raw_buffer_load_b128(ryr, off, 0, 0);
                    q.y[i] = make_uint4(u[0], u[1], u[2], u[3]);
                    xm |= (unsigned)ok << (16 + i);
                }
            }
            if constexpr (BNB) q.dbase = dbase;
#pragma unroll
            for (int i = 0; i < HXP; ++i) {
                const unsigned gg = (hgeo[i / 2] >> (16 * (i & 1))) & 0xffffu;
                const int hy = (int)(gg >> 8), hx = (int)(gg & 0xff);
                const bool ok = (gg != 0xffffu) & (hy >= rlo) & (hy < rhi) & (hx >= clo) & (hx < chi);
                xm |= (unsigned)ok << i;
                const unsigned off = ok ? (unsigned)(xbase + xpo[i]) * 2u : 0x80000000u;
                if constexpr (SPAN) {
                    const auto v0 = __builtin_amdgcn_raw_buffer_load_b128(rx, lsrc1 ? OOB : off, 0, 0);
                    const auto v1 = __builtin_amdgcn_raw_buffer_load_b128(rx1, lsrc1 ? off : OOB, 0, 0);
                    q.x[i] = make_uint4(v0[0] | v1[0], v0[1] | v1[1], v0[2] | v1[2], v0[3] | v1[3]);
                } else {
                    const auto v = __builtin_amdgcn_raw_buffer_load_b128(rx, off, 0, 0);
                    q.x[i] = make_uint4(v[0], v[1], v[2], v[3]);
                }
            }
            q.xm = xm;
        };
        auto store = [&](TSet& q, int buf) __attribute__((always_inline)) {
            if (WG_EXP & (128 | 256)) return;
            __bf16* dys = smem + buf * BUF;
            __bf16* hxs = dys + DY_E;
            if constexpr (BNB) {
                // dy pieces outside the tile are zero (the raw pair loaded as zeros gives dy = C there); the
                // writer block also stores them (buffer stores: out-of-range pieces dropped, no branch)
                const __amdgpu_buffer_rsrc_t rdo = __builtin_amdgcn_make_buffer_rsrc(  // no dy destination: 0 records
                    (void*)(p.dy + (size_t)q.img * p.H * p.W * p.M), (short)0, p.dy ? p.H * p.W * p.M * 2 : 0, 0x00020000);
#pragma unroll
                for (int i = 0; i < DYP; ++i) {
                    const bool ok = (q.xm >> (16 + i)) & 1u;
                    uint4 v = (WG_EXP & 524288) ? q.d[i] : bn_bwd_pk(q.d[i], q.y[i], ksc, ksh, kB, kC);
                    v = ok ? v : make_uint4(0, 0, 0, 0);
                    *reinterpret_cast<uint4*>(dys + (dpix0 + (256 / DPP) * i) * DLD + dpiece * 8) = v;
                    __attribute__((ext_vector_type(4))) unsigned data = {v.x, v.y, v.z, v.w};
                    const unsigned off = (ok & q.wr) ? (unsigned)(q.dbase + dpo[i]) * 2u : OOB;
                    if (!(WG_EXP & 1048576)) __builtin_amdgcn_raw_buffer_store_b128(data, rdo, off, 0, WS_ST_AUX);
                }
            } else if constexpr (!DYDMA) {
#pragma unroll
                for (int i = 0; i < DYP; ++i)  // out-of-range pieces were loaded as zeros
                    *reinterpret_cast<uint4*>(dys + (dpix0 + (256 / DPP) * i) * DLD + dpiece * 8) = q.d[i];
            }
#pragma unroll
            for (int i = 0; i < HXP; ++i)
                *reinterpret_cast<uint4*>(hxs + (xpix0 + (256 / XPP) * i) * XLD + xpiece * 8) =
                    (WG_EXP & 2048) ? q.x[i] : halo_finish_pk(hc, (q.xm >> i) & 1u, q.x[i]);
        };
        // Iteration i stores tile i (set i & 1, loaded two iterations ago) into LDS buffer i & 1 and refills
        // the set with tile i + 2, then meets the MFMA waves at the barrier before their tile i: two tiles'
        // loads in flight. Every iteration issues the same loads and waits (past the block's range the
        // loads are out of range and fetch nothing), and the prologue issues what an iteration would have:
        // a load or a wait on only some paths makes the compiler's vmcnt bookkeeping drain every load
        constexpr bool DG = (WG_EXP & 1024) != 0;
        unsigned long long t_st = 0, t_ld = 0, t_br = 0, t0 = 0, t1 = 0, t_all = DG ? __builtin_amdgcn_s_memtime() : 0;
        // DYDMA: tile `tile`'s dy -> LDS buffer buf
        auto dma_dy = [&](int buf, int tile) __attribute__((always_inline)) {
            const int tx = tile % p.tiles_x;
            const int rest = tile / p.tiles_x;
            const int ty = rest % p.tiles_y, b = rest / p.tiles_y;
            const int h0 = ty * p.th, w0 = tx * p.tw;
            const int nimg = p.H * p.W;
            const __amdgpu_buffer_rsrc_t rdy = __builtin_amdgcn_make_buffer_rsrc(
                (void*)(p.dy + (size_t)b * nimg * p.M), (short)0, nimg * p.M * 2, 0x00020000);
            int rhi = p.H - h0, chi = p.W - w0;  // tile rows / columns inside the image
            if (tile >= t_begin + ntile) rhi = 0;  // past the block's range: nothing loaded
            const int dbase = (h0 * p.W + w0) * p.M;
            const unsigned m0b = __builtin_amdgcn_readfirstlane(lds_dy0 + (unsigned)(buf * BUF * 2));
#pragma unroll
            for (int j = 0; j < DDI; ++j) {
                if (NDI % 4 != 0 && lw * DDI + j >= NDI) break;  // wave-uniform
                const bool ok = (ddo[j] >= 0) & ((int)(ddrc[j] >> 8) < rhi) & ((int)(ddrc[j] & 0xffu) < chi);
                const unsigned off = ok ? (unsigned)(dbase + ddo[j]) * 2u : OOB;
                unsigned keep;
                asm volatile(
                    "s_mov_b32 %0, m0\n\t"
                    "s_mov_b32 m0, %2\n\t"
                    "s_nop 0\n\t"
                    "buffer_load_dwordx4 %1, %3, 0 offen lds\n\t"
                    "s_mov_b32 m0, %0"
                    : "=&s"(keep)
                    : "v"(off), "s"(m0b + (unsigned)j * 1024u), "s"(rdy)
                    : "memory");
            }
        };
        auto iter = [&](TSet& q, int buf, int tile) __attribute__((always_inline)) {
            if (DG) t0 = __builtin_amdgcn_s_memtime();
            store(q, buf);
            if (DG) { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); t1 = __builtin_amdgcn_s_memtime(); t_st += t1 - t0; }
            if constexpr (DYDMA) {
                __builtin_amdgcn_sched_barrier(0);
                dma_dy(buf, tile - 2);  // the tile this iteration stages (the set was loaded two iterations ago)
                __builtin_amdgcn_sched_barrier(0);
            }
            load(q, tile);
            if (DG) { t0 = t1; t1 = __builtin_amdgcn_s_memtime(); t_ld += t1 - t0; t0 = t1; }
            if constexpr (DYDMA) {  // this tile's dy landed; the x loads just issued stay in flight
                __builtin_amdgcn_sched_barrier(0);
                asm volatile("s_waitcnt vmcnt(%0)" ::"i"(HXP) : "memory");
            }
            __syncthreads();
            if (DG) t_br += __builtin_amdgcn_s_memtime() - t0;
        };
        load(sa, t_begin);
        __builtin_amdgcn_sched_barrier(0);  // issue order = an iteration's (the scheduler swapped the sets)
        load(sb, t_begin + 1);
        // an even number of iterations (no exit between the two sets: the compiler's vmcnt bookkeeping then
        // treats both alike); an odd count's last one stores a tile past the range into the buffer the MFMA
        // waves no longer read, and they meet it with one extra barrier
        for (int i = 0; i < ntile; i += 2) {
            iter(sa, 0, t_begin + i + 2);
            iter(sb, 1, t_begin + i + 3);
        }
        if (DG && p.dbg && lane == 0) {
            unsigned long long* d = p.dbg + ((size_t)(blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z)) * 8 + 4 + wid) * 4;
            d[0] = t_st;
            d[1] = t_ld;
            d[2] = t_br;
            d[3] = __builtin_amdgcn_s_memtime() - t_all;
        }
        return;
    }

    // =============================================================== MFMA waves
    if constexpr (MF32) {
        ws_mfma32<HP, DLD, XLD, DY_E, BUF>(p, smem, lane, wid, cc, mb, split, ntile, mvalid);
        return;
    }
    const int g = lane >> 4, q = (lane & 15) >> 2, pp = lane & 3;
    const int pc = 16 * (g >> 1) + 4 * (g & 1) + q;  // pixel within the k-step (0..23), +8 for the 2nd read
    const int ci0 = 16 * (wid % NCI), co0 = (wid / NCI) * (COUT / NCO);
    // byte offsets (within the halo region) of this lane's two halo rows of each k-step at tap (0,0)
    unsigned xoff[KS][2];
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
            const int m = ks * 32 + pc + 8 * h;
            const int hm = m / p.tw;
            const int px = m < mvalid ? hm * HP + (m - hm * p.tw) : 0;  // dy is 0 past the tile
            xoff[ks][h] = (unsigned)(px * XLD + ci0 + 4 * pp) * 2u;
        }
    f32x4 acc[9][RM];
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
        for (int i = 0; i < RM; ++i) acc[t][i] = f32x4{0.f, 0.f, 0.f, 0.f};

    constexpr int NSTEP = KS * 9;
    bf16x8 bring[WS_PD + 1];
    bf16x8 aring[2][RM];
    const char* lds = reinterpret_cast<const char*>(smem);
    constexpr bool DG = (WG_EXP & 1024) != 0;
    unsigned long long t_cp = 0, t_br = 0, t0 = 0, t_all = DG ? __builtin_amdgcn_s_memtime() : 0;
    for (int it = 0; it < ntile; ++it) {
        if (DG) t0 = __builtin_amdgcn_s_memtime();
        __syncthreads();  // tile it is in buffer it & 1 (and the loaders may overwrite the other one)
        if (DG) {
            const unsigned long long t1 = __builtin_amdgcn_s_memtime();
            t_br += t1 - t0;
            t0 = t1;
        }
        const unsigned bufb = (unsigned)((it & 1) * BUF * 2);  // byte offset of this buffer
        unsigned abase = bufb + (unsigned)(pc * DLD + co0 + 4 * pp) * 2u;
        asm volatile("" : "+v"(abase));
        unsigned xb[KS][2];  // this tile's read addresses; opaque so the compiler keeps them per tile
#pragma unroll
        for (int ks = 0; ks < KS; ++ks)
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                xb[ks][h] = xoff[ks][h] + bufb + (unsigned)(DY_E * 2);
                asm volatile("" : "+v"(xb[ks][h]));
            }
        auto issue = [&](int j) __attribute__((always_inline)) {
            const int ks = j / 9, tap = j - ks * 9;
            if (tap == 0) {
#pragma unroll
                for (int i = 0; i < RM; ++i) {
                    const __bf16* a0 = reinterpret_cast<const __bf16*>(lds + abase) + ks * 32 * DLD + i * 16;
                    aring[ks & 1][i] = tr_pair(a0, a0 + 8 * DLD);
                }
            }
            const int toff = ((tap / 3) * HP + tap % 3) * XLD;  // compile-time: folds into the ds offset
            bring[j % (WS_PD + 1)] = tr_pair(reinterpret_cast<const __bf16*>(lds + xb[ks][0]) + toff,
                                             reinterpret_cast<const __bf16*>(lds + xb[ks][1]) + toff);
        };
        if (!(WG_EXP & 64)) {
#pragma unroll
            for (int j = 0; j < WS_PD; ++j) issue(j);
#pragma unroll
            for (int j = 0; j < NSTEP; ++j) {
                if (j + WS_PD < NSTEP) issue(j + WS_PD);
                __builtin_amdgcn_sched_barrier(0);
                const int ks = j / 9, tap = j - ks * 9;
#pragma unroll
                for (int i = 0; i < RM; ++i)
                    acc[tap][i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(aring[ks & 1][i], bring[j % (WS_PD + 1)],
                                                                         acc[tap][i], 0, 0, 0);
                __builtin_amdgcn_sched_barrier(0);
            }
        }
        if (DG) t_cp += __builtin_amdgcn_s_memtime() - t0;
    }
    if (ntile & 1) __syncthreads();  // the loaders' last (even-count) iteration
    if (DG && p.dbg && lane == 0) {
        unsigned long long* d = p.dbg + ((size_t)(blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z)) * 8 + wid) * 4;
        d[0] = t_cp;
        d[1] = 0;
        d[2] = t_br;
        d[3] = __builtin_amdgcn_s_memtime() - t_all;
    }
    // slab[split][co][tap*ctot + cc*CIB + ci]   (C layout 16x16: row = 4*(lane>>4) + r, col = lane&15)
    float* slab = p.slab + (size_t)split * p.M * p.N;
    const int ci = cc * CIB + ci0 + (lane & 15);
#pragma unroll
    for (int tap = 0; tap < 9; ++tap)
#pragma unroll
        for (int i = 0; i < RM; ++i)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int co = mb + co0 + i * 16 + 4 * (lane >> 4) + r;
                slab[(size_t)co * p.N + tap * p.x.ctot + ci] = acc[tap][i][r];
            }
}

}  // namespace

// ---------------------------------------------------------------------- host side
// diagnostics: per-wave cycle counters of timing builds (WG_EXP & 1024) go to this device buffer
static unsigned long long* g_wg_dbg = nullptr;
extern "C" int sd_debug_buffer(void* p) {
    g_wg_dbg = (unsigned long long*)p;
    return 0;
}
unsigned long long* sd_debug_ptr() { return g_wg_dbg; }  // the fused backward's timing build (bwd_fused.hip)

bool sd_halo_fwd_shape(int N) { return N == 32 || N % 64 == 0; }
bool sd_halo_fwd_ok(const sd_src& a, int N, int epi) {
    return a.taps == 9 && !a.pool && sd_halo_fwd_shape(N) && epi != SD_EPI_PIXSHUF &&
           a.chans[0] + a.chans[1] <= SBN_MAX;
}

// XCD-contiguous block numbering in the halo kernels (SD_HALO_XCD=0: hardware order, for A/B runs)
static bool halo_xcd_enabled() {
    static const bool on = [] {
        const char* e = getenv("SD_HALO_XCD");
        return !(e && atoi(e) == 0);
    }();
    return on;
}

// k_halo_wgrad's 8-channel x layout (X8) for sources of at most 8 channels (SD_WG_X8=0: the 32-channel chunk layout,
// read per call: A/B runs, tests)
static bool wg_x8(int ctot) {
    const char* e = getenv("SD_WG_X8");
    if (e && *e && atoi(e) == 0) return false;
    return ctot > 0 && ctot <= 8;
}

// the all-LDS-DMA loaders for launches whose sources are all raw (SD_HALO_RAW=0: register-staged halos, A/B runs)
static bool halo_raw_enabled() {  // read per call (A/B modes within one process)
    const char* e = getenv("SD_HALO_RAW");
    return !(e && atoi(e) == 0);
}

// loader-wave priority where the loaders run the BN+ReLU transform (SD_HALO_PRIO=0/1/2 forces one, A/B runs)
static int halo_prio(const sd_src& a) {
    static const int env = [] {
        const char* e = getenv("SD_HALO_PRIO");
        return e ? atoi(e) : -1;
    }();
    if (env >= 0) return env;
    return (a.xform[0] == SD_BNRELU || (a.chans[1] > 0 && a.xform[1] == SD_BNRELU)) ? 2 : 0;
}

// Spatial tile of the forward/dgrad kernel: th x tw output pixels, RT 32-pixel column tiles per MFMA
// wave (th*tw <= 128*RT), CK-channel chunks.
struct HTile {
    int th, tw, rt, ck;
    int it = 1;  // items per pass (k_halo_conv IT)
};
// per-CU cycles of one chunk: the MFMA pipe of one SIMD vs the LDS (fragment reads at 4 cycles per
// ds_read_b128, staging stores at ~79 B/cycle: MI355X_MICROARCH.md LDS table)
static double halo_chunk_cycles(int th, int tw, int rt, int ck, int nt) {
    const int ks = 9 * ck / 16;
    const double mfma = (double)rt * nt * ks * 32;
    const double reads = 4.0 * ks * (rt + nt) * 4;
    const double stores = ((double)(th + 2) * (tw + 2) * ck * 2 + 32.0 * nt * 9 * ck * 2) / 79.0;
    return mfma > reads + stores ? mfma : reads + stores;
}
static HTile halo_tile(int H, int W, int N, bool stats) {
    const int nt = N == 32 ? 1 : 2;
    // CK = 32 (RT <= 3) measured faster than the CK = 16 / 512-pixel tiling at every N % 64 layer of
    // the 320x240 step (tools/conv_micro.py); SD_HALO_CK=16 selects the latter (tests, experiments)
    const char* env = getenv("SD_HALO_CK");
    const int ck = nt == 1 ? 32 : (env && atoi(env) == 16 ? 16 : 32);
    if (nt == 1 && W % 32 == 0 && H % 16 == 0) {
        // full-res N=32: 16x32 tiles (RT 4), also for the STATS epilogue since the r02 epilogue (no spill at
        // RT 4: dec1.0 fwd 313 -> 278 us, enc1.0 127 -> 109 us against 8x32); SD_HALO_N32=8/16 forces one
        const char* e32 = getenv("SD_HALO_N32");
        const int rows = e32 ? atoi(e32) : 16;
        (void)stats;
        return rows == 8 ? HTile{8, 32, 2, 32} : HTile{16, 32, 4, 32};
    }
    if (ck == 32) {  // 8x32, 6x40, a whole small image, rows of the image (<= 320 pixels, <= 384 halo)
        auto fits = [](int th, int tw) { return (th + 2) * (tw + 2) <= 384 && th * tw <= 320; };
        HTile t{8, 32, 2, 32};
        if (fits(H, W))
            t = {H, W, 0, 32};
        else if (W % 32 == 0)
            t = {8, 32, 0, 32};
        else if (W % 40 == 0)
            t = {6, 40, 0, 32};
        else if (W <= 256) {
            int th = 256 / W < 63 ? 256 / W : 63;
            while (th > 1 && !fits(th, W)) --th;
            if (fits(th, W)) t = {th, W, 0, 32};
        }
        t.rt = t.th * t.tw > 256 ? 3 : 2;
        return t;
    }
    // CK = 16: search tiles of <= 128*RT pixels (halo within the RT's LDS capacity) minimising the
    // modelled chunk cycles over the image; tw runs over the width, its divisors <= 128 and 32
    const int rt_max = 4;
    HTile best{8, 32, 2, 16};
    double best_cost = 1e300;
    for (int tw = 1; tw <= (W < 128 ? W : 128); ++tw) {
        if (tw != W && tw != 32 && W % tw) continue;
        for (int th = 1; th <= H && th < 64 && th * tw <= 128 * rt_max; ++th) {
            int rt = (th * tw + 127) / 128;
            if (rt < 2) rt = 2;
            while (rt <= rt_max && (th + 2) * (tw + 2) > halo_px_cap(rt, 16)) ++rt;
            if (rt > rt_max) continue;
            const double tiles = (double)cdiv(H, th) * cdiv(W, tw);
            const double cost = tiles * (halo_chunk_cycles(th, tw, rt, 16, nt) + 100.0);  // + epilogue share
            if (cost < best_cost) {
                best_cost = cost;
                best = {th, tw, rt, 16};
            }
        }
    }
    return best;
}

// persistent grid: nblk N-blocks x gper blocks each (gper = stats rows)
static void halo_grid(const HTile& t, int batch, int H, int W, int N, int& nblk, int& gper, int& nsp) {
    nblk = N == 32 ? 1 : N / 64;
    const long long sp = (long long)batch * cdiv(W, t.tw) * cdiv(H, t.th);
    nsp = sp > (1LL << 30) ? (1 << 30) : (int)sp;
    gper = PERSIST_BLOCKS / nblk;
    if (gper < 1) gper = 1;
    if (gper > nsp) gper = nsp;
}

// stats rows of the forward (STATS) launch
int sd_halo_fwd_rows(int batch, int H, int W, int N) {
    int nblk, gper, nsp;
    halo_grid(halo_tile(H, W, N, true), batch, H, W, N, nblk, gper, nsp);
    return gper;
}

// the tile plus its chunk width: 8-channel sources (the padded network input) with N = 32 take CK = 8
// chunks (5 k-steps per tile instead of 18 over 24 zero channels), same tiles (and stat rows)
// SD_HALO_IT=2: N % 64 layers with more than one 32-channel chunk run two items per pass at CK = 16 (each chunk's
// weights staged once for two halos)
static int halo_it_env() {
    static const int v = [] {
        const char* e = getenv("SD_HALO_IT");
        return e && atoi(e) == 2 ? 2 : 1;
    }();
    return v;
}
static HTile fwd_tile(int ctot, int H, int W, int N, bool stats) {
    HTile t = halo_tile(H, W, N, stats);
    if (ctot <= 8 && N == 32) t.ck = 8;
    if (halo_it_env() == 2 && N % 64 == 0 && t.ck == 32 && ctot > 32 && t.rt == 2 &&
        (t.th + 2) * (t.tw + 2) <= 384) {
        t.ck = 16;
        t.it = 2;
    }
    return t;
}

// partial rows of a STORE launch (sd_conv_gemm_bnsum): one per block of an N-block, like STATS
int sd_halo_store_rows(int batch, int H, int W, int N, int ctot) {
    int nblk, gper, nsp;
    halo_grid(fwd_tile(ctot, H, W, N, false), batch, H, W, N, nblk, gper, nsp);  // BNS launches
    return gper;
}
bool sd_halo_bnsum_ok(const sd_src& a, int N) {
    if (!sd_halo_fwd_ok(a, N, SD_EPI_STORE)) return false;
    const HTile t = fwd_tile(a.chans[0] + a.chans[1], a.H, a.W, N, false);
    return t.ck == 32 && t.it == 1 && !(N != 32 && t.rt == 3);
}

// weights resident in LDS for the whole launch (k_halo_conv WCONST): one or two chunks per item (SD_HALO_WC2=0: one
// only, A/B runs)
static bool wconst_chunks(int nchunks) {
    static const bool two = [] {
        const char* e = getenv("SD_HALO_WC2");
        return !(e && atoi(e) == 0);
    }();
    return nchunks == 1 || (two && nchunks == 2);
}

// the instance as rocprofv3 names it: k_halo_conv<NT, RT, CK, STATS, WCONST> (launch_halo's choice)
const char* sd_halo_fwd_name(int H, int W, int N, int epi, int c0, int c1, bool bns, bool wsplit, bool oaff, bool raw) {
    static thread_local char buf[96];
    const bool stats = epi == SD_EPI_STATS || epi == SD_EPI_SPLIT_STATS;
    const HTile t = fwd_tile(c0 + c1, H, W, N, stats);
    const bool wc = wconst_chunks((cdiv(c0, t.ck) + cdiv(c1, t.ck)) * (wsplit ? 2 : 1));
    const bool wconst = t.ck == 8 ? true : (t.ck != 16 && wc);
    const bool r = raw && halo_raw_enabled() && t.ck == 32 && t.it == 1 && !bns;
    // every template argument, as rocprofv3 names the instance
    snprintf(buf, sizeof(buf), "k_halo_conv<%d, %d, %d, %s, %s, %d, %s, %s, %s>", N == 32 ? 1 : 2, t.rt, t.ck,
             stats && !oaff ? "true" : "false", wconst ? "true" : "false", t.it, bns ? "true" : "false",
             oaff ? "true" : "false", r ? "true" : "false");
    return buf;
}

// wconst (one or two chunks per item): the weights are staged once per block. CK = 8 always has one chunk; CK = 16
// (experiments) always takes the general instance, which is also correct with one chunk.
// sum of the split-K partials part[ks][pixel][N] (fp32, the groups in order: deterministic), then the output affine
// (OAFF launches) -> bf16 out[pixel][N]; 8 channels per thread
__global__ __launch_bounds__(256) void k_halo_split_reduce(const float* __restrict__ part, int ksplit, long long n8, int N,
                                                           const float* __restrict__ osc, const float* __restrict__ osh,
                                                           __bf16* __restrict__ out) {
    const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
    if (i >= n8) return;
    const float4* src = reinterpret_cast<const float4*>(part) + 2 * i;
    float v[8];
    {
        const float4 a = src[0], b = src[1];
        v[0] = a.x, v[1] = a.y, v[2] = a.z, v[3] = a.w, v[4] = b.x, v[5] = b.y, v[6] = b.z, v[7] = b.w;
    }
    for (int k = 1; k < ksplit; ++k) {
        const float4 a = src[(size_t)k * 2 * n8], b = src[(size_t)k * 2 * n8 + 1];
        v[0] += a.x, v[1] += a.y, v[2] += a.z, v[3] += a.w, v[4] += b.x, v[5] += b.y, v[6] += b.z, v[7] += b.w;
    }
    if (osc) {
        const int c = (int)((8 * i) % N);
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = fmaf(v[j], osc[c + j], osh[c + j]);
    }
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = (__bf16)v[j];
    reinterpret_cast<bf16x8*>(out)[i] = o;
}

// split-K plan of an eval STORE launch (SD_HALO_SPLIT=0 disables it and the 32-channel N-blocks, for A/B runs): where
// the grid has fewer than 128 blocks, 32-channel N-blocks for N % 64 == 0 (twice the blocks) and then groups of blocks
// over slices of the chunks, up to 256 blocks with at least one chunk each
struct HSplit {
    int ksplit, cps, nblk, gper;
    bool nt1;
};
static HSplit halo_split_plan(const HTile& t, int nblk, int gper, int nsp, int N, int nch_v, int epi, bool bns) {
    static const bool on = [] {
        const char* e = getenv("SD_HALO_SPLIT");
        return !(e && atoi(e) == 0);
    }();
    HSplit q{1, nch_v, nblk, gper, false};
    if (!on || epi != SD_EPI_STORE || bns || t.it != 1 || t.ck == 16) return q;
    auto grid_of = [&](int nb) {
        q.nblk = nb;
        q.gper = PERSIST_BLOCKS / nb;
        if (q.gper < 1) q.gper = 1;
        if (q.gper > nsp) q.gper = nsp;
        q.ksplit = 1;
        q.cps = nch_v;
        const int gblk = q.gper * nb;
        if (gblk < 128 && nch_v >= 2) {
            int ks = PERSIST_BLOCKS / gblk;
            if (ks > nch_v) ks = nch_v;
            if (ks > 1) {
                q.cps = cdiv(nch_v, ks);
                q.ksplit = cdiv(nch_v, q.cps);
            }
        }
    };
    grid_of(nblk);
    if (N % 64 == 0 && t.ck == 32 && t.rt <= 3 && q.gper * q.nblk * q.ksplit < 128) {
        q.nt1 = true;
        grid_of(N / 32);
    }
    return q;
}

template <int NT, int RT, int CK, int IT = 1>
static void launch_halo(bool stats, bool wconst, dim3 grid, hipStream_t st, const HFwdArgs& p, bool bns = false,
                        bool raw = false) {
    constexpr bool W0 = CK == 8, W1 = CK != 16;  // the instance for wconst false / true
    // every source raw (dgrads, pooled encoder inputs): the all-LDS-DMA loaders (k_halo_conv RAW)
    if constexpr (IT == 1 && CK == 32) {
        if (raw && !bns) {
            auto go = [&](auto ST, auto WC, auto OA) {
                hipLaunchKernelGGL((k_halo_conv<NT, RT, CK, decltype(ST)::v, decltype(WC)::v, 1, false, decltype(OA)::v,
                                                true>),
                                   grid, dim3(512), 0, st, p);
            };
            auto by_wc = [&](auto ST, auto OA) {
                if (wconst) go(ST, BoolC<true>{}, OA);
                else go(ST, BoolC<false>{}, OA);
            };
            if (p.osc) by_wc(BoolC<false>{}, BoolC<true>{});
            else if (stats) by_wc(BoolC<true>{}, BoolC<false>{});
            else by_wc(BoolC<false>{}, BoolC<false>{});
            return;
        }
    }
    if constexpr (IT == 1 && CK != 16) {
        if (p.osc) {  // eval forwards with the BN affine in the epilogue (sd_conv3x3_ex)
            if (wconst ? W1 : W0)
                hipLaunchKernelGGL((k_halo_conv<NT, RT, CK, false, W1, IT, false, true>), grid, dim3(512), 0, st, p);
            else
                hipLaunchKernelGGL((k_halo_conv<NT, RT, CK, false, W0, IT, false, true>), grid, dim3(512), 0, st, p);
            return;
        }
    }
    // BN-backward sums (dgrad STORE launches, sd_conv_gemm_bnsum); not NT 2 x RT 3 (the second accumulator set
    // and the prefetched y pieces spill there: sd_halo_bnsum_ok)
    if constexpr (CK == 32 && IT == 1 && !(NT == 2 && RT == 3)) {
        if (bns) {
            if (wconst ? W1 : W0)
                hipLaunchKernelGGL((k_halo_conv<NT, RT, CK, false, W1, IT, true>), grid, dim3(512), 0, st, p);
            else
                hipLaunchKernelGGL((k_halo_conv<NT, RT, CK, false, W0, IT, true>), grid, dim3(512), 0, st, p);
            return;
        }
    }
    if (stats && (wconst ? W1 : W0))
        hipLaunchKernelGGL((k_halo_conv<NT, RT, CK, true, W1, IT, false>), grid, dim3(512), 0, st, p);
    else if (stats)
        hipLaunchKernelGGL((k_halo_conv<NT, RT, CK, true, W0, IT, false>), grid, dim3(512), 0, st, p);
    else if (wconst ? W1 : W0)
        hipLaunchKernelGGL((k_halo_conv<NT, RT, CK, false, W1, IT, false>), grid, dim3(512), 0, st, p);
    else
        hipLaunchKernelGGL((k_halo_conv<NT, RT, CK, false, W0, IT, false>), grid, dim3(512), 0, st, p);
}

// split-K workspace bytes of an eval STORE launch (0: the shape runs unsplit)
long long sd_halo_split_ws_bytes(const sd_src& a, int batch, int H, int W, int N, int epi, bool wsplit) {
    const HTile t = fwd_tile(a.chans[0] + a.chans[1], H, W, N, false);  // eval launches
    int nblk, gper, nsp;
    halo_grid(t, batch, H, W, N, nblk, gper, nsp);
    const int nch = cdiv(a.chans[0], t.ck) + cdiv(a.chans[1], t.ck);
    const HSplit q = halo_split_plan(t, nblk, gper, nsp, N, nch * (wsplit ? 2 : 1), epi, false);
    return q.ksplit > 1 ? (long long)q.ksplit * batch * H * W * N * 4 : 0;
}

int sd_halo_conv_fwd(const sd_src& a, int batch, int H, int W, const void* wpack, int N, int kpad, int epi, void* out0,
                     void* out1, int n_split, float* stats, hipStream_t st, const HaloBnSum* bns, bool wsplit,
                     const float* osc, const float* osh, void* ws, long long ws_bytes) {
    const bool st_ = epi == SD_EPI_STATS || epi == SD_EPI_SPLIT_STATS;
    const HTile t = fwd_tile(a.chans[0] + a.chans[1], H, W, N, st_);
    HFwdArgs p;
    p.a = make_halo_src(a);
    p.H = H;
    p.W = W;
    p.th = t.th;
    p.tw = t.tw;
    p.tiles_x = cdiv(W, t.tw);
    p.tiles = p.tiles_x * cdiv(H, t.th);
    halo_grid(t, batch, H, W, N, p.nblk, p.gper, p.nsp);
    p.hw = t.tw + 2;
    p.nhalo = (t.th + 2) * (t.tw + 2);
    p.wp = (const __bf16*)wpack;
    p.N = N;
    p.kpad = kpad;
    p.wsplit = wsplit ? 1 : 0;
    p.osc = osc;
    p.osh = osh;
    SD_REQUIRE(!osc || (osh && epi == SD_EPI_STORE && !bns && t.it == 1 && t.ck != 16),
               "sd_conv_gemm(halo): the affine epilogue is a STORE of a CK 8 / 32 shape");
    SD_REQUIRE(!wsplit || (!bns && kpad >= 18 * (a.chans[0] + a.chans[1])),
               "sd_conv_gemm(halo): split weights need kpad >= 18 * channels (and no BN-backward sums)");
    p.epi = epi;
    p.out0 = (__bf16*)out0;
    p.out1 = (__bf16*)out1;
    p.n_split = n_split;
    p.stats = stats;
    p.by = nullptr;
    p.bsc = p.bsh = p.bmu = p.bis = nullptr;
    if (bns) {
        SD_REQUIRE(epi == SD_EPI_STORE && t.ck == 32 && t.it == 1 && stats,
                   "sd_conv_gemm_bnsum: STORE epilogue of a CK = 32 halo shape with a partials buffer");
        p.by = (const __bf16*)bns->y;
        p.bsc = bns->scale;
        p.bsh = bns->shift;
        p.bmu = bns->mean;
        p.bis = bns->invstd;
    }
    const int nch = cdiv(p.a.c0, t.ck) + cdiv(p.a.c1, t.ck);
    HSplit q = halo_split_plan(t, p.nblk, p.gper, p.nsp, N, nch * (wsplit ? 2 : 1), epi, bns != nullptr);
    const long long need = q.ksplit > 1 ? (long long)q.ksplit * batch * H * W * N * 4 : 0;
    if (q.ksplit > 1 && (!ws || ws_bytes < need || ((uintptr_t)ws & 15) != 0)) {  // no workspace: one group
        q.ksplit = 1;
        q.cps = nch * (wsplit ? 2 : 1);
    }
    p.nblk = q.nblk;
    p.gper = q.gper;
    p.gblk = q.gper * q.nblk;
    p.ksplit = q.ksplit;
    p.cps = q.cps;
    p.npix = batch * H * W;
    p.part = q.ksplit > 1 ? (float*)ws : nullptr;
    p.xcd = halo_xcd_enabled() && (p.gblk * q.ksplit) % 8 == 0;
    p.prio = halo_prio(a);
    p.dbg = g_wg_dbg;
    const int cap = t.it == 2 ? 384 : halo_px_cap(t.rt, t.ck);
    SD_REQUIRE(t.rt >= 2 && t.rt <= 4 && p.nhalo <= cap && t.th * t.tw <= 128 * t.rt &&
                   t.th < 64 && t.tw < 512,
               "sd_conv_gemm(halo): tile %dx%d (RT %d, CK %d)", t.th, t.tw, t.rt, t.ck);
    SD_REQUIRE((long long)batch * p.tiles < (1LL << 30), "sd_conv_gemm(halo): too many tiles");
    // 32-bit buffer offsets: image-local halo offsets (24-bit pixel index) and the packed weights
    SD_REQUIRE((long long)H * W < (1LL << 24) && (long long)H * W * (a.chans[0] > a.chans[1] ? a.chans[0] : a.chans[1]) * 2 <
                   (1LL << 31) && (long long)N * kpad * 2 < (1LL << 31) && (long long)H * W * N * 2 < (1LL << 31),
               "sd_conv_gemm(halo): image %dx%d or weights %dx%d too large for 32-bit offsets", H, W, N, kpad);
    const dim3 grid(p.gblk * q.ksplit);
    const bool wc = wconst_chunks(q.cps);
    const bool raw = halo_raw_enabled() && t.ck == 32 && t.it == 1 && !bns && a.xform[0] != SD_BNRELU &&
                     (a.chans[1] == 0 || a.xform[1] != SD_BNRELU);
    SD_REQUIRE(!(N == 32 && t.ck == 32 && t.rt == 4) || (t.th == 16 && t.tw == 32),
               "sd_conv_gemm(halo): the N = 32 RT 4 instances (vertical reuse) need 16x32 tiles, got %dx%d", t.th, t.tw);
    SD_REQUIRE(t.ck != 8 || nch == 1, "sd_conv_gemm(halo): CK = 8 needs <= 8 input channels");
    if (q.nt1) {  // 32-channel N-blocks of an N % 64 layer (batch-1 eval)
        if (t.rt == 3) launch_halo<1, 3, 32>(st_, wc, grid, st, p, false, raw);
        else launch_halo<1, 2, 32>(st_, wc, grid, st, p, false, raw);
    } else if (t.ck == 8) {
        if (t.rt == 4) launch_halo<1, 4, 8>(st_, wc, grid, st, p);
        else if (t.rt == 3) launch_halo<1, 3, 8>(st_, wc, grid, st, p);
        else launch_halo<1, 2, 8>(st_, wc, grid, st, p);
    } else if (N == 32) {
        if (t.rt == 4) launch_halo<1, 4, 32>(st_, wc, grid, st, p, bns, raw);
        else if (t.rt == 3) launch_halo<1, 3, 32>(st_, wc, grid, st, p, bns, raw);
        else launch_halo<1, 2, 32>(st_, wc, grid, st, p, bns, raw);
    } else if (t.ck == 32) {
        if (t.rt == 3) launch_halo<2, 3, 32>(st_, wc, grid, st, p, bns, raw);
        else launch_halo<2, 2, 32>(st_, wc, grid, st, p, bns, raw);
    } else if (t.it == 2) {  // RT = 2 only (RT = 3 with two accumulator sets spills)
        launch_halo<2, 2, 16, 2>(st_, wc, grid, st, p);
    } else if (t.rt == 4) {
        launch_halo<2, 4, 16>(st_, wc, grid, st, p);
    } else if (t.rt == 3) {
        launch_halo<2, 3, 16>(st_, wc, grid, st, p);
    } else {
        launch_halo<2, 2, 16>(st_, wc, grid, st, p);
    }
    if (q.ksplit > 1) {
        const long long n8 = (long long)batch * H * W * N / 8;
        hipLaunchKernelGGL(k_halo_split_reduce, dim3((unsigned)((n8 + 255) / 256)), dim3(256), 0, st, p.part, q.ksplit,
                           n8, N, osc, osh, (__bf16*)out0);
    }
    return sd_check_launch("sd_conv_gemm(halo)");
}

bool sd_halo_wgrad_shape(int M, int N) { return (M == 32 || M % 64 == 0) && N % 9 == 0 && (N / 9) % 8 == 0; }
bool sd_halo_wgrad_ok(const sd_src& a, const sd_src& b, int M) {
    return a.taps == 1 && b.taps == 9 && !a.pool && !b.pool && a.chans[1] == 0 && (M == 32 || M % 64 == 0);
}

// wgrad tile: th x tw (<= 256 pixels, halo <= HMAX) minimising k-step work plus halo staging
// over the whole image; tw runs over the image width and its divisors (and 32)
static HTile wgrad_tile(int H, int W) {
    HTile best{8, 32, 8};
    double best_cost = 1e300;
    for (int tw = W < 8 ? W : 8; tw <= (W < WG_MAXPX ? W : WG_MAXPX); ++tw) {
        if (tw != W && tw != 32 && W % tw) continue;
        for (int th = 1; th <= H && th * tw <= WG_MAXPX; ++th) {
            if ((th + 2) * (tw + 2) > HMAX) break;
            const double tiles = (double)cdiv(H, th) * cdiv(W, tw);
            const double cost = tiles * (cdiv(th * tw, 32) * 32 + 0.5 * (th + 2) * (tw + 2));
            if (cost < best_cost) {
                best_cost = cost;
                best = {th, tw, cdiv(th * tw, 32)};
            }
        }
    }
    return best;
}


// warp-specialised wgrad (k_halo_wgrad_ws): dy channels per block COUT = 64 (M % 64 == 0) or 32 (M == 32),
// x channels per block CIB = 64 or 32 (the channel count and the first source's width divisible by it;
// c0 < 0: unknown, sizing only). 0: not applicable (enc1.0's 8-channel input), k_halo_wgrad runs.
// SD_WG_WS=0 keeps k_halo_wgrad everywhere (A/B runs).
struct WsCfg {
    int cout, cib;
    bool span = false;  // a block's CIB channels straddle the two sources (k_halo_wgrad_ws SPAN)
};
static WsCfg wgrad_ws(int M, int N, int c0 = -1) {
    static const bool on = [] {
        const char* e = getenv("SD_WG_WS");
        return !(e && atoi(e) == 0);
    }();
    const int ctot = N / 9;
    WsCfg c{M % 64 == 0 ? 64 : (M == 32 ? 32 : 0), 0};
    if (!on || c.cout == 0 || N % 9) return {0, 0};
    // SD_WS_CIB64=1: 64-channel x blocks straddling the two sources for 32 dy channels (dec1.0's cat(32 + 32): one dy
    // transform instead of two). Off: measured 590 us against 378 us for its two 32-channel blocks on one box
    // (gpurun_out/sp1; one block per CU and two loads per halo piece)
    static const bool span = [] {
        const char* e = getenv("SD_WS_CIB64");
        return e && atoi(e) == 1;
    }();
    // the straddling (SPAN) instance is built for 32 dy channels only (dec1.0): 64 dy channels keep 32-channel x blocks
    if (ctot % 64 == 0 && (c0 < 0 || c0 % 64 == 0 || (span && c.cout == 32 && c0 % 8 == 0))) {
        c.cib = 64;
        c.span = c0 > 0 && c0 % 64 != 0;
    } else if (ctot % 32 == 0 && (c0 < 0 || c0 % 32 == 0)) {
        c.cib = 32;
    }
    return c.cib ? c : WsCfg{0, 0};
}

// its tile and halo layout: th x tw <= 128 pixels fitting one of the two layouts, minimising the MFMA work
// (a tile always costs 128 pixels) plus the staged halo slots (each one costs the loaders a transform)
struct WsTile {
    int th, tw, hp, hr;
};
static WsTile wgrad_tile_ws(int H, int W) {
    WsTile best{4, 32, 34, 6};
    double best_cost = 1e300;
    const int layouts[2][2] = {{34, 6}, {22, 8}};
    for (const auto& l : layouts) {
        const int slots = (l[0] * l[1] * 8 + 255) / 256 * 32;
        for (int tw = W < 8 ? W : 8; tw <= (W < l[0] - 2 ? W : l[0] - 2); ++tw) {
            if (tw != W && tw != 32 && W % tw) continue;
            for (int th = 1; th <= H && th * tw <= WS_TPX && th + 2 <= l[1]; ++th) {
                const double tiles = (double)cdiv(H, th) * cdiv(W, tw);
                const double cost = tiles * (WS_TPX + 1.0 * slots);
                if (cost < best_cost) {
                    best_cost = cost;
                    best = {th, tw, l[0], l[1]};
                }
            }
        }
    }
    return best;
}

// SD_WS_MF32=1: the 64 x 64 blocks on v_mfma_f32_32x32x16_bf16 (opt-in, read per call). Bit-identical to the 16x16x32
// form, and 4-9 % slower at every step shape (tools/conv_micro.py --wgrad-step, r06): DESIGN.md §3 r06
static bool ws_mf32_enabled() {
    const char* e = getenv("SD_WS_MF32");
    return e && atoi(e) == 1;
}

// SD_WS_CO128 (read per call; 0 = off): the plain (no BatchNorm-backward) weight gradients with M % 128 == 0 take
// 128 dy x 32 x channels per block instead of 64 x 64. The MFMA waves' layout is unchanged (each owns 64 dy rows x 16 x
// channels x 9 taps, RM = 4) and so is the block count, hence the splits and the slab layout; per tile the loaders
// transform and stage half the x halo (the BN+ReLU transform is their VALU, and the loaders paced the 64 x 64 blocks:
// busy 92 % of their cycles at every step shape, tools/conv_micro.py SD_WG_DIAG) and LDS-DMA twice the dy rows (no VALU)
static bool ws_co128_enabled() {
    const char* e = getenv("SD_WS_CO128");
    return !(e && atoi(e) == 0);
}
static WsCfg wgrad_ws_launch(int M, int N, int c0, bool bnb) {
    WsCfg c = wgrad_ws(M, N, c0);
    if (!bnb && c.cout == 64 && c.cib && !c.span && M % 128 == 0 && (N / 9) % 32 == 0 && c0 % 32 == 0 &&
        ws_co128_enabled())
        c = WsCfg{128, 32};
    return c;
}

int sd_halo_wgrad_splits(int batch, int H, int W, int M, int N) {
    const WsCfg ws = wgrad_ws(M, N);
    HTile t = wgrad_tile(H, W);
    if (ws.cib) {
        const WsTile w = wgrad_tile_ws(H, W);
        t = {w.th, w.tw, 4, 32};
    }
    const int nblk = ws.cib ? (N / 9 / ws.cib) * (M / ws.cout) : cdiv(N / 9, CK) * (M == 32 ? 1 : M / 64);
    const int nt = cdiv(W, t.tw) * cdiv(H, t.th) * batch;
    static const int blocks = [] {  // SD_WG_BLOCKS: total split-K blocks (A/B runs)
        const char* e = getenv("SD_WG_BLOCKS");
        return e && atoi(e) > 0 ? atoi(e) : 512;
    }();
    // one round of blocks: 2 per CU for k_halo_wgrad (LDS, registers), 1 per CU for the warp-specialised one
    int splits = cdiv(ws.cib ? PERSIST_BLOCKS * ws_blocks_per_cu(ws.cout, ws.cib) : blocks, nblk);
    if (splits > nt) splits = nt;
    return splits < 1 ? 1 : splits;
}

const char* sd_halo_wgrad_name(int M, int N, int c0, int H, int W, bool bnb) {
    static thread_local char buf[64];
    const WsCfg ws = wgrad_ws_launch(M, N, c0, bnb);
    if (!ws.cib)
        return M == 32 ? (bnb ? (wg_x8(c0) ? "k_halo_wgrad<32, true, true>" : "k_halo_wgrad<32, true>")
                              : "k_halo_wgrad<32, false>")
                       : "k_halo_wgrad<64, false>";
    const WsTile t = wgrad_tile_ws(H, W);
    const bool mf32 = ws.cout == 64 && ws.cib == 64 && ws_mf32_enabled();
    snprintf(buf, sizeof(buf), "k_halo_wgrad_ws<%d, %d, %d, %d, %s, %s%s>", ws.cout, ws.cib, t.hp, t.hr, bnb ? "true" : "false",
             ws.span ? "true" : "false", mf32 ? ", true" : "");
    return buf;
}

template <int COUT, int CIB, bool BNB, bool SPAN = false, bool MF32 = false>
static void launch_wgrad_ws(int hp, dim3 grid, hipStream_t st, const HWgArgs& p) {
    if (hp == 34)
        hipLaunchKernelGGL((k_halo_wgrad_ws<COUT, CIB, 34, 6, BNB, SPAN, MF32>), grid, dim3(512), 0, st, p);
    else
        hipLaunchKernelGGL((k_halo_wgrad_ws<COUT, CIB, 22, 8, BNB, SPAN, MF32>), grid, dim3(512), 0, st, p);
}
template <bool BNB>
static void launch_wgrad_ws(const WsCfg& ws, int hp, dim3 grid, hipStream_t st, const HWgArgs& p) {
    if (!BNB && ws.cout == 128) launch_wgrad_ws<128, 32, false>(hp, grid, st, p);
    else if (ws.cout == 64 && ws.cib == 64 && ws_mf32_enabled()) launch_wgrad_ws<64, 64, BNB, false, true>(hp, grid, st, p);
    else if (ws.cout == 64 && ws.cib == 64) launch_wgrad_ws<64, 64, BNB>(hp, grid, st, p);
    else if (ws.cout == 64) launch_wgrad_ws<64, 32, BNB>(hp, grid, st, p);
    else if (ws.cib == 64 && ws.span) launch_wgrad_ws<32, 64, BNB, true>(hp, grid, st, p);
    else if (ws.cib == 64) launch_wgrad_ws<32, 64, BNB>(hp, grid, st, p);
    else launch_wgrad_ws<32, 32, BNB>(hp, grid, st, p);
}

// the BatchNorm-backward apply fused into the dy staging: warp-specialised instances only. Returns the number
// of x-channel blocks (grid.x) that each form the same dy tile (0: no fused kernel for the shape)
// k_halo_wgrad<32, true> (x channels not a multiple of 32: enc1.0) only without a dy destination.
int sd_halo_wgrad_bnbwd_blocks(const sd_src& a, const sd_src& b, int M, int N) {
    if (!sd_halo_wgrad_ok(a, b, M)) return 0;
    const WsCfg ws = wgrad_ws(M, N, b.chans[0]);
    if (ws.cib) return (N / 9) / ws.cib;
    return M == 32 && !a.ptr[0] ? cdiv(b.chans[0] + b.chans[1], CK) : 0;
}

int sd_halo_wgrad(const sd_src& a, const sd_src& b, int batch, int H, int W, int M, int N, float* slab, int splits,
                  hipStream_t st, const HaloBnBwd* bnb) {
    const WsCfg ws = wgrad_ws_launch(M, N, b.chans[0], bnb != nullptr);  // one source per block of x channels
    const WsTile wt = wgrad_tile_ws(H, W);
    const HTile t = ws.cib ? HTile{wt.th, wt.tw, 4, 32} : wgrad_tile(H, W);
    HWgArgs p;
    p.dy = (const __bf16*)a.ptr[0];
    p.x = make_halo_src(b);
    p.H = H;
    p.W = W;
    p.th = t.th;
    p.tw = t.tw;
    p.hw = t.tw + 2;
    p.nhalo = (t.th + 2) * (t.tw + 2);
    p.tiles_x = cdiv(W, t.tw);
    p.tiles_y = cdiv(H, t.th);
    p.ntiles = p.tiles_x * p.tiles_y * batch;
    p.tiles_per_split = cdiv(p.ntiles, splits);
    p.M = M;
    p.N = N;
    p.slab = slab;
    p.dbg = g_wg_dbg;
    p.bda = p.by = nullptr;
    p.bsc = p.bsh = p.bmu = p.bis = p.bcoef = nullptr;
    p.ncc = 1;
    if (bnb) {
        p.bda = (const __bf16*)bnb->da;
        p.by = (const __bf16*)bnb->y;
        p.bsc = bnb->scale;
        p.bsh = bnb->shift;
        p.bmu = bnb->mean;
        p.bis = bnb->invstd;
        p.bcoef = bnb->coef;
    }
    if (ws.cib) {
        const int ncc = p.x.ctot / ws.cib;
        p.xcd = halo_xcd_enabled() && (ncc * splits * (M / ws.cout)) % 8 == 0;
        SD_REQUIRE(t.th + 2 <= wt.hr && t.tw + 2 <= wt.hp && t.th * t.tw <= WS_TPX, "sd_wgrad_gemm(halo ws): tile %dx%d",
                   t.th, t.tw);
        const dim3 grid(ncc, splits, M / ws.cout);
        p.ncc = ncc;
        if (bnb) launch_wgrad_ws<true>(ws, wt.hp, grid, st, p);
        else launch_wgrad_ws<false>(ws, wt.hp, grid, st, p);
        return sd_check_launch(bnb ? "sd_wgrad_gemm_bnbwd(halo ws)" : "sd_wgrad_gemm(halo ws)");
    }
    p.xcd = halo_xcd_enabled() && (cdiv(p.x.ctot, CK) * splits * (M == 32 ? 1 : M / 64)) % 8 == 0;
    SD_REQUIRE(p.nhalo <= HMAX && t.th * t.tw <= WG_MAXPX, "sd_wgrad_gemm(halo): tile %dx%d", t.th, t.tw);
    if (bnb) {  // enc1.0 (no dgrad): dy is not written
        if (M != 32 || a.ptr[0]) {
            sd_set_error("sd_wgrad_gemm_bnbwd: k_halo_wgrad fuses M = 32 without a dy destination only (M=%d)", M);
            return SD_EINVAL;
        }
        if (wg_x8(p.x.ctot))
            hipLaunchKernelGGL((k_halo_wgrad<32, true, true>), dim3(cdiv(p.x.ctot, CK), splits, 1), dim3(256), 0, st, p);
        else
            hipLaunchKernelGGL((k_halo_wgrad<32, true>), dim3(cdiv(p.x.ctot, CK), splits, 1), dim3(256), 0, st, p);
    } else if (M == 32) {
        hipLaunchKernelGGL((k_halo_wgrad<32, false>), dim3(cdiv(p.x.ctot, CK), splits, 1), dim3(256), 0, st, p);
    } else {
        hipLaunchKernelGGL((k_halo_wgrad<64, false>), dim3(cdiv(p.x.ctot, CK), splits, M / 64), dim3(256), 0, st, p);
    }
    return sd_check_launch(bnb ? "sd_wgrad_gemm_bnbwd(halo)" : "sd_wgrad_gemm(halo)");
}
