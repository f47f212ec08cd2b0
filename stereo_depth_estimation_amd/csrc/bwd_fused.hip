// Fused backward of a full-resolution 32 -> 32 channel 3x3 conv + BatchNorm + ReLU layer (model.py:36-41; enc1.1 and
// dec1.1 of the 320x240 StereoUNet, whose tensors are 315 MB each at B = 64). One pass over the layer produces
//   dy = BatchNorm-backward(da, y)        staged in LDS as a halo, never stored (bn_bwd_pk)
//   dW = sum_px x[px + tap] dy[px]^T      x = relu(bn_prev(y_prev)), split-K partial slab per block
//   dx = sum_tap dy[px + tap] Wd[tap]     the dgrad (Wd: the dgrad-packed, flipped weights) = da of the previous
//                                         BatchNorm layer, stored
//   the previous layer's BatchNorm-backward sums (sum dz, sum dz*xhat over dx and y_prev), one partial row per block
// It replaces the fused BatchNorm-backward weight gradient (k_halo_wgrad_ws<32, 32, ..., BNB>: read da, y, y_prev,
// wrote dy) and the BatchNorm-sums dgrad (k_halo_conv<1, 4, 32, ..., BNS>: read dy, y_prev, wrote dx): per layer
// 4 full-resolution tensor passes (da, y, y_prev in; dx out) instead of 7.
//
// One 512-thread block per CU, persistent over a contiguous range of 8x16-pixel tiles (its split-K range):
//   waves 4-7 (loaders): per tile, the 10x18 halo of (da, y) -> dy and of y_prev -> x (BN + ReLU), through registers
//                        (two tiles in flight) into an LDS double buffer, plus the raw y_prev of the tile (the
//                        sums' operand);
//   waves 0-3 (MFMA)   : weight gradient (two taps and a quarter of the third per wave, 32 co x 32 ci,
//                        v_mfma_f32_32x32x16_bf16 on transposed fragments, k = tile pixels) and dgrad (32 tile
//                        pixels = two rows per wave, all 32 ci, 32x32x16 MFMAs over 9 taps x 32 dy channels with the
//                        dgrad weights resident in LDS), then the dgrad epilogue.
#include <stdio.h>

#include "halo_util.h"

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int FB_TH = 8, FB_TW = 16;               // output tile: 4 units of 32 pixels (2 rows each)
constexpr int FB_HW = FB_TW + 2, FB_HH = FB_TH + 2;  // halo width / rows
constexpr int FB_HPX = FB_HW * FB_HH;              // 180 halo pixels
constexpr int FB_NI = (FB_HPX * 4 + 255) / 256;    // loader items per thread (3 x 256 >= 180 pixels x 4 pieces)
constexpr int FB_HSL = (FB_NI * 256 / 32) * 8;     // halo pixel slots (items past the halo land in slots >= FB_HPX)
static_assert(FB_TH * FB_TW == 128 && FB_TW % 16 == 0, "4 MFMA waves x 32 pixels; tr_pair rows p, p + 8 in one row");
constexpr int FB_DL = 40;                          // dy halo pixel pitch (80 B: odd 16-B slot count, b128 reads)
constexpr int FB_XL = 48;                          // x halo pixel pitch (96 B)
// x halo: channels 16..31 of pixel p sit FB_XC elements after its channels 0..15 (past the next pixel's first half):
// the transposed reads of a 32-lane half (4 pixels x channels {0..15, 16..31}) then cover the 64 banks once, where the
// plain +16 layout put pixel 3's first half on pixel 0's second (2-way conflicts, PMC 0.37 extra cycles per access)
constexpr int FB_XC = 64;
__device__ __forceinline__ int fb_xoff(int c) { return (c & 15) + (c >> 4) * FB_XC; }  // channel c's element offset
constexpr int FB_WL = 9 * 32 + 8;                  // dgrad weight row (592 B, odd slot count)
constexpr int FB_SL = 40;                          // raw y_prev stash pitch (the sums' operand)
constexpr int FB_DYH = FB_HSL * FB_DL, FB_XH = FB_HSL * FB_XL + (FB_XC - FB_XL + 16), FB_ST = FB_TH * FB_TW * FB_SL;
constexpr int FB_BUF = FB_DYH + FB_XH + FB_ST;     // elements per LDS buffer
constexpr int FB_BLOCKS = 256;                     // one per CU
#ifndef FB_EXP
#define FB_EXP 0  // timing-only builds (results wrong): 1 no loader transform, 16 no loads after the first two
                  // tiles, 32 per-wave phase cycle counters (sd_debug_buffer), 128 loader waves at s_setprio 1
#endif
constexpr bool FB_DG = (FB_EXP & 32) != 0;
__device__ __forceinline__ unsigned long long fb_clk() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    return __builtin_amdgcn_s_memtime();
}

struct BwdArgs {
    const __bf16 *da, *y, *yp;                        // [B*H*W][32]
    const float *sc, *sh, *mu, *is, *coef;            // this layer's BatchNorm: forward affine, statistics, backward coef
    const float *psc, *psh, *pmu, *pis;               // the previous BatchNorm layer (x = relu(psc*yp + psh))
    const __bf16* wd;                                 // dgrad-packed weights [32 ci][kpad], k = tap*32 + co (flipped)
    int kpad;
    int B, H, W, tiles_x, tiles_y;                    // tiles per block: fb_ntile (its split-K range)
    __bf16* dx;                                       // [B*H*W][32]
    float* slab;                                      // [blocks][32 co][288], k = tap*32 + ci
    float2* part;                                     // [blocks][32] (sum dz, sum dz*xhat) of the previous layer
    unsigned long long* dbg;                          // timing build only: [block][wave][8] phase cycles
};

template <bool B> struct BoolC { static constexpr bool v = B; };

template <int PPX>
__device__ __forceinline__ int fb_pixel(int item) { return (item / (8 * PPX)) * 8 + (item & 7); }
template <int PPX>
__device__ __forceinline__ int fb_piece(int item) { return (item >> 3) % PPX; }

// A block's k-th tile -> (column strip tx, tile row ty, image b). Blocks own whole 16-pixel column strips (strip
// bid, bid + nblk, ...) and walk down each, ty fastest: the two halo rows a tile shares with the one above were
// loaded one tile earlier (L2 hits), and the blocks of one XCD (consecutive bid) walk adjacent strips side by side,
// so the halo columns two strips share are fetched once for both (row-major order re-fetched the shared rows from
// beyond L2: 1.5x the algorithmic reads; one contiguous strip range per block: 1.24x, PMC)
__device__ __forceinline__ void fb_tile(int tiles_x, int tiles_y, int bid, int nblk, int k, int& tx, int& ty, int& b) {
    const int strip = bid + (k / tiles_y) * nblk;
    ty = k % tiles_y;
    tx = strip % tiles_x;
    b = strip / tiles_x;
}
__device__ __forceinline__ int fb_ntile(int tiles_x, int tiles_y, int B, int bid, int nblk) {
    const int nstrips = tiles_x * B;
    return bid < nstrips ? ((nstrips - 1 - bid) / nblk + 1) * tiles_y : 0;
}

__global__ __launch_bounds__(512) void k_bwd_fused32(const BwdArgs p) {
    __shared__ __attribute__((aligned(16))) __bf16 smem[2 * FB_BUF];
    __shared__ __attribute__((aligned(16))) __bf16 wds[32 * FB_WL];
    __shared__ __attribute__((aligned(16))) __bf16 scr[4 * 32 * 32];  // per-wave dgrad epilogue transpose
    __shared__ __attribute__((aligned(16))) float redf[4 * 32 * 2];

    const int tid = threadIdx.x, lane = tid & 63;
    const bool is_loader = tid >= 256;
    const int wid = (tid >> 6) & 3;
    // XCD-contiguous block numbering: the tile ranges of one XCD's blocks are neighbours (shared halo rows in its L2)
    const int bid = (blockIdx.x & 7) * (gridDim.x >> 3) + (blockIdx.x >> 3);
    const int t_begin = 0;  // tiles are numbered per block (fb_tile)
    const int ntile = fb_ntile(p.tiles_x, p.tiles_y, p.B, bid, gridDim.x);
    const int hw = p.H * p.W;

    // the dgrad weights, resident for the launch (all threads; before the first barrier)
    for (int i = tid; i < 32 * 36; i += 512) {
        const int r = i / 36, c8 = i - r * 36;
        *reinterpret_cast<uint4*>(wds + r * FB_WL + c8 * 8) =
            *reinterpret_cast<const uint4*>(p.wd + (size_t)r * p.kpad + c8 * 8);
    }

    if (is_loader) {
        // =========================================================== loader waves
        const int ltid = tid - 256;
        if (FB_EXP & 128) __builtin_amdgcn_s_setprio(1);  // experiment: the loaders win VALU issue arbitration
        const int piece = fb_piece<4>(ltid);  // fixed per thread (256 * i keeps (item >> 3) % 4)
        constexpr unsigned OOB = 0x80000000u;
        // this thread's 8 channels: this layer's folded BatchNorm-backward constants and the previous layer's affine
        float ksc[8], ksh[8], kB[8], kC[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int c = piece * 8 + j;
            const float k1 = p.coef[3 * c + 1], k2 = p.coef[3 * c + 2], is = p.is[c], sc = p.sc[c], sh = p.sh[c];
            ksc[j] = sc;
            ksh[j] = sh;
            kB[j] = -is * k2;
            kC[j] = is * k2 * sh + sc * (p.mu[c] * is * k2 - k1);
        }
        const float4 s0 = *reinterpret_cast<const float4*>(p.psc + piece * 8);
        const float4 s1 = *reinterpret_cast<const float4*>(p.psc + piece * 8 + 4);
        const float4 t0 = *reinterpret_cast<const float4*>(p.psh + piece * 8);
        const float4 t1 = *reinterpret_cast<const float4*>(p.psh + piece * 8 + 4);
        // halo geometry of the items: (row << 8 | col), ~0 past the halo; interior stash slot or -1
        unsigned geo[FB_NI];
        int stash[FB_NI];
#pragma unroll
        for (int i = 0; i < FB_NI; ++i) {
            const int px = fb_pixel<4>(ltid + 256 * i);
            const int hy = px / FB_HW, hx = px - hy * FB_HW;
            geo[i] = px < FB_HPX ? (unsigned)(hy << 8 | hx) : 0xffffffffu;
            const bool in = px < FB_HPX && hy >= 1 && hy <= FB_TH && hx >= 1 && hx <= FB_TW;
            stash[i] = in ? ((hy - 1) * FB_TW + hx - 1) * FB_SL + piece * 8 : -1;
        }
        // items FB_HPX * 4.. are past the halo: a loader wave whose first item of the last slot is past it skips that
        // slot (wave-uniform)
        const bool w3 = (ltid & ~63) + 256 * (FB_NI - 1) < FB_HPX * 4;
        unsigned need = 0;
#pragma unroll
        for (int i = 0; i < FB_NI; ++i) need |= (unsigned)(geo[i] != 0xffffffffu) << i;
        struct Set {
            uint4 a[FB_NI], y[FB_NI], x[FB_NI];
            unsigned m;  // bit i: item i inside the image
            bool edge;   // wave-uniform: some halo item of the wave is padding (outside the image or the range)
        };
        Set sa, sb;
        auto load = [&](Set& q, int tile) __attribute__((always_inline)) {
            if ((FB_EXP & 16) && tile >= t_begin + 2) return;
            const bool live = tile < t_begin + ntile;
            const int tl = live ? tile : t_begin;
            int tx, ty, b;
            fb_tile(p.tiles_x, p.tiles_y, bid, gridDim.x, tl, tx, ty, b);
            const int h0 = ty * FB_TH - 1, w0 = tx * FB_TW - 1;
            const size_t img = (size_t)b * hw * 32;
            const __amdgpu_buffer_rsrc_t ra =
                __builtin_amdgcn_make_buffer_rsrc((void*)(p.da + img), (short)0, hw * 64, 0x00020000);
            const __amdgpu_buffer_rsrc_t ry =
                __builtin_amdgcn_make_buffer_rsrc((void*)(p.y + img), (short)0, hw * 64, 0x00020000);
            const __amdgpu_buffer_rsrc_t rp =
                __builtin_amdgcn_make_buffer_rsrc((void*)(p.yp + img), (short)0, hw * 64, 0x00020000);
            unsigned m = 0;
#pragma unroll
            for (int i = 0; i < FB_NI; ++i) {
                if (i == FB_NI - 1 && !w3) break;
                const int h = h0 + (int)(geo[i] >> 8), w = w0 + (int)(geo[i] & 0xffu);
                const bool ok = live & (geo[i] != 0xffffffffu) & (h >= 0) & (h < p.H) & (w >= 0) & (w < p.W);
                m |= (unsigned)ok << i;
                const unsigned off = ok ? (unsigned)(h * p.W + w) * 64u + (unsigned)piece * 16u : OOB;
                const auto va = __builtin_amdgcn_raw_buffer_load_b128(ra, off, 0, 0);
                const auto vy = __builtin_amdgcn_raw_buffer_load_b128(ry, off, 0, 0);
                const auto vp = __builtin_amdgcn_raw_buffer_load_b128(rp, off, 0, 0);
                q.a[i] = make_uint4(va[0], va[1], va[2], va[3]);
                q.y[i] = make_uint4(vy[0], vy[1], vy[2], vy[3]);
                q.x[i] = make_uint4(vp[0], vp[1], vp[2], vp[3]);
            }
            q.m = m;
            q.edge = __builtin_amdgcn_ballot_w64(m != (w3 ? need : need & ((1u << (FB_NI - 1)) - 1))) != 0;
        };
        auto store = [&](Set& q, int buf) __attribute__((always_inline)) {
            __bf16* dyh = smem + buf * FB_BUF;
            __bf16* xh = dyh + FB_DYH;
            __bf16* st = xh + FB_XH;
            auto put = [&](auto SEL) __attribute__((always_inline)) {
#pragma unroll
                for (int i = 0; i < FB_NI; ++i) {
                    if (i == FB_NI - 1 && !w3) break;
                    const bool ok = (q.m >> i) & 1u;
                    const int px = fb_pixel<4>(ltid + 256 * i);  // < FB_HSL (items past the halo unused)
                    uint4 d = (FB_EXP & 1) ? q.a[i] : bn_bwd_pk(q.a[i], q.y[i], ksc, ksh, kB, kC);
                    uint4 x = (FB_EXP & 1) ? q.x[i] : bnrelu_pk(q.x[i], s0, s1, t0, t1);
                    if constexpr (decltype(SEL)::v) {  // the dgrad's zero padding, and dy past the image
                        d = ok ? d : make_uint4(0, 0, 0, 0);
                        x = ok ? x : make_uint4(0, 0, 0, 0);
                    }
                    *reinterpret_cast<uint4*>(dyh + px * FB_DL + piece * 8) = d;
                    *reinterpret_cast<uint4*>(xh + px * FB_XL + fb_xoff(piece * 8)) = x;
                    if (stash[i] >= 0) *reinterpret_cast<uint4*>(st + stash[i]) = q.x[i];  // raw y_prev (0 outside)
                }
            };
            if (q.edge)
                put(BoolC<true>{});
            else
                put(BoolC<false>{});
        };
        load(sa, t_begin);
        __builtin_amdgcn_sched_barrier(0);
        load(sb, t_begin + 1);
        __syncthreads();  // the resident weights (the MFMA waves meet it before their first tile)
        // an even number of iterations (no exit between the two register sets); an odd count's last one stores a
        // tile past the range into the buffer the MFMA waves no longer read
        unsigned long long tc[5] = {0, 0, 0, 0, 0}, tm0 = 0, t_all = FB_DG ? fb_clk() : 0;
        auto stamp = [&](int k) __attribute__((always_inline)) {
            if (FB_DG) {
                const unsigned long long t1 = fb_clk();
                tc[k] += t1 - tm0;
                tm0 = t1;
            }
        };
        for (int i = 0; i < ntile; i += 2) {
            if (FB_DG) {
                tm0 = fb_clk();
                asm volatile("s_waitcnt vmcnt(9)" ::: "memory");  // this set's loads (9-12 of the other set stay)
                stamp(3);
            }
            store(sa, 0);
            stamp(0);
            load(sa, t_begin + i + 2);
            stamp(1);
            __syncthreads();
            stamp(2);
            if (FB_DG) {
                asm volatile("s_waitcnt vmcnt(9)" ::: "memory");
                stamp(3);
            }
            store(sb, 1);
            stamp(0);
            load(sb, t_begin + i + 3);
            stamp(1);
            __syncthreads();
            stamp(2);
        }
        if (FB_DG && p.dbg && lane == 0) {
            unsigned long long* d = p.dbg + ((size_t)bid * 8 + 4 + wid) * 8;
            d[0] = tc[0];
            d[1] = tc[1];
            d[2] = tc[2];
            d[3] = tc[3];
            d[4] = fb_clk() - t_all;
            d[5] = ntile;
        }
        __syncthreads();  // the statistics reduction (MFMA waves)
        return;
    }

    // =============================================================== MFMA waves
    __syncthreads();  // the resident weights
    // weight gradient, 32 co x 32 ci per tap (v_mfma_f32_32x32x16_bf16, k = 16 pixels = one tile row): wave w owns
    // taps w and w + 4 over the tile's 8 rows and tap 8 over rows 2w, 2w + 1 (summed over the waves at the end).
    // Transposed fragments (tr_pair): 16-lane group g holds channels 16 (g & 1) + (lane & 15) of the pixels
    // 4 (g >> 1) + {0..3, 8..11} of the row (the MFMA's k-half g >> 1); lane 4q + pp supplies the address of pixel
    // 4 (g >> 1) + q, channels 16 (g & 1) + 4 pp
    const int g = lane >> 4, q4 = (lane & 15) >> 2, pp = lane & 3;
    const int pk = 4 * (g >> 1) + q4, ch16 = 16 * (g & 1) + 4 * pp;
    const int tw0 = wid, tw1 = wid + 4;
    const int toffx0 = ((tw0 / 3) * FB_HW + tw0 % 3) * FB_XL, toffx1 = ((tw1 / 3) * FB_HW + tw1 % 3) * FB_XL;
    f32x16 accw[3];
#pragma unroll
    for (int t = 0; t < 3; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) accw[t][r] = 0.f;
    // dgrad epilogue: this lane's 8 channels (lane % 4) of the previous BatchNorm layer, for its sums
    BnsK bk[4];
    {
        const int c = (lane & 3) * 8;
#pragma unroll
        for (int q = 0; q < 4; ++q) {
            float v[4][2];
#pragma unroll
            for (int h = 0; h < 2; ++h) {
                const int ch = c + 2 * q + h;
                v[0][h] = p.psc[ch];
                v[1][h] = p.psh[ch];
                v[2][h] = p.pis[ch];
                v[3][h] = -p.pmu[ch] * p.pis[ch];
            }
            bk[q].sc = f32x2{v[0][0], v[0][1]};
            bk[q].sh = f32x2{v[1][0], v[1][1]};
            bk[q].is = f32x2{v[2][0], v[2][1]};
            bk[q].nmi = f32x2{v[3][0], v[3][1]};
        }
    }
    float own[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) own[j] = 0.f;
    __bf16* const scw = scr + wid * 32 * 32;
    auto swz = [](int j, int px) { return j ^ ((px >> 1) & 3); };
    unsigned long long tc[6] = {0, 0, 0, 0, 0, 0}, t0 = 0, t_all = FB_DG ? fb_clk() : 0;
    auto stamp = [&](int k) __attribute__((always_inline)) {
        if (FB_DG) {
            const unsigned long long t1 = fb_clk();
            tc[k] += t1 - t0;
            t0 = t1;
        }
    };
    // dgrad epilogue of a tile (acc: its C^T[ci][px], yv: the raw y_prev pieces of its stores): lanes l / l + 32 hold
    // the 4-channel halves of each 8-channel group of pixel l & 31; v_permlane32_swap pairs them into whole 16-B
    // pieces, which go through the wave's scratch and leave as pixel rows (16 pixels x 4 pieces per store
    // instruction), with the previous layer's BatchNorm-backward sums
    auto epilogue = [&](const f32x16& acc, const uint4* yv, int tl) __attribute__((always_inline)) {
        uint2 pk2[4];
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
            bf16x4 v;
#pragma unroll
            for (int q = 0; q < 4; ++q) v[q] = (__bf16)acc[4 * g4 + q];
            pk2[g4] = *reinterpret_cast<uint2*>(&v);
        }
#pragma unroll
        for (int k = 0; k < 4; k += 2) {
            const auto rx = __builtin_amdgcn_permlane32_swap(pk2[k].x, pk2[k + 1].x, false, false);
            const auto ry = __builtin_amdgcn_permlane32_swap(pk2[k].y, pk2[k + 1].y, false, false);
            const int px = lane & 31, j = k + (lane >> 5);
            *reinterpret_cast<uint4*>(scw + px * 32 + swz(j, px) * 8) = make_uint4(rx[0], ry[0], rx[1], ry[1]);
        }
        asm volatile("" ::: "memory");  // LDS is in order per wave: the reads below see the writes above
        int tx, ty, b;
        fb_tile(p.tiles_x, p.tiles_y, bid, gridDim.x, tl, tx, ty, b);
        const __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc(
            (void*)(p.dx + (size_t)b * hw * 32), (short)0, hw * 64, 0x00020000);
        uint4 vv[2];
#pragma unroll
        for (int rr = 0; rr < 2; ++rr) {
            const int px = rr * 16 + (lane >> 2), j = lane & 3;
            vv[rr] = *reinterpret_cast<const uint4*>(scw + px * 32 + swz(j, px) * 8);
        }
        asm volatile("" ::: "memory");  // the next tile's scratch writes after these reads
#pragma unroll
        for (int rr = 0; rr < 2; ++rr) {
            const int q = wid * 32 + rr * 16 + (lane >> 2), j = lane & 3;
            const int h = ty * FB_TH + q / FB_TW, w = tx * FB_TW + q % FB_TW;  // inside the image (H % 8, W % 16)
            bns_add(own, vv[rr], yv[rr], true, bk);
            __attribute__((ext_vector_type(4))) unsigned data = {vv[rr].x, vv[rr].y, vv[rr].z, vv[rr].w};
            __builtin_amdgcn_raw_buffer_store_b128(data, rd, (unsigned)(h * p.W + w) * 64u + (unsigned)j * 16u, 0, 2);
        }
    };
    // software pipeline: tile it - 1's epilogue (VALU, LDS, stores) sits between tile it's weight-gradient MFMAs in one
    // branch-free block (the first tile peeled), so its VALU issues in the MFMAs' shadow; its raw y_prev pieces were
    // read before the barrier that hands its buffer back
    f32x16 accp;
    uint4 yvp[2];
    auto tile = [&](int it, auto EPI) __attribute__((always_inline)) {
        if (FB_DG) t0 = fb_clk();
        __syncthreads();  // tile it is in buffer it & 1
        stamp(0);
        const __bf16* dyh = smem + (it & 1) * FB_BUF;
        const __bf16* xh = dyh + FB_DYH;
        const __bf16* st = xh + FB_XH;  // the raw y_prev of the tile (the sums' xhat and ReLU mask)
        // ---- weight gradient: k = the tile's pixels, one 16-pixel row per k-step; this wave's two tap-8 rows first
#pragma unroll
        for (int rr = 0; rr < FB_TH; ++rr) {
            const int r = (2 * wid + rr) & (FB_TH - 1);
            const __bf16* a0 = dyh + ((r + 1) * FB_HW + 1 + pk) * FB_DL + ch16;  // dy^T of row r
            const bf16x8 af = tr_pair(a0, a0 + 8 * FB_DL);
            const __bf16* xr = xh + (r * FB_HW + pk) * FB_XL + fb_xoff(ch16);
            const bf16x8 b0 = tr_pair(xr + toffx0, xr + toffx0 + 8 * FB_XL);
            const bf16x8 b1 = tr_pair(xr + toffx1, xr + toffx1 + 8 * FB_XL);
            accw[0] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, b0, accw[0], 0, 0, 0);
            accw[1] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, b1, accw[1], 0, 0, 0);
            if (rr < 2) {  // tap 8 on rows 2 wid, 2 wid + 1
                const __bf16* x8 = xr + (2 * FB_HW + 2) * FB_XL;
                accw[2] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, tr_pair(x8, x8 + 8 * FB_XL), accw[2], 0, 0, 0);
            }
            if constexpr (decltype(EPI)::v)
                if (rr == 2) epilogue(accp, yvp, t_begin + it - 1);
        }
        stamp(1);
        // ---- dgrad of tile pixels 32 wid ..: C^T[ci][px] over 9 taps x 2 k-steps of 16 dy channels
        f32x16 accd;
#pragma unroll
        for (int r = 0; r < 16; ++r) accd[r] = 0.f;
        const int c8 = 8 * (lane >> 5);
        const __bf16* wrow = wds + (lane & 31) * FB_WL + c8;
        const int qd = wid * 32 + (lane & 31);
        const __bf16* drow = dyh + ((qd / FB_TW) * FB_HW + qd % FB_TW) * FB_DL + c8;
#pragma unroll
        for (int tap = 0; tap < 9; ++tap) {
            const int toff = ((tap / 3) * FB_HW + tap % 3) * FB_DL;
#pragma unroll
            for (int kk = 0; kk < 2; ++kk) {
                const bf16x8 a = *reinterpret_cast<const bf16x8*>(wrow + tap * 32 + kk * 16);
                const bf16x8 b = *reinterpret_cast<const bf16x8*>(drow + toff + kk * 16);
                accd = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, accd, 0, 0, 0);
            }
        }
        accp = accd;
#pragma unroll
        for (int rr = 0; rr < 2; ++rr) {
            const int px = rr * 16 + (lane >> 2), j = lane & 3;
            yvp[rr] = *reinterpret_cast<const uint4*>(st + (wid * 32 + px) * FB_SL + j * 8);
        }
        stamp(2);
    };
    if (ntile > 0) tile(0, BoolC<false>{});
    for (int it = 1; it < ntile; ++it) tile(it, BoolC<true>{});
    if (ntile > 0) epilogue(accp, yvp, t_begin + ntile - 1);
    if (FB_DG && p.dbg && lane == 0) {
        unsigned long long* d = p.dbg + ((size_t)bid * 8 + wid) * 8;
#pragma unroll
        for (int k = 0; k < 6; ++k) d[k] = tc[k];
        d[6] = fb_clk() - t_all;
        d[7] = ntile;
    }
    if (ntile & 1) __syncthreads();  // the loaders' last (even-count) iteration

    // weight-gradient partial slab: slab[bid][co][tap * 32 + ci]   (32x32 C layout: element i of lane l is row
    // co = 8 (i / 4) + 4 (l / 32) + i % 4, column ci = l % 32); tap 8's four wave partials go through the LDS buffer
    // the last tile is not in (the loaders are past their last store; other MFMA waves may still read the last tile)
    float* slab = p.slab + (size_t)bid * 32 * 288;
    float* red8 = reinterpret_cast<float*>(smem + (ntile & 1) * FB_BUF);
    static_assert(FB_BUF * 2 >= 4 * 1024 * 4, "tap-8 partials fit one halo buffer");
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const int co = 8 * (i / 4) + 4 * (lane >> 5) + i % 4, ci = lane & 31;
        slab[(size_t)co * 288 + tw0 * 32 + ci] = accw[0][i];
        slab[(size_t)co * 288 + tw1 * 32 + ci] = accw[1][i];
        red8[wid * 1024 + co * 32 + ci] = accw[2][i];
    }
    // the previous layer's BatchNorm-backward sums: lanes l, l + 4, ... hold the same 8 channels
#pragma unroll
    for (int k = 0; k < 16; ++k)
#pragma unroll
        for (int o = 4; o < 64; o <<= 1) own[k] += __shfl_xor(own[k], o);
    if (lane < 4) {
#pragma unroll
        for (int k = 0; k < 16; ++k)  // k: channel k / 2, {sum, sum*xhat} k & 1 (bns_add's layout)
            redf[(wid * 32 + lane * 8 + k / 2) * 2 + (k & 1)] = own[(k & ~3) | ((k & 1) << 1) | ((k >> 1) & 1)];
    }
    __syncthreads();
#pragma unroll
    for (int e = tid; e < 1024; e += 256)
        slab[(size_t)(e >> 5) * 288 + 8 * 32 + (e & 31)] = (red8[e] + red8[1024 + e]) + (red8[2048 + e] + red8[3072 + e]);
    if (tid < 32) {
        float s = 0.f, sx = 0.f;
#pragma unroll
        for (int w = 0; w < 4; ++w) {
            s += redf[(w * 32 + tid) * 2];
            sx += redf[(w * 32 + tid) * 2 + 1];
        }
        p.part[(size_t)bid * 32 + tid] = make_float2(s, sx);
    }
}


// =====================================================================================================================
// Fused backward of the full-resolution decoder conv0 (dec1.0: cat(up1, enc1) 64 -> 32 channels + BatchNorm + ReLU,
// model.py:89-95 and 36-41). One pass produces
//   dy = BatchNorm-backward(da, y)       staged in LDS (bn_bwd_pk), never stored
//   dW = sum_px x[px + tap] dy[px]^T     x = cat(u, relu(bn_skip(y_skip))), split-K partial slab per block
//   dx = sum_tap dy[px + tap] Wd[tap]    64 channels, stored as the two tensors the cat backward hands on: d(up)
//                                        (ConvTranspose2d backward) and d(skip) (the encoder's pool-backward add)
//   the column sums of d(up) (the ConvTranspose2d bias gradient), one partial row per block
// It replaces the fused BatchNorm-backward weight gradient over two 32-channel x blocks (k_halo_wgrad_ws<32, 32, ...,
// BNB>: each block re-formed dy from (da, y) and one wrote dy) and the SPLIT_STATS dgrad that read dy back:
// per launch da, y, u, y_skip in and d(up), d(skip) out, 1.9 GB at B = 64 instead of 2.9 GB.
// Block structure as k_bwd_fused32 (4 loader + 4 MFMA waves, 8x16 tiles in column-strip order, one block per CU):
//   loaders: per halo item (pixel, 8 channels) da, y, u, y_skip -> dy, x_up, x_skip into the LDS double buffer;
//   MFMA waves: weight gradient: wave w owns x half w & 1 (up / skip) and taps 4 (w >> 1) .. + 3 over the tile's 8
//   rows, plus tap 8 over rows 4 (w >> 1) .. + 3 (the wave pair's partials summed at the end); dgrad: 32 pixels x 64
//   ci per wave (two 32x32 accumulators over 9 taps x 32 dy channels, weights resident in LDS); its epilogue runs
//   behind the next tile's weight-gradient MFMAs.
struct DecArgs {
    const __bf16 *da, *y, *xu, *xs;         // [B*H*W][32]: this layer's da and raw y; u; the skip layer's raw y
    const float *sc, *sh, *mu, *is, *coef;  // this layer's BatchNorm: forward affine, statistics, backward coef
    const float *ssc, *ssh;                 // the skip layer's forward affine (x_skip = relu(ssc*xs + ssh))
    const __bf16* wd;                       // dgrad-packed weights [64 ci][kpad], k = tap*32 + co (flipped)
    int kpad;
    int B, H, W, tiles_x, tiles_y;
    __bf16 *du, *dsk;                       // [B*H*W][32] each
    float* slab;                            // [blocks][32 co][576], k = tap*64 + ci
    float2* part;                           // [blocks][32]: (sum d(up), 0) per channel
    unsigned long long* dbg;                // timing build only: [block][wave][8] phase cycles
};
constexpr int FD_BUF = FB_DYH + 2 * FB_XH;  // dy, x_up, x_skip halos

__global__ __launch_bounds__(512) void k_bwd_fused_dec(const DecArgs p) {
    __shared__ __attribute__((aligned(16))) __bf16 smem[2 * FD_BUF];
    __shared__ __attribute__((aligned(16))) __bf16 wds[64 * FB_WL];
    __shared__ __attribute__((aligned(16))) __bf16 scr[4 * 32 * 32];  // per-wave dgrad epilogue transpose
    __shared__ __attribute__((aligned(16))) float redf[4 * 32];

    const int tid = threadIdx.x, lane = tid & 63;
    const bool is_loader = tid >= 256;
    const int wid = (tid >> 6) & 3;
    const int bid = (blockIdx.x & 7) * (gridDim.x >> 3) + (blockIdx.x >> 3);  // XCD-contiguous tile ranges
    const int t_begin = 0;  // tiles are numbered per block (fb_tile)
    const int ntile = fb_ntile(p.tiles_x, p.tiles_y, p.B, bid, gridDim.x);
    const int hw = p.H * p.W;
    auto tile_of = [&](int tl, int& tx, int& ty, int& b) __attribute__((always_inline)) {
        fb_tile(p.tiles_x, p.tiles_y, bid, gridDim.x, tl, tx, ty, b);
    };

    for (int i = tid; i < 64 * 36; i += 512) {  // the dgrad weights, resident for the launch
        const int r = i / 36, c8 = i - r * 36;
        *reinterpret_cast<uint4*>(wds + r * FB_WL + c8 * 8) =
            *reinterpret_cast<const uint4*>(p.wd + (size_t)r * p.kpad + c8 * 8);
    }

    if (is_loader) {
        // =========================================================== loader waves
        const int ltid = tid - 256;
        const int piece = fb_piece<4>(ltid);
        constexpr unsigned OOB = 0x80000000u;
        float ksc[8], ksh[8], kB[8], kC[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const int c = piece * 8 + j;
            const float k1 = p.coef[3 * c + 1], k2 = p.coef[3 * c + 2], is = p.is[c], sc = p.sc[c], sh = p.sh[c];
            ksc[j] = sc;
            ksh[j] = sh;
            kB[j] = -is * k2;
            kC[j] = is * k2 * sh + sc * (p.mu[c] * is * k2 - k1);
        }
        const float4 s0 = *reinterpret_cast<const float4*>(p.ssc + piece * 8);
        const float4 s1 = *reinterpret_cast<const float4*>(p.ssc + piece * 8 + 4);
        const float4 t0 = *reinterpret_cast<const float4*>(p.ssh + piece * 8);
        const float4 t1 = *reinterpret_cast<const float4*>(p.ssh + piece * 8 + 4);
        unsigned geo[FB_NI];
#pragma unroll
        for (int i = 0; i < FB_NI; ++i) {
            const int px = fb_pixel<4>(ltid + 256 * i);
            const int hy = px / FB_HW, hx = px - hy * FB_HW;
            geo[i] = px < FB_HPX ? (unsigned)(hy << 8 | hx) : 0xffffffffu;
        }
        const bool w3 = (ltid & ~63) + 256 * (FB_NI - 1) < FB_HPX * 4;
        unsigned need = 0;
#pragma unroll
        for (int i = 0; i < FB_NI; ++i) need |= (unsigned)(geo[i] != 0xffffffffu) << i;
        struct Set {
            uint4 a[FB_NI], y[FB_NI], u[FB_NI], s[FB_NI];
            unsigned m;
            bool edge;
        };
        Set sa, sb;
        auto load = [&](Set& q, int tile) __attribute__((always_inline)) {
            const bool live = tile < t_begin + ntile;
            int tx, ty, b;
            tile_of(live ? tile : t_begin, tx, ty, b);
            const int h0 = ty * FB_TH - 1, w0 = tx * FB_TW - 1;
            const size_t img = (size_t)b * hw * 32;
            const __amdgpu_buffer_rsrc_t ra =
                __builtin_amdgcn_make_buffer_rsrc((void*)(p.da + img), (short)0, hw * 64, 0x00020000);
            const __amdgpu_buffer_rsrc_t ry =
                __builtin_amdgcn_make_buffer_rsrc((void*)(p.y + img), (short)0, hw * 64, 0x00020000);
            const __amdgpu_buffer_rsrc_t ru =
                __builtin_amdgcn_make_buffer_rsrc((void*)(p.xu + img), (short)0, hw * 64, 0x00020000);
            const __amdgpu_buffer_rsrc_t rs =
                __builtin_amdgcn_make_buffer_rsrc((void*)(p.xs + img), (short)0, hw * 64, 0x00020000);
            unsigned m = 0;
#pragma unroll
            for (int i = 0; i < FB_NI; ++i) {
                if (i == FB_NI - 1 && !w3) break;
                const int h = h0 + (int)(geo[i] >> 8), w = w0 + (int)(geo[i] & 0xffu);
                const bool ok = live & (geo[i] != 0xffffffffu) & (h >= 0) & (h < p.H) & (w >= 0) & (w < p.W);
                m |= (unsigned)ok << i;
                const unsigned off = ok ? (unsigned)(h * p.W + w) * 64u + (unsigned)piece * 16u : OOB;
                const auto va = __builtin_amdgcn_raw_buffer_load_b128(ra, off, 0, 0);
                const auto vy = __builtin_amdgcn_raw_buffer_load_b128(ry, off, 0, 0);
                const auto vu = __builtin_amdgcn_raw_buffer_load_b128(ru, off, 0, 0);
                const auto vs = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0);
                q.a[i] = make_uint4(va[0], va[1], va[2], va[3]);
                q.y[i] = make_uint4(vy[0], vy[1], vy[2], vy[3]);
                q.u[i] = make_uint4(vu[0], vu[1], vu[2], vu[3]);
                q.s[i] = make_uint4(vs[0], vs[1], vs[2], vs[3]);
            }
            q.m = m;
            q.edge = __builtin_amdgcn_ballot_w64(m != (w3 ? need : need & ((1u << (FB_NI - 1)) - 1))) != 0;
        };
        auto store = [&](Set& q, int buf) __attribute__((always_inline)) {
            __bf16* dyh = smem + buf * FD_BUF;
            __bf16* xuh = dyh + FB_DYH;
            __bf16* xsh = xuh + FB_XH;
            auto put = [&](auto SEL) __attribute__((always_inline)) {
#pragma unroll
                for (int i = 0; i < FB_NI; ++i) {
                    if (i == FB_NI - 1 && !w3) break;
                    const bool ok = (q.m >> i) & 1u;
                    const int px = fb_pixel<4>(ltid + 256 * i);
                    uint4 d = bn_bwd_pk(q.a[i], q.y[i], ksc, ksh, kB, kC);
                    uint4 xs = bnrelu_pk(q.s[i], s0, s1, t0, t1);
                    uint4 xu = q.u[i];
                    if constexpr (decltype(SEL)::v) {  // zero padding (and dy past the image)
                        d = ok ? d : make_uint4(0, 0, 0, 0);
                        xs = ok ? xs : make_uint4(0, 0, 0, 0);
                        xu = ok ? xu : make_uint4(0, 0, 0, 0);
                    }
                    *reinterpret_cast<uint4*>(dyh + px * FB_DL + piece * 8) = d;
                    *reinterpret_cast<uint4*>(xuh + px * FB_XL + fb_xoff(piece * 8)) = xu;
                    *reinterpret_cast<uint4*>(xsh + px * FB_XL + fb_xoff(piece * 8)) = xs;
                }
            };
            if (q.edge)
                put(BoolC<true>{});
            else
                put(BoolC<false>{});
        };
        load(sa, t_begin);
        __builtin_amdgcn_sched_barrier(0);
        load(sb, t_begin + 1);
        __syncthreads();  // the resident weights
        unsigned long long tc[3] = {0, 0, 0}, tm0 = 0, t_all = FB_DG ? fb_clk() : 0;
        auto stamp = [&](int k) __attribute__((always_inline)) {
            if (FB_DG) {
                const unsigned long long t1 = fb_clk();
                tc[k] += t1 - tm0;
                tm0 = t1;
            }
        };
        for (int i = 0; i < ntile; i += 2) {  // as k_bwd_fused32: an even number of iterations
            if (FB_DG) tm0 = fb_clk();
            store(sa, 0);
            stamp(0);
            load(sa, t_begin + i + 2);
            stamp(1);
            __syncthreads();
            stamp(2);
            store(sb, 1);
            stamp(0);
            load(sb, t_begin + i + 3);
            stamp(1);
            __syncthreads();
            stamp(2);
        }
        if (FB_DG && p.dbg && lane == 0) {
            unsigned long long* d = p.dbg + ((size_t)bid * 8 + 4 + wid) * 8;
            d[0] = tc[0];
            d[1] = tc[1];
            d[2] = tc[2];
            d[3] = 0;
            d[4] = fb_clk() - t_all;
            d[5] = ntile;
        }
        __syncthreads();  // the final reductions (MFMA waves)
        return;
    }

    // =============================================================== MFMA waves
    __syncthreads();  // the resident weights
    const int g = lane >> 4, q4 = (lane & 15) >> 2, pp = lane & 3;
    const int pk = 4 * (g >> 1) + q4, ch16 = 16 * (g & 1) + 4 * pp;  // tr_pair addressing as k_bwd_fused32
    const int hh = wid & 1, tg = wid >> 1;                            // x half, tap group
    int toffx[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        const int t = 4 * tg + j;
        toffx[j] = ((t / 3) * FB_HW + t % 3) * FB_XL;
    }
    f32x16 accw[5];
#pragma unroll
    for (int t = 0; t < 5; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) accw[t][r] = 0.f;
    float ownb[8];  // column sums of d(up): channels 8 (lane & 3) ..
#pragma unroll
    for (int j = 0; j < 8; ++j) ownb[j] = 0.f;
    __bf16* const scw = scr + wid * 32 * 32;
    auto swz = [](int j, int px) { return j ^ ((px >> 1) & 3); };
    auto epilogue = [&](const f32x16& acc, __bf16* out, bool bias, int tl) __attribute__((always_inline)) {
        uint2 pk2[4];
#pragma unroll
        for (int g4 = 0; g4 < 4; ++g4) {
            bf16x4 v;
#pragma unroll
            for (int q = 0; q < 4; ++q) v[q] = (__bf16)acc[4 * g4 + q];
            pk2[g4] = *reinterpret_cast<uint2*>(&v);
        }
#pragma unroll
        for (int k = 0; k < 4; k += 2) {
            const auto rx = __builtin_amdgcn_permlane32_swap(pk2[k].x, pk2[k + 1].x, false, false);
            const auto ry = __builtin_amdgcn_permlane32_swap(pk2[k].y, pk2[k + 1].y, false, false);
            const int px = lane & 31, j = k + (lane >> 5);
            *reinterpret_cast<uint4*>(scw + px * 32 + swz(j, px) * 8) = make_uint4(rx[0], ry[0], rx[1], ry[1]);
        }
        asm volatile("" ::: "memory");
        int tx, ty, b;
        tile_of(tl, tx, ty, b);
        const __amdgpu_buffer_rsrc_t rd =
            __builtin_amdgcn_make_buffer_rsrc((void*)(out + (size_t)b * hw * 32), (short)0, hw * 64, 0x00020000);
        uint4 vv[2];
#pragma unroll
        for (int rr = 0; rr < 2; ++rr) {
            const int px = rr * 16 + (lane >> 2), j = lane & 3;
            vv[rr] = *reinterpret_cast<const uint4*>(scw + px * 32 + swz(j, px) * 8);
        }
        asm volatile("" ::: "memory");  // the next scratch writes after these reads
#pragma unroll
        for (int rr = 0; rr < 2; ++rr) {
            const int q = wid * 32 + rr * 16 + (lane >> 2), j = lane & 3;
            const int h = ty * FB_TH + q / FB_TW, w = tx * FB_TW + q % FB_TW;
            if (bias) {
                const unsigned wv[4] = {vv[rr].x, vv[rr].y, vv[rr].z, vv[rr].w};
#pragma unroll
                for (int e = 0; e < 4; ++e) {
                    ownb[2 * e] += __uint_as_float(wv[e] << 16);
                    ownb[2 * e + 1] += __uint_as_float(wv[e] & 0xffff0000u);
                }
            }
            __attribute__((ext_vector_type(4))) unsigned data = {vv[rr].x, vv[rr].y, vv[rr].z, vv[rr].w};
            __builtin_amdgcn_raw_buffer_store_b128(data, rd, (unsigned)(h * p.W + w) * 64u + (unsigned)j * 16u, 0, 2);
        }
    };
    unsigned long long tc[4] = {0, 0, 0, 0}, t0 = 0, t_all = FB_DG ? fb_clk() : 0;
    auto stamp = [&](int k) __attribute__((always_inline)) {
        if (FB_DG) {
            const unsigned long long t1 = fb_clk();
            tc[k] += t1 - t0;
            t0 = t1;
        }
    };
    f32x16 accp0, accp1;
    auto tile = [&](int it, auto EPI) __attribute__((always_inline)) {  // as k_bwd_fused32's: branch-free, first peeled
        if (FB_DG) t0 = fb_clk();
        __syncthreads();  // tile it is in buffer it & 1
        stamp(0);
        const __bf16* dyh = smem + (it & 1) * FD_BUF;
        const __bf16* xsrc = dyh + FB_DYH + hh * FB_XH;
        // ---- weight gradient: one 16-pixel row per k-step, 4 taps of this wave's x half (+ tap 8 on its 4 rows,
        // first); tile it - 1's two epilogue halves between the rows
#pragma unroll
        for (int rr = 0; rr < FB_TH; ++rr) {
            const int r = (4 * tg + rr) & (FB_TH - 1);
            const __bf16* a0 = dyh + ((r + 1) * FB_HW + 1 + pk) * FB_DL + ch16;
            const bf16x8 af = tr_pair(a0, a0 + 8 * FB_DL);
            const __bf16* xr = xsrc + (r * FB_HW + pk) * FB_XL + fb_xoff(ch16);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const bf16x8 bfr = tr_pair(xr + toffx[j], xr + toffx[j] + 8 * FB_XL);
                accw[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, bfr, accw[j], 0, 0, 0);
            }
            if (rr < 4) {
                const __bf16* x8 = xr + (2 * FB_HW + 2) * FB_XL;
                accw[4] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(af, tr_pair(x8, x8 + 8 * FB_XL), accw[4], 0, 0, 0);
            }
            if constexpr (decltype(EPI)::v) {
                if (rr == 1) epilogue(accp0, p.du, true, t_begin + it - 1);
                if (rr == 5) epilogue(accp1, p.dsk, false, t_begin + it - 1);
            }
        }
        stamp(1);
        // ---- dgrad of tile pixels 32 wid ..: C^T[ci][px], ci halves up / skip
        f32x16 accd0, accd1;
#pragma unroll
        for (int r = 0; r < 16; ++r) accd0[r] = accd1[r] = 0.f;
        const int c8 = 8 * (lane >> 5);
        const __bf16* wrow = wds + (lane & 31) * FB_WL + c8;
        const int qd = wid * 32 + (lane & 31);
        const __bf16* drow = dyh + ((qd / FB_TW) * FB_HW + qd % FB_TW) * FB_DL + c8;
#pragma unroll
        for (int tap = 0; tap < 9; ++tap) {
            const int toff = ((tap / 3) * FB_HW + tap % 3) * FB_DL;
#pragma unroll
            for (int kk = 0; kk < 2; ++kk) {
                const bf16x8 bdy = *reinterpret_cast<const bf16x8*>(drow + toff + kk * 16);
                const bf16x8 a0 = *reinterpret_cast<const bf16x8*>(wrow + tap * 32 + kk * 16);
                const bf16x8 a1 = *reinterpret_cast<const bf16x8*>(wrow + 32 * FB_WL + tap * 32 + kk * 16);
                accd0 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a0, bdy, accd0, 0, 0, 0);
                accd1 = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a1, bdy, accd1, 0, 0, 0);
            }
        }
        accp0 = accd0;
        accp1 = accd1;
        stamp(2);
    };
    if (ntile > 0) tile(0, BoolC<false>{});
    for (int it = 1; it < ntile; ++it) tile(it, BoolC<true>{});
    if (FB_DG && p.dbg && lane == 0) {
        unsigned long long* d = p.dbg + ((size_t)bid * 8 + wid) * 8;
#pragma unroll
        for (int k = 0; k < 4; ++k) d[k] = tc[k];
        d[4] = d[5] = 0;
        d[6] = fb_clk() - t_all;
        d[7] = ntile;
    }
    if (ntile > 0) {
        epilogue(accp0, p.du, true, t_begin + ntile - 1);
        epilogue(accp1, p.dsk, false, t_begin + ntile - 1);
    }
    if (ntile & 1) __syncthreads();  // the loaders' last (even-count) iteration

    // weight-gradient partial slab: slab[bid][co][tap * 64 + ci] (32x32 C layout as k_bwd_fused32); tap 8's partials
    // of the two waves of an x half go through the LDS buffer the last tile is not in
    float* slab = p.slab + (size_t)bid * 32 * 576;
    float* red8 = reinterpret_cast<float*>(smem + (ntile & 1) * FD_BUF);
    static_assert(FD_BUF * 2 >= 4 * 1024 * 4, "tap-8 partials fit one halo buffer");
#pragma unroll
    for (int i = 0; i < 16; ++i) {
        const int co = 8 * (i / 4) + 4 * (lane >> 5) + i % 4, ci = hh * 32 + (lane & 31);
#pragma unroll
        for (int j = 0; j < 4; ++j) slab[(size_t)co * 576 + (4 * tg + j) * 64 + ci] = accw[j][i];
        red8[wid * 1024 + co * 32 + (lane & 31)] = accw[4][i];
    }
    // column sums of d(up): lanes l, l + 4, ... hold the same 8 channels
#pragma unroll
    for (int k = 0; k < 8; ++k)
#pragma unroll
        for (int o = 4; o < 64; o <<= 1) ownb[k] += __shfl_xor(ownb[k], o);
    if (lane < 4) {
#pragma unroll
        for (int k = 0; k < 8; ++k) redf[wid * 32 + lane * 8 + k] = ownb[k];
    }
    __syncthreads();
    for (int e = tid; e < 2 * 1024; e += 256) {  // e = hh * 1024 + co * 32 + ci; waves hh and hh + 2 hold tap 8
        const int h2 = e >> 10, r = e & 1023;
        slab[(size_t)(r >> 5) * 576 + 8 * 64 + h2 * 32 + (r & 31)] = red8[h2 * 1024 + r] + red8[(h2 + 2) * 1024 + r];
    }
    if (tid < 32)
        p.part[(size_t)bid * 32 + tid] =
            make_float2((redf[tid] + redf[32 + tid]) + (redf[64 + tid] + redf[96 + tid]), 0.f);
}

}  // namespace

unsigned long long* sd_debug_ptr();

extern "C" int sd_conv3x3_bwd_fused_ok(int C, int Cx, int H, int W) {
    return C == 32 && Cx == 32 && H % FB_TH == 0 && W % FB_TW == 0 && W / FB_TW < 256 && (long long)H * W * 64 < (1LL << 31)
               ? 1
               : 0;
}

extern "C" int sd_conv3x3_bwd_fused_splits(int batch, int H, int W) {
    const long long ns = (long long)batch * (W / FB_TW);  // column strips: the blocks' unit of work (fb_tile)
    return ns < FB_BLOCKS ? (int)((ns + 7) / 8 * 8) : FB_BLOCKS;
}

extern "C" int sd_conv3x3_bwd_fused(const void* da, const void* y, const float* scale, const float* shift,
                                    const float* mean, const float* invstd, const float* coef, const void* yp,
                                    const float* pscale, const float* pshift, const float* pmean, const float* pinvstd,
                                    const void* wd, int kpad, int batch, int H, int W, void* dx, float* slab,
                                    float* partials, sd_stream s) {
    SD_REQUIRE(sd_conv3x3_bwd_fused_ok(32, 32, H, W) == 1 && batch > 0,
               "sd_conv3x3_bwd_fused: 32 -> 32 channels, H %% %d == 0, W %% %d == 0 (got %dx%d)", FB_TH, FB_TW, H, W);
    SD_REQUIRE(da && y && scale && shift && mean && invstd && coef && yp && pscale && pshift && pmean && pinvstd && wd &&
                   dx && slab && partials && kpad >= 288,
               "sd_conv3x3_bwd_fused: bad args");
    BwdArgs p;
    p.da = (const __bf16*)da;
    p.y = (const __bf16*)y;
    p.yp = (const __bf16*)yp;
    p.sc = scale;
    p.sh = shift;
    p.mu = mean;
    p.is = invstd;
    p.coef = coef;
    p.psc = pscale;
    p.psh = pshift;
    p.pmu = pmean;
    p.pis = pinvstd;
    p.wd = (const __bf16*)wd;
    p.kpad = kpad;
    p.B = batch;
    p.H = H;
    p.W = W;
    p.tiles_x = W / FB_TW;
    p.tiles_y = H / FB_TH;
    const long long nt = (long long)batch * p.tiles_x * p.tiles_y;
    SD_REQUIRE(nt < (1LL << 30), "sd_conv3x3_bwd_fused: too many tiles");
    const int blocks = sd_conv3x3_bwd_fused_splits(batch, H, W);
    p.dx = (__bf16*)dx;
    p.slab = slab;
    p.part = reinterpret_cast<float2*>(partials);
    p.dbg = FB_DG ? sd_debug_ptr() : nullptr;
    hipLaunchKernelGGL(k_bwd_fused32, dim3(blocks), dim3(512), 0, to_stream(s), p);
    return sd_check_launch("sd_conv3x3_bwd_fused");
}

extern "C" int sd_conv3x3_bwd_fused_dec_ok(int C, int Cu, int Cs, int H, int W) {
    return C == 32 && Cu == 32 && Cs == 32 && sd_conv3x3_bwd_fused_ok(32, 32, H, W) == 1 ? 1 : 0;
}

extern "C" int sd_conv3x3_bwd_fused_dec(const void* da, const void* y, const float* scale, const float* shift,
                                        const float* mean, const float* invstd, const float* coef, const void* xu,
                                        const void* xs, const float* sscale, const float* sshift, const void* wd,
                                        int kpad, int batch, int H, int W, void* du, void* dskip, float* slab,
                                        float* partials, sd_stream s) {
    SD_REQUIRE(sd_conv3x3_bwd_fused_dec_ok(32, 32, 32, H, W) == 1 && batch > 0,
               "sd_conv3x3_bwd_fused_dec: 32 + 32 -> 32 channels, H %% %d == 0, W %% %d == 0 (got %dx%d)", FB_TH,
               FB_TW, H, W);
    SD_REQUIRE(da && y && scale && shift && mean && invstd && coef && xu && xs && sscale && sshift && wd && du &&
                   dskip && slab && partials && kpad >= 288,
               "sd_conv3x3_bwd_fused_dec: bad args");
    DecArgs p;
    p.da = (const __bf16*)da;
    p.y = (const __bf16*)y;
    p.xu = (const __bf16*)xu;
    p.xs = (const __bf16*)xs;
    p.sc = scale;
    p.sh = shift;
    p.mu = mean;
    p.is = invstd;
    p.coef = coef;
    p.ssc = sscale;
    p.ssh = sshift;
    p.wd = (const __bf16*)wd;
    p.kpad = kpad;
    p.B = batch;
    p.H = H;
    p.W = W;
    p.tiles_x = W / FB_TW;
    p.tiles_y = H / FB_TH;
    const long long nt = (long long)batch * p.tiles_x * p.tiles_y;
    SD_REQUIRE(nt < (1LL << 30), "sd_conv3x3_bwd_fused_dec: too many tiles");
    const int blocks = sd_conv3x3_bwd_fused_splits(batch, H, W);
    p.du = (__bf16*)du;
    p.dsk = (__bf16*)dskip;
    p.slab = slab;
    p.part = reinterpret_cast<float2*>(partials);
    p.dbg = FB_DG ? sd_debug_ptr() : nullptr;
    hipLaunchKernelGGL(k_bwd_fused_dec, dim3(blocks), dim3(512), 0, to_stream(s), p);
    return sd_check_launch("sd_conv3x3_bwd_fused_dec");
}
