// fp8 (OCP e4m3) 3x3 convolution of the live-camera inference forward with STATIC activation scales
// (depth_live_dl.py:516-529 -> model.py:79-104 in eval mode; SURVEY §8f row 2, BASELINE config 5).
//
// The engine calibrates once per model state: its first eval forward runs the dynamic path (conv_fp8.hip: per-layer
// (min, max) rows and sd_fp8_qparams), which leaves every conv input's activation scale s_a and the folded per-channel
// quantisation affine q = y*qs + qh (BN eval coefficients / s_a). While the parameters and BN buffers stay unchanged
// (the live app's loop) the forwards reuse them and run this kernel alone: no min/max passes, no per-layer scale
// reductions, 18 fewer launches.
//
// Structure: the bf16 halo kernel's (conv_halo.hip) r02 design, on e4m3 operands. One 512-thread block per CU,
// persistent over (spatial tile, N-block) items. Loader waves 4-7: global bf16 -> registers (two chunks in flight,
// 32-bit buffer offsets, out-of-range pieces = zeros with no traffic, the same loads on every path so the compiler's
// vmcnt bookkeeping stays exact) -> quantise (fma, med3 clamp with the ReLU folded in, v_cvt_pk_fp8_f32) -> LDS double
// buffer. MFMA waves 0-3: v_mfma_scale_f32_32x32x64_f8f6f4 (unit block scales), one k-step per tap of a 64-channel
// chunk, computing C^T (channels x pixels), then the dequantised (s_a * s_w[co]) bf16 tile goes through the wave's
// LDS scratch and leaves as whole-pixel 16-B nontemporal stores.
// A 64-channel chunk is 64 e4m3 bytes per halo pixel, the LDS footprint of a 32-channel bf16 chunk: the MFMA does
// twice the channels per k-step at the same LDS traffic, and a layer needs half the chunks.
#include <type_traits>

#include "common.h"

namespace {

typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int QC = 64;             // channels per chunk
constexpr int QHX = 80;            // halo pixel stride in LDS, bytes (5 16-B slots: odd, conflict-free fragment reads)
constexpr int QW = 9 * QC + 16;    // weight row stride, bytes (37 slots, odd)
constexpr int QSBN = 512;          // input channels (LDS quantisation affine)
constexpr int QPPX = 4;            // 16-B (16-channel) pieces per halo pixel
constexpr int QPERSIST = 256;      // one block per CU
constexpr float Q8_MAX = 448.f;    // largest finite OCP e4m3fn value
__host__ __device__ constexpr int q_halo_cap(int RT) { return RT == 4 ? 640 : 384; }

struct QArgs {
    const __bf16* p0;
    const __bf16* p1;
    const float *qs0, *qh0, *qs1, *qh1;  // per-channel quantisation affine of each source: q = y*qs + qh
    int c0, c1, relu0, relu1;
    int H, W;             // image (GEMM grid)
    int th, tw, tiles_x;  // spatial tile and tiling
    int tiles, nsp;       // tiles per image, batch * tiles
    int nblk, gper;       // N-blocks, blocks per N-block
    int hw, nhalo;        // halo width (tw+2) and pixel count ((th+2)*(tw+2))
    const uint8_t* wq;    // [co][kpad] e4m3, k = tap*ctap + c
    const float* wscale;  // [co]
    const float* act_scale;  // [1]: s_a of this conv's input
    int N, kpad, ctap;
    __bf16* out;
    int xcd;              // XCD-contiguous block numbering (grid % 8 == 0)
};

// 16 bf16 channels (lo: 0-7, hi: 8-15) -> 16 e4m3 bytes: med3(y*qs + qh, lo_clamp, 448), lo_clamp = 0 for a ReLU
// source (relu and the upper clamp in one v_med3_f32), -448 for a signed one
__device__ __forceinline__ uint4 quant16(uint4 lo, uint4 hi, const float* s, const float* h, float lo_clamp) {
    const unsigned w[8] = {lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
    float v[16];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        v[2 * i] = __builtin_amdgcn_fmed3f(__builtin_fmaf(__uint_as_float(w[i] << 16), s[2 * i], h[2 * i]), lo_clamp, Q8_MAX);
        v[2 * i + 1] = __builtin_amdgcn_fmed3f(__builtin_fmaf(__uint_as_float(w[i] & 0xffff0000u), s[2 * i + 1], h[2 * i + 1]),
                                               lo_clamp, Q8_MAX);
    }
    unsigned o[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        int x = __builtin_amdgcn_cvt_pk_fp8_f32(v[4 * i], v[4 * i + 1], 0, false);
        x = __builtin_amdgcn_cvt_pk_fp8_f32(v[4 * i + 2], v[4 * i + 3], x, true);
        o[i] = (unsigned)x;
    }
    return make_uint4(o[0], o[1], o[2], o[3]);
}

__device__ __forceinline__ i32x8 qfrag(const uint8_t* p) {
    const uint4 a = *reinterpret_cast<const uint4*>(p);
    const uint4 b = *reinterpret_cast<const uint4*>(p + 16);
    return i32x8{(int)a.x, (int)a.y, (int)a.z, (int)a.w, (int)b.x, (int)b.y, (int)b.z, (int)b.w};
}

// loader piece item -> halo pixel / 16-B piece: each 8-lane group takes 8 consecutive pixels at one piece (distinct
// bank slots at the odd 5-slot pixel stride), the piece is fixed per thread (item = ltid + 256 * i)
__device__ __forceinline__ int q_pixel(int item) { return (item / (8 * QPPX)) * 8 + (item & 7); }
__device__ __forceinline__ int q_piece(int item) { return (item >> 3) % QPPX; }

template <int NT, int RT, bool WCONST>
__global__ __launch_bounds__(512) void k_halo_conv_q8(const QArgs p) {
    constexpr int BN = 32 * NT;
    constexpr int HPX = q_halo_cap(RT);
    constexpr int HP = HPX * QPPX / 256;      // halo pieces per loader thread
    constexpr int WPIECES = BN * 9 * QPPX;    // 16-B weight pieces per chunk
    constexpr int WPT = (WPIECES + 255) / 256;
    constexpr int HALO_B = HPX * QHX, W_B = BN * QW, BUF = HALO_B + W_B;
    static_assert(HP * 256 == HPX * QPPX, "the loader pieces tile the halo region exactly");
    __shared__ __attribute__((aligned(16))) uint8_t smem[2 * BUF];
    __shared__ __attribute__((aligned(16))) __bf16 scr[4 * 32 * BN];  // epilogue transpose, 32 pixels per MFMA wave
    __shared__ __attribute__((aligned(16))) float sq[2 * QSBN + 2 * QC];  // qs | qh per input channel (+ a chunk tail)
    __shared__ __attribute__((aligned(16))) float deq[BN];               // s_a * s_w[co]

    const int tid = threadIdx.x, lane = tid & 63;
    const bool is_loader = (tid >> 6) >= 4;
    const int wid = (tid >> 6) & 3;
    const int bid = p.xcd ? (blockIdx.x & 7) * (gridDim.x >> 3) + (blockIdx.x >> 3) : blockIdx.x;
    const int nb = bid % p.nblk, slot = bid / p.nblk;
    const int n0 = nb * BN;
    // chunks never straddle the two sources (a source's last chunk may be partial)
    const int nc0 = (p.c0 + QC - 1) / QC;
    const int nchunks = nc0 + (p.c1 + QC - 1) / QC;
    constexpr int c_lo = 0;
    const int mvalid = p.th * p.tw;
    const int my_items = slot < p.nsp ? (p.nsp - 1 - slot) / p.gper + 1 : 0;
    const int total = my_items * nchunks;
    constexpr int LS = 2;  // loader register sets
    const int padded = (total + LS - 1) / LS * LS;
    const int ctot = p.c0 + p.c1;
    // filled by both roles before the launch's first barrier, the loaders' after they issued their first loads (one
    // memory latency for the tables, weights and first halos: the serial latencies are what a batch-1 launch costs)
    auto fill_tables = [&]() __attribute__((always_inline)) {
        for (int c = tid; c < ctot; c += 512) {
            const bool first = c < p.c0;
            const int cl = first ? c : c - p.c0;
            sq[c] = (first ? p.qs0 : p.qs1)[cl];
            sq[QSBN + c] = (first ? p.qh0 : p.qh1)[cl];
        }
        if (tid < BN) deq[tid] = n0 + tid < p.N ? p.act_scale[0] * p.wscale[n0 + tid] : 0.f;
    };

    if (is_loader) {
        // ================================================================= loader waves
        const int ltid = wid * 64 + lane;
        constexpr unsigned OOB = 0x80000000u;
        const int hw_img = p.H * p.W;
        const int lpiece = q_piece(ltid);
        unsigned pgeo[HP];  // (halo row << 16 | halo col) of each piece, ~0 past the halo
#pragma unroll
        for (int i = 0; i < HP; ++i) {
            const int px = q_pixel(ltid + i * 256);
            const int hy = px / p.hw;
            pgeo[i] = px < p.nhalo ? ((unsigned)hy << 16) | (unsigned)(px - hy * p.hw) : 0xffffffffu;
        }
        int hpx[HP];  // image-local pixel of each piece for the item being loaded, -1 outside the image
        const __bf16* ib0 = p.p0;
        const __bf16* ib1 = p.p0;
        int ld_item = 0, ld_cc = 0;
        auto geometry = [&]() __attribute__((always_inline)) {
            const bool live = ld_item < my_items;  // past the last item: every piece out of range, no traffic
            const int sp = slot + (live ? ld_item : 0) * p.gper;
            const int b = sp / p.tiles, tl = sp - b * p.tiles;
            const int ty = tl / p.tiles_x;
            const int h0 = ty * p.th - 1, w0 = (tl - ty * p.tiles_x) * p.tw - 1;
            ib0 = p.p0 + (size_t)b * hw_img * p.c0;
            ib1 = p.c1 ? p.p1 + (size_t)b * hw_img * p.c1 : p.p0;
#pragma unroll
            for (int i = 0; i < HP; ++i) {
                const int h = h0 + (int)(pgeo[i] >> 16), w = w0 + (int)(pgeo[i] & 0xffffu);
                const bool in = live & (pgeo[i] != 0xffffffffu) & (h >= 0) & (w >= 0) & (h < p.H) & (w < p.W);
                hpx[i] = in ? h * p.W + w : -1;
            }
        };
        const __amdgpu_buffer_rsrc_t wrs = __builtin_amdgcn_make_buffer_rsrc((void*)p.wq, (short)0, p.N * p.kpad, 0x00020000);
        unsigned woff[WPT];  // byte offset of each weight piece in chunk 0 (OOB past this N-block's rows)
#pragma unroll
        for (int i = 0; i < WPT; ++i) {
            const int item = ltid + i * 256;
            const int co = item / (9 * QPPX), r = item - co * (9 * QPPX), tap = r / QPPX, sp = r - tap * QPPX;
            woff[i] = ((item < WPIECES) & (n0 + co < p.N)) ? (unsigned)((n0 + co) * p.kpad + tap * p.ctap + sp * 16) : OOB;
            asm volatile("" : "+v"(woff[i]));
        }
        struct HSet {
            uint4 lo[HP], hi[HP];  // channels 0-7 / 8-15 of the thread's piece
            unsigned m, mh;        // bit i: piece i inside the image (m), and its upper 8 channels inside the source (mh)
            int cb;                // the chunk's first channel (concatenated index, the affine in sq)
            bool relu;
        };
        HSet st0, st1;
        auto set_of = [&](auto S) __attribute__((always_inline)) -> HSet& {
            if constexpr (decltype(S)::value == 0) return st0;
            else return st1;
        };
        uint4 wr[WPT];
        // WCONST: the second chunk's weights (two chunks per item) in registers of their own, loaded with the first's
        // (not at RT 4: its 640-pixel halo sets leave no room; there the second chunk's weights follow the barrier)
        constexpr bool W2 = WCONST && RT != 4;
        uint4 wr2[W2 ? WPT : 1];
        int w_cc = 0;
        auto load_w_into = [&](uint4 (&wdst)[WPT]) __attribute__((always_inline)) {  // weights of chunk w_cc, advance
            const int wc = c_lo + w_cc;
            const bool s1 = wc >= nc0;
            const int C = s1 ? p.c1 : p.c0;
            const int cl = (s1 ? wc - nc0 : wc) * QC;
            if (++w_cc == nchunks) w_cc = 0;
            unsigned v[WPT];
#pragma unroll
            for (int i = 0; i < WPT; ++i) v[i] = woff[i];
            if (cl + QC > C) {  // partial chunk: pieces past the source's channels read zeros
#pragma unroll
                for (int i = 0; i < WPT; ++i) {
                    const int sp = ((ltid + i * 256) % (9 * QPPX)) % QPPX;
                    if (cl + sp * 16 >= C) v[i] = OOB;
                }
            }
            const int cbg = (s1 ? p.c0 : 0) + cl;  // first channel of the chunk in k = tap*ctap + c
#pragma unroll
            for (int i = 0; i < WPT; ++i) {
                const auto x = __builtin_amdgcn_raw_buffer_load_b128(wrs, v[i], cbg, 0);
                wdst[i] = make_uint4(x[0], x[1], x[2], x[3]);
            }
        };
        auto load_w = [&]() __attribute__((always_inline)) { load_w_into(wr); };
        auto store_w_from = [&](int buf, const uint4 (&wsrc)[WPT]) __attribute__((always_inline)) {
            uint8_t* wl = smem + buf * BUF + HALO_B;
#pragma unroll
            for (int i = 0; i < WPT; ++i) {
                const int item = ltid + i * 256;
                const int co = item / (9 * QPPX), r = item - co * (9 * QPPX);
                if (item < WPIECES) *reinterpret_cast<uint4*>(wl + co * QW + r * 16) = wsrc[i];
            }
        };
        auto store_w = [&](int buf) __attribute__((always_inline)) { store_w_from(buf, wr); };
        auto load = [&](auto S) __attribute__((always_inline)) {  // halo of chunk (ld_item, ld_cc) -> set S, advance
            HSet& q = set_of(S);
            const int hc = c_lo + ld_cc;
            const bool s1 = hc >= nc0;
            const int C = s1 ? p.c1 : p.c0;
            const int cl = (s1 ? hc - nc0 : hc) * QC;
            q.cb = (s1 ? p.c0 : 0) + cl;
            q.relu = (s1 ? p.relu1 : p.relu0) != 0;
            const bool cok = cl + lpiece * 16 < C, hok = cl + lpiece * 16 + 8 < C;
            const __amdgpu_buffer_rsrc_t hrs =
                __builtin_amdgcn_make_buffer_rsrc((void*)(s1 ? ib1 : ib0), (short)0, hw_img * C * 2, 0x00020000);
            unsigned m = 0, mh = 0;
#pragma unroll
            for (int i = 0; i < HP; ++i) {
                const bool ok = (hpx[i] >= 0) & cok, okh = ok & hok;
                m |= (unsigned)ok << i;
                mh |= (unsigned)okh << i;
                unsigned off;
                asm("v_mad_u32_u24 %0, %1, %2, %3" : "=v"(off) : "v"(hpx[i]), "s"(C * 2), "v"(lpiece * 32));
                const unsigned o_lo = ok ? off : OOB, o_hi = okh ? off + 16u : OOB;
                const auto x = __builtin_amdgcn_raw_buffer_load_b128(hrs, o_lo, cl * 2, 0);
                const auto y = __builtin_amdgcn_raw_buffer_load_b128(hrs, o_hi, cl * 2, 0);
                q.lo[i] = make_uint4(x[0], x[1], x[2], x[3]);
                q.hi[i] = make_uint4(y[0], y[1], y[2], y[3]);
            }
            q.m = m;
            q.mh = mh;
            if (++ld_cc == nchunks) {
                ld_cc = 0;
                ++ld_item;
                geometry();
            }
        };
        auto store = [&](auto S, int buf) __attribute__((always_inline)) {  // halo set S (+ weights) -> LDS buffer buf
            HSet& q = set_of(S);
            uint8_t* hx = smem + buf * BUF;
            float s[16], h[16];
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const float4 a = *reinterpret_cast<const float4*>(sq + q.cb + lpiece * 16 + 4 * k);
                const float4 b = *reinterpret_cast<const float4*>(sq + QSBN + q.cb + lpiece * 16 + 4 * k);
                s[4 * k] = a.x, s[4 * k + 1] = a.y, s[4 * k + 2] = a.z, s[4 * k + 3] = a.w;
                h[4 * k] = b.x, h[4 * k + 1] = b.y, h[4 * k + 2] = b.z, h[4 * k + 3] = b.w;
            }
            const float lo_clamp = q.relu ? 0.f : -Q8_MAX;
#pragma unroll
            for (int i = 0; i < HP; ++i) {  // zero padding of the conv applies after the quantised activation
                uint4 v = quant16(q.lo[i], q.hi[i], s, h, lo_clamp);
                const bool ok = (q.m >> i) & 1u, okh = (q.mh >> i) & 1u;
                v.x = ok ? v.x : 0u;
                v.y = ok ? v.y : 0u;
                v.z = okh ? v.z : 0u;
                v.w = okh ? v.w : 0u;
                const int item = ltid + i * 256;
                *reinterpret_cast<uint4*>(hx + q_pixel(item) * QHX + q_piece(item) * 16) = v;
            }
            if constexpr (!WCONST) store_w(buf);
        };
        constexpr std::integral_constant<int, 0> S0{};
        constexpr std::integral_constant<int, 1> S1{};
        auto iter = [&](auto U) __attribute__((always_inline)) {
            store(U, decltype(U)::value & 1);
            if constexpr (!WCONST) load_w();
            load(U);
            __syncthreads();
        };
        if (total > 0) {
            // the loads an iteration would have issued before chunk 0 (same issue order, pinned by sched barriers):
            // the halo of chunk 0, the weights of chunk 0, the halo of chunk 1 (WCONST: the weights of both chunks
            // first, stored after the tables)
            geometry();
            if constexpr (WCONST) {
                load_w();  // chunk 0
                if constexpr (W2)
                    if (nchunks > 1) load_w_into(wr2);  // chunk 1
                __builtin_amdgcn_sched_barrier(0);
            }
            load(S0);
            __builtin_amdgcn_sched_barrier(0);
            if constexpr (!WCONST) load_w();
            __builtin_amdgcn_sched_barrier(0);
            load(S1);
        }
        fill_tables();
        __syncthreads();  // the tables (the MFMA waves meet it before their first chunk)
        if (total > 0) {
            if constexpr (WCONST) {
                store_w(0);
                if (nchunks > 1) {
                    if constexpr (W2) {
                        store_w_from(1, wr2);
                    } else {
                        load_w();  // chunk 1
                        store_w(1);
                    }
                } else {
                    store_w(1);  // one chunk per item: chunk 0 in both buffers
                }
            }
            // a multiple of LS iterations: past the last chunk the loads are out of range and the stores go to a
            // buffer the MFMA waves no longer read (they meet these iterations with extra barriers)
            for (int gi = 0; gi < total; gi += LS) {
                iter(S0);
                iter(S1);
            }
        }
        return;
    }

    // =============================================================== MFMA waves
    fill_tables();
    __syncthreads();  // the tables
    int abase[RT];  // LDS byte offset of this lane's B fragment (pixel lane & 31 of column tile i, tap (0,0))
#pragma unroll
    for (int i = 0; i < RT; ++i) {
        const int m = (wid + 4 * i) * 32 + (lane & 31);
        const int hm = m / p.tw, wm = m - hm * p.tw;
        abase[i] = (m < mvalid ? hm * p.hw + wm : 0) * QHX + (lane >> 5) * 32;
    }
    // epilogue (as conv_halo.hip's): EPR whole pixels per 16-B store instruction, ER instructions per 32-pixel tile
    constexpr int PPP = NT * 4;
    constexpr int EPR = 64 / PPP;
    constexpr int ER = 32 / EPR;
    auto swz = [](int j, int px) { return NT == 2 ? j ^ (px & 7) : j ^ ((px >> 1) & 3); };
    unsigned erel[(RT * ER + 1) / 2];  // tile-relative (row << 9 | col) of each store row, two per register
#pragma unroll
    for (int k = 0; k < (RT * ER + 1) / 2; ++k) erel[k] = 0xffffffffu;
#pragma unroll
    for (int i = 0; i < RT; ++i)
#pragma unroll
        for (int r = 0; r < ER; ++r) {
            const int m = (wid + 4 * i) * 32 + r * EPR + lane / PPP;
            const int hm = m / p.tw, wm = m - hm * p.tw;
            const unsigned v = m < mvalid ? (unsigned)((hm << 9) | wm) : 0xffffu;
            const int k = i * ER + r;
            erel[k / 2] = (erel[k / 2] & ~(0xffffu << (16 * (k & 1)))) | (v << (16 * (k & 1)));
        }
    __bf16* const scw = scr + wid * 32 * BN;
    f32x16 acc[RT][NT];
    int cc = 0, item = 0;
    for (int gi = 0; gi < total; ++gi) {
        __syncthreads();  // chunk gi is in buffer gi & 1
        if (cc == 0) {
#pragma unroll
            for (int i = 0; i < RT; ++i)
#pragma unroll
                for (int t = 0; t < NT; ++t)
#pragma unroll
                    for (int r = 0; r < 16; ++r) acc[i][t][r] = 0.f;
        }
        const uint8_t* hx = smem + (gi & 1) * BUF;
        const uint8_t* wl = hx + HALO_B;
        i32x8 af[2][RT], bfr[2][NT];
        auto rd = [&](int tap) __attribute__((always_inline)) {
            const int sl = tap & 1;
            const int toff = ((tap / 3) * p.hw + tap % 3) * QHX;
#pragma unroll
            for (int t = 0; t < NT; ++t) bfr[sl][t] = qfrag(wl + (t * 32 + (lane & 31)) * QW + tap * QC + (lane >> 5) * 32);
#pragma unroll
            for (int i = 0; i < RT; ++i) af[sl][i] = qfrag(hx + abase[i] + toff);
        };
        rd(0);
#pragma unroll
        for (int tap = 0; tap < 9; ++tap) {
            if (tap + 1 < 9) rd(tap + 1);
            __builtin_amdgcn_sched_barrier(0);
            const int sl = tap & 1;
            // C^T[co][pixel]: A = weight rows (output channels), B = halo pixels; both operands hold the same 32
            // channels in each lane half, so the K pairing is the identity
#pragma unroll
            for (int i = 0; i < RT; ++i)
#pragma unroll
                for (int t = 0; t < NT; ++t)
                    acc[i][t] = __builtin_amdgcn_mfma_scale_f32_32x32x64_f8f6f4(bfr[sl][t], af[sl][i], acc[i][t], 0, 0,
                                                                                0, 0, 0, 0);
            __builtin_amdgcn_sched_barrier(0);
        }
        if (++cc == nchunks) {
            // ------------------------------------------------------------ epilogue of `item`
            const int sp = slot + item * p.gper;
            const int b = sp / p.tiles, tl = sp - b * p.tiles;
            const int ty = tl / p.tiles_x;
            const int h0 = ty * p.th, w0 = (tl - ty * p.tiles_x) * p.tw;
            const int hw_img = p.H * p.W;
            const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
                (void*)(p.out + (size_t)b * hw_img * p.N), (short)0, hw_img * p.N * 2, 0x00020000);
            const int chq = 4 * (lane >> 5);
            // all tiles' scratch writes and read-backs issue back to back, then the stores: one LDS round trip per
            // item (LDS is in order per wave, so a tile's writes land after the previous tile's reads)
            uint4 rows[RT][ER];
#pragma unroll
            for (int i = 0; i < RT; ++i) {
#pragma unroll
                for (int t = 0; t < NT; ++t) {
                    uint2 pk[4];  // this lane's 4 channels of each 8-channel group g4, dequantised, packed bf16
#pragma unroll
                    for (int g4 = 0; g4 < 4; ++g4) {
                        const float4 d = *reinterpret_cast<const float4*>(deq + t * 32 + 8 * g4 + chq);
                        bf16x4 v;
                        v[0] = (__bf16)(acc[i][t][4 * g4] * d.x);
                        v[1] = (__bf16)(acc[i][t][4 * g4 + 1] * d.y);
                        v[2] = (__bf16)(acc[i][t][4 * g4 + 2] * d.z);
                        v[3] = (__bf16)(acc[i][t][4 * g4 + 3] * d.w);
                        pk[g4] = *reinterpret_cast<uint2*>(&v);
                    }
                    // lanes l and l+32 hold the two 4-channel halves of each 8-channel group of one pixel: one
                    // v_permlane32_swap per dword on groups (k, k+1) leaves group k whole in lane l, k+1 in l+32
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
                for (int r = 0; r < ER; ++r) {
                    const int px = r * EPR + lane / PPP, j = lane % PPP;
                    rows[i][r] = *reinterpret_cast<const uint4*>(scw + px * BN + swz(j, px) * 8);
                }
                asm volatile("" ::: "memory");  // the next tile's writes after these reads
            }
#pragma unroll
            for (int i = 0; i < RT; ++i) {
#pragma unroll
                for (int r = 0; r < ER; ++r) {
                    const unsigned rel = (erel[(i * ER + r) / 2] >> (16 * ((i * ER + r) & 1))) & 0xffffu;
                    const int h = h0 + (int)(rel >> 9), w = w0 + (int)(rel & 511u);
                    const int c = n0 + (lane % PPP) * 8;
                    const bool in = (rel != 0xffffu) & (h < p.H) & (w < p.W) & (c < p.N);
                    const unsigned off = in ? (unsigned)((h * p.W + w) * p.N + c) * 2u : 0x80000000u;
                    const uint4 v = rows[i][r];
                    __attribute__((ext_vector_type(4))) unsigned data = {v.x, v.y, v.z, v.w};
                    __builtin_amdgcn_raw_buffer_store_b128(data, rs, off, 0, 2);  // nontemporal
                }
            }
            cc = 0;
            ++item;
        }
    }
    for (int e = total; e < padded; ++e) __syncthreads();  // the loaders' iterations past the last chunk
}

// spatial tile: full-resolution N = 32 layers 16x32 (RT 4, 640-pixel halo); otherwise <= 256 pixels with a <= 384-pixel
// halo: the whole image if it fits, 8x32, 6x40, rows of the image
struct QTile {
    int th, tw, rt;
};
static QTile q8_tile(int H, int W, int N, int nch) {
    // RT 4 only with the weights resident (<= 2 chunks): its second loader set plus per-chunk weights would spill
    if (N == 32 && nch <= 2 && W % 32 == 0 && H >= 16) return {16, 32, 4};
    auto fits = [](int th, int tw) { return (th + 2) * (tw + 2) <= 384 && th * tw <= 256; };
    if (fits(H, W)) return {H, W, 2};
    if (W % 32 == 0) return {8, 32, 2};
    if (W % 40 == 0) return {6, 40, 2};
    if (W <= 256) {
        int th = 256 / W;
        while (th > 1 && !fits(th, W)) --th;
        if (fits(th, W)) return {th, W, 2};
    }
    return {8, 32, 2};
}

template <int NT, int RT>
static void launch_q8(bool wconst, dim3 grid, hipStream_t st, const QArgs& p) {
    if constexpr (RT == 4)
        hipLaunchKernelGGL((k_halo_conv_q8<NT, RT, true>), grid, dim3(512), 0, st, p);
    else if (wconst)
        hipLaunchKernelGGL((k_halo_conv_q8<NT, RT, true>), grid, dim3(512), 0, st, p);
    else
        hipLaunchKernelGGL((k_halo_conv_q8<NT, RT, false>), grid, dim3(512), 0, st, p);
}

// launch plan of one conv: tile, N-blocks, blocks per N-block. (A split-K form for the batch-1 deep layers, groups of
// blocks over slices of the input chunks plus a reduce launch, saved 4.8 us of kernel against the 5.0 us of its reduce
// launch at the live app's 960x720 (r04), so it was removed in r05: the e4m3 chunks hold 64 channels and these layers
// have only 4-8 chunks per item.)
struct QPlan {
    QTile t;
    int nt, nblk, gper, nsp, nch;
    bool wconst;
};
static QPlan q8_plan(int batch, int H, int W, int N, int c0, int c1) {
    QPlan q{};
    q.nch = cdiv(c0, QC) + cdiv(c1, QC);
    q.t = q8_tile(H, W, N, q.nch);
    const long long sp = (long long)batch * cdiv(W, q.t.tw) * cdiv(H, q.t.th);
    q.nsp = sp < (1LL << 30) ? (int)sp : (1 << 30);
    q.nt = N == 32 ? 1 : 2;
    q.nblk = N == 32 ? 1 : N / 64;
    q.gper = QPERSIST / q.nblk;
    if (q.gper < 1) q.gper = 1;
    if (q.gper > q.nsp) q.gper = q.nsp;
    q.wconst = q.nch <= 2;  // chunk c of every item lands in LDS buffer c: weights staged once per block
    return q;
}

}  // namespace

int sd_validate_src(const sd_src* s, const char* what);

extern "C" const char* sd_conv3x3_q8_kernel_name(int batch, int H, int W, int N, int c0, int c1) {
    static thread_local char buf[64];
    if (batch <= 0 || H <= 0 || W <= 0 || !(N == 32 || (N > 0 && N % 64 == 0)) || c0 <= 0 || c1 < 0) return "";
    const QPlan q = q8_plan(batch, H, W, N, c0, c1);
    snprintf(buf, sizeof(buf), "k_halo_conv_q8<%d, %d, %s>", q.nt, q.t.rt, q.wconst || q.t.rt == 4 ? "true" : "false");
    return buf;
}

extern "C" int sd_conv3x3_q8(const sd_src* a, int batch, int H, int W, const void* wq, const float* wscale,
                             const float* act_scale, int N, int kpad, void* out, sd_stream s) {
    if (int e = sd_validate_src(a, "sd_conv3x3_q8")) return e;
    SD_REQUIRE(a->taps == 9 && !a->pool, "sd_conv3x3_q8: needs an unpooled 3x3 source");
    SD_REQUIRE(a->H == H && a->W == W, "sd_conv3x3_q8: source grid %dx%d != %dx%d", a->H, a->W, H, W);
    for (int i = 0; i < 2; ++i)
        if (i == 0 || a->chans[1] > 0)
            SD_REQUIRE((a->xform[i] == SD_BNRELU || a->xform[i] == SD_AFFINE) && a->scale[i] && a->shift[i],
                       "sd_conv3x3_q8: source %d needs its quantisation affine (SD_BNRELU or SD_AFFINE)", i);
    SD_REQUIRE(batch > 0 && wq && wscale && act_scale && out, "sd_conv3x3_q8: bad args");
    SD_REQUIRE(N == 32 || N % 64 == 0, "sd_conv3x3_q8: N=%d must be 32 or a multiple of 64", N);
    const int ctot = a->chans[0] + a->chans[1];
    SD_REQUIRE(ctot <= QSBN && a->chans[0] % 8 == 0 && a->chans[1] % 8 == 0,
               "sd_conv3x3_q8: %d + %d input channels (multiples of 8, <= %d)", a->chans[0], a->chans[1], QSBN);
    // sources start on 16-channel pieces (a piece never mixes the two sources)
    SD_REQUIRE(a->chans[1] == 0 || a->chans[0] % 16 == 0, "sd_conv3x3_q8: first source of a concatenation %d % 16",
               a->chans[0]);
    const int ctap = (ctot + 15) / 16 * 16;
    SD_REQUIRE(kpad % 64 == 0 && kpad >= 9 * ctap, "sd_conv3x3_q8: kpad %d < 9*%d", kpad, ctap);
    const QPlan q = q8_plan(batch, H, W, N, a->chans[0], a->chans[1]);
    const QTile t = q.t;
    QArgs p;
    p.p0 = (const __bf16*)a->ptr[0];
    p.p1 = (const __bf16*)a->ptr[1];
    p.qs0 = a->scale[0];
    p.qh0 = a->shift[0];
    p.qs1 = a->chans[1] > 0 ? a->scale[1] : a->scale[0];
    p.qh1 = a->chans[1] > 0 ? a->shift[1] : a->shift[0];
    p.c0 = a->chans[0];
    p.c1 = a->chans[1];
    p.relu0 = a->xform[0] == SD_BNRELU;
    p.relu1 = a->xform[1] == SD_BNRELU;
    p.H = H;
    p.W = W;
    p.th = t.th;
    p.tw = t.tw;
    p.tiles_x = cdiv(W, t.tw);
    p.tiles = p.tiles_x * cdiv(H, t.th);
    SD_REQUIRE((long long)batch * p.tiles < (1LL << 30), "sd_conv3x3_q8: too many tiles");
    p.nsp = q.nsp;
    p.nblk = q.nblk;
    p.gper = q.gper;
    p.hw = t.tw + 2;
    p.nhalo = (t.th + 2) * (t.tw + 2);
    p.wq = (const uint8_t*)wq;
    p.wscale = wscale;
    p.act_scale = act_scale;
    p.N = N;
    p.kpad = kpad;
    p.ctap = ctap;
    p.out = (__bf16*)out;
    const int grid_n = q.gper * q.nblk;
    p.xcd = grid_n % 8 == 0;
    SD_REQUIRE(p.nhalo <= q_halo_cap(t.rt) && t.th * t.tw <= 128 * t.rt && t.th < 64 && t.tw < 512,
               "sd_conv3x3_q8: tile %dx%d", t.th, t.tw);
    // 32-bit buffer offsets: image-local pixel index (24-bit) times the channel stride, and the weights
    SD_REQUIRE((long long)H * W < (1LL << 24) && (long long)H * W * (p.c0 > p.c1 ? p.c0 : p.c1) * 2 < (1LL << 31) &&
                   (long long)N * kpad < (1LL << 31) && (long long)H * W * N * 2 < (1LL << 31),
               "sd_conv3x3_q8: image %dx%d or weights too large for 32-bit offsets", H, W);
    const dim3 grid(grid_n);
    if (q.nt == 1) {
        if (t.rt == 4) launch_q8<1, 4>(q.wconst, grid, to_stream(s), p);
        else launch_q8<1, 2>(q.wconst, grid, to_stream(s), p);
    } else {
        launch_q8<2, 2>(q.wconst, grid, to_stream(s), p);
    }
    return sd_check_launch("sd_conv3x3_q8");
}

