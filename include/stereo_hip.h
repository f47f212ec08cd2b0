/*
 * stereo_hip.h — C ABI of libstereo_hip.so, the MI355X (gfx950) kernel library
 * behind the stereo-disparity U-Net training path.
 *
 * The reference (sdfgeoff/stereo_depth_estimation) has no FFI: its boundary is the
 * PyTorch module / train-step API.  Every entry point below replaces
 * one ATen op family that the reference dispatches on that path; the reference
 * call site it replaces is cited per function.  Host-side mirror of the reference
 * interface: stereo_depth_estimation_amd/{model,engine,train}.py (Python, ctypes).
 *
 * Conventions
 *  - Plain C: raw device pointers, sizes, and a hipStream_t passed as an opaque
 *    pointer (sd_stream).  No torch types.  The caller (PyTorch) owns every buffer.
 *  - Every call is stream-ordered on the given stream, never synchronizes the device,
 *    never allocates or frees device memory (safe inside hipGraph capture).
 *  - Return 0 on success, SD_EINVAL for a rejected argument (checked on the host
 *    before any launch), SD_EHIP for a HIP launch error; sd_last_error() returns a
 *    thread-local message for the last failure.
 *  - Activations are NHWC, element type `dtype` (SD_F32 = fp32 parity mode, SD_BF16 =
 *    bf16 storage with fp32 accumulation).  Channel counts are multiples of 8.
 *  - Per-channel BN affines, statistics, parameters, gradients, optimizer state: fp32.
 */
#ifndef STEREO_HIP_H
#define STEREO_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void* sd_stream; /* hipStream_t */

enum { SD_OK = 0, SD_EINVAL = 1, SD_EHIP = 2 };
enum { SD_F32 = 0, SD_BF16 = 1 };
/* gather transforms: identity, max(scale*x + shift, 0), scale*x + shift (fp8 quantisation of a signed source) */
enum { SD_IDENT = 0, SD_BNRELU = 1, SD_AFFINE = 2 };
/* conv-GEMM epilogues */
enum { SD_EPI_STORE = 0, SD_EPI_STATS = 1, SD_EPI_SPLIT = 2, SD_EPI_PIXSHUF = 3, SD_EPI_SPLIT_STATS = 4 };
/* weight-gradient layouts */
enum { SD_W_CONV3 = 0, SD_W_CONVT = 1, SD_W_ROWSUM = 2 };
/* heads modes */
enum { SD_HEADS_INFER = 0, SD_HEADS_LOSS = 1, SD_HEADS_GRADS = 2 };

/*
 * Operand source of an implicit GEMM (the im2col gather).  Up to two NHWC sources
 * concatenated along channels (model.py:89-95 torch.cat([up, skip], 1)); each with an
 * optional fused BN+ReLU transform y -> max(scale[c]*y + shift[c], 0) (model.py:37-41),
 * an optional 2x2 max pool after the transform (model.py:59,83-86), and a tap pattern:
 *   taps = 1  : 1x1 (pixel (h,w) of the GEMM grid)
 *   taps = 9  : 3x3, pad 1 (pixel (h+kh-1, w+kw-1)), K index = tap*Ctot + c
 *   taps = 4  : 2x2 sub-pixel gather from a 2x-resolution source (2h+a, 2w+b)
 * H, W are the source's stored spatial dims.  Ctot = chans[0] + chans[1].
 */
typedef struct sd_src {
    const void* ptr[2];
    const float* scale[2];
    const float* shift[2];
    int chans[2];
    int xform[2];
    int H, W;
    int taps;
    int pool;
} sd_src;

int sd_version(void);
/* Diagnostics: device buffer for the per-wave cycle counters of timing builds (-DWG_EXP=1024; no effect
   otherwise). Not a reference interface. */
int sd_debug_buffer(void* dev_ptr);
/* Diagnostics: effective shader clock under MFMA load (bench.py "clock"). blocks x 256 threads of back-to-back bf16
   MFMAs; out[4 * block + {0,1,2,3}] = s_memtime start/end, s_memrealtime (100 MHz) start/end; sink: >= 256 floats
   (never written in practice). Not a reference interface. */
int sd_clock_probe(int blocks, int iters, unsigned long long* out, float* sink, sd_stream s);
const char* sd_last_error(void);
int sd_device_init(int device);

/* ---- packing (weights are fp32 PyTorch layout in, dtype MFMA-ready layout out) ---- */
/* reference input [B,6,H,W] f32 (train.py:320) -> NHWC dtype with cpad channels (zero pad). */
int sd_pack_input(int dtype, const float* x_nchw, int batch, int cin, int H, int W, int cpad, void* out, sd_stream s);
/* The same pack, also writing max |x| over the batch as float bits into amax[slot] (atomicMax into a zeroed word) and
 * zeroing amax[clear] for a later call (clear < 0: none): the fp8 live loop's input-range check (a frame brighter than
 * the calibration frame of the static e4m3 scales triggers a recalibration), read back asynchronously. */
int sd_pack_input_amax(int dtype, const float* x_nchw, int batch, int cin, int H, int W, int cpad, void* out,
                       unsigned* amax, int slot, int clear, sd_stream s);
/* Conv2d(k3,p1,no bias) weight [co][ci][3][3] (model.py:36,39) -> fwd [co][kpad] (k = tap*ci_pad + ci)
 * or, dgrad != 0, the flipped/transposed [ci][kpad] (k = tap*co + o, W[o][ci][8-tap]). */
int sd_pack_conv3_w(int dtype, const float* w, int co, int ci, int ci_pad, int dgrad, int kpad, void* out, sd_stream s);
/* ConvTranspose2d(k2,s2) weight [ci][co][2][2] (model.py:67-73) -> fwd [(t,o)][kpad=ci]
 * or, dgrad != 0, [ci][kpad] (k = t*co + o). */
int sd_pack_convT_w(int dtype, const float* w, int ci, int co, int dgrad, int kpad, void* out, sd_stream s);
/* Every pack of a step in ONE launch (the per-tensor forms above, up to 64 jobs): job j writes
 * out + out_off (elements of dtype) exactly as the per-tensor call of its kind would.
 * The weights it reads are the reference's Conv2d/ConvTranspose2d parameters (model.py:36,39,67-73). */
enum { SD_PACK_CONV3_FWD = 0, SD_PACK_CONV3_DGRAD = 1, SD_PACK_CONVT_FWD = 2, SD_PACK_CONVT_DGRAD = 3,
       /* bf16 hi/lo pairs of the fp32 weights (w = hi + lo to ~2^-17 relative; sd_conv3x3_wsplit and the doubled-K
        * ConvTranspose forward): conv3 fwd [co][kpad], k = tap*2*ci_pad + {ci: hi | ci_pad + ci: lo};
        * convT fwd [(t,o)][kpad], k = {i: hi | ci + i: lo} */
       SD_PACK_CONV3_FWD_SPLIT = 4, SD_PACK_CONVT_FWD_SPLIT = 5 };
typedef struct sd_pack_job {
    const float* w; /* fp32 PyTorch layout: conv3 [co][ci][3][3], convT [ci][co][2][2] */
    int kind;
    int co, ci, ci_pad; /* ci_pad: conv3 fwd only */
    int kpad;
    int64_t out_off;
} sd_pack_job;
int sd_pack_weights(int dtype, const sd_pack_job* jobs, int njobs, void* out, sd_stream s);

/* ---- implicit-GEMM convolution (replaces mkldnn_convolution / convolution_backward dgrad,
 *      model.py:36,39,67-77) ----
 * out[m, n] = sum_k A[m,k] * Wp[n,k], m = (b,h,w) over batch x H x W, n < N, k < K.
 * epi SD_EPI_STORE  : out0 NHWC [M][N]
 *     SD_EPI_STATS  : as STORE + stats[rows][N] float2 (sum, sumsq) per M-block (BN batch stats)
 *     SD_EPI_SPLIT  : n < n_split -> out0 [M][n_split], else out1 [M][N-n_split]  (cat backward)
 *     SD_EPI_PIXSHUF: n = t*C + o -> out0 [b][2h+t/2][2w+t%2][o] + bias[o]  (ConvTranspose2d)
 *     SD_EPI_SPLIT_STATS: SPLIT + stats rows over all N columns (bf16, 3x3 halo shapes only): the dgrad of a
 *                    decoder conv0 also yields the column sums of d(up), the ConvTranspose2d bias gradient
 *                    (sd_stat_rows_sum) */
int sd_conv_gemm(int dtype, const sd_src* a, int batch, int H, int W, const void* wpack, int N, int kpad, int epi,
                 void* out0, void* out1, int n_split, const float* bias, float* stats, sd_stream s);
/* number of float2 stat rows sd_conv_gemm(SD_EPI_STATS) writes for this shape */
int sd_conv_gemm_stat_rows(int dtype, int batch, int H, int W, int N);
/* name of the kernel instance sd_conv_gemm / sd_wgrad_gemm launches for a shape (as rocprofv3 shows it) */
const char* sd_conv_gemm_kernel_name(int dtype, const sd_src* a, int batch, int H, int W, int N, int epi);
const char* sd_wgrad_kernel_name(int dtype, const sd_src* a, const sd_src* b, int M, int N);

/* sd_conv_gemm(SD_EPI_STORE) of a dgrad whose output `out` is the upstream gradient da of a BatchNorm layer with raw
 * output y (model.py:37,40): the same launch also writes that layer's BatchNorm-backward partial sums (what
 * sd_bn_bwd_reduce computes from da and y in a pass of its own), sd_conv_gemm_bnsum_rows() rows of float2[N],
 * for sd_bn_bwd_finalize. bf16 3x3 halo shapes and the ConvTranspose2d dgrad (4-tap sub-pixel source, model.py:67-73)
 * where the LDS-resident-weight kernel takes it: sd_conv_gemm_bnsum_ok. */
int sd_conv_gemm_bnsum(int dtype, const sd_src* a, int batch, int H, int W, const void* wpack, int N, int kpad,
                       void* out, const void* y, const float* scale, const float* shift, const float* mean,
                       const float* invstd, float* partials, sd_stream s);
int sd_conv_gemm_bnsum_ok(int dtype, const sd_src* a, int N);

/* The bf16 3x3 convolution (model.py:36,39) of the halo kernel with two precision options for the eval forwards:
 *  flags & SD_CONV_WSPLIT: the fp32 weights as bf16 hi/lo pairs (sd_pack_weights kind SD_PACK_CONV3_FWD_SPLIT): each
 *      chunk of input channels meets the hi then the lo halves, so the weights carry fp32 precision into the MFMA
 *      while the activations stay bf16 (twice the MFMA work). The weights' bf16 rounding is a systematic change of
 *      the function that shifted the EPE of trained checkpoints by 2e-3..1e-2 px (tools/precision_study.py).
 *  out_scale / out_shift (both or neither; STORE only): the stored value is bf16(acc*out_scale[n] + out_shift[n]),
 *      the layer's eval-mode BatchNorm applied before the rounding (model.py:37,40), so consumers apply only the ReLU
 *      (pass scale 1, shift 0) and bf16 keeps its relative precision on the normalised activation.
 * epi: SD_EPI_STORE or SD_EPI_STATS (stats as sd_conv_gemm). bf16 3x3 halo shapes only (N = 32 or N % 64 == 0,
 * unpooled source): sd_conv3x3_ex_ok. */
enum { SD_CONV_WSPLIT = 1 };
int sd_conv3x3_ex(const sd_src* a, int batch, int H, int W, const void* wpack, int N, int kpad, int epi, int flags,
                  const float* out_scale, const float* out_shift, void* out, float* stats, sd_stream s);
int sd_conv3x3_ex_ok(const sd_src* a, int N);
const char* sd_conv3x3_ex_kernel_name(const sd_src* a, int H, int W, int N, int epi, int flags, int out_affine);
/* The same with a split-K workspace: a STORE launch whose items would leave most CUs idle (the batch-1 forwards of the
 * deep layers) runs in groups of blocks over slices of the input-channel chunks (and of the hi/lo passes), and a
 * second launch adds their fp32 partial sums, applies the output affine and stores bf16. ws (16-B aligned) must hold
 * sd_conv3x3_ex_ws_bytes(...) bytes (0: no split for the shape); a NULL or smaller ws runs unsplit. Results equal
 * sd_conv3x3_ex's up to the fp32 summation order. */
long long sd_conv3x3_ex_ws_bytes(const sd_src* a, int batch, int H, int W, int N, int epi, int flags);
int sd_conv3x3_ex_ws(const sd_src* a, int batch, int H, int W, const void* wpack, int N, int kpad, int epi, int flags,
                     const float* out_scale, const float* out_shift, void* out, float* stats, void* ws,
                     long long ws_bytes, sd_stream s);
int sd_conv_gemm_bnsum_rows(const sd_src* a, int batch, int H, int W, int N);
const char* sd_conv_gemm_bnsum_kernel_name(const sd_src* a, int H, int W, int N);

/* ---- weight gradient (replaces convolution_backward wgrad, model.py:36,39,67-73) ----
 * slab[z][m][n] = sum over the z-th pixel range of A(p, m) * B(p, n), p over batch x H x W. */
int sd_wgrad_splits(int dtype, int batch, int H, int W, int M, int N);
int sd_wgrad_gemm(int dtype, const sd_src* a, const sd_src* b, int batch, int H, int W, int M, int N, float* slab,
                  int splits, sd_stream s);
/* The BatchNorm2d backward apply (sd_bn_bwd_apply, model.py:37,40) fused into the bf16 3x3 weight gradient
 * (convolution_backward wgrad, model.py:36,39): the kernel stages A = dy formed from the raw pair
 * (da, y) as sd_bn_bwd_apply defines it, dy = coef0*(dz - coef1 - xhat*coef2), dz = da*[scale*y+shift > 0],
 * xhat = (y-mean)*invstd, and also writes that dy to a->ptr[0] ([pixels][M], for the dgrad). Same b/slab/splits
 * contract as sd_wgrad_gemm (a: the plain 1x1 [pixels][M] source, used as the dy destination). The kernel
 * takes coef0 = scale (both are gamma*invstd as sd_bn_fwd_finalize / sd_bn_eval_coeffs and
 * sd_bn_bwd_finalize write them) and reads coef1, coef2 from coef. a->ptr[0] may be NULL: dy is not written
 * (a layer without a dgrad); the shapes with x channels not a multiple of 32 (M = 32 only) require that.
 * sd_wgrad_bnbwd_ok: 0 when the shape has no fused kernel (then apply + sd_wgrad_gemm), else the number of
 * x-channel blocks that each form the same dy tile (1: dy is formed once; more: the transform is repeated per
 * block, which costs more than the separate apply pass at the model's deep layers). */
int sd_wgrad_bnbwd_ok(int dtype, const sd_src* a, const sd_src* b, int M, int N);
int sd_wgrad_gemm_bnbwd(int dtype, const sd_src* a, const sd_src* b, int batch, int H, int W, int M, int N,
                        const void* da, const void* y, const float* scale, const float* shift, const float* mean,
                        const float* invstd, const float* coef, float* slab, int splits, sd_stream s);
const char* sd_wgrad_bnbwd_kernel_name(const sd_src* a, const sd_src* b, int M, int N);
/* sum the slabs and write the PyTorch-layout fp32 gradient:
 *   SD_W_CONV3: M = co, N = 9*ci_pad -> dw[co][ci_real][3][3]
 *   SD_W_CONVT: M = ci, N = 4*co     -> dw[ci][co][2][2] */
int sd_wgrad_reduce(const float* slab, int splits, int M, int N, int layout, int ci_real, float* dw, sd_stream s);
/* up to 48 of those reduces in ONE launch, each bit-identical to its sd_wgrad_reduce call (the slabs must be
 * distinct buffers: the engine defers a step's reduces into one launch per gradient-ready group).
 * layout SD_W_ROWSUM: dw[c] = sum over r < splits of ((const float2*)slab)[r * N + c].x for c < ci_real (M = 1),
 * bit-identical to sd_stat_rows_sum(slab, splits, N, ci_real, dw): the ConvTranspose2d bias gradients joined to the
 * batch instead of a launch each */
typedef struct sd_wred_job {
    const float* slab;
    int splits, M, N, layout, ci_real;
    float* dw;
} sd_wred_job;
int sd_wgrad_reduce_batch(const sd_wred_job* jobs, int njobs, sd_stream s);

/* ---- host data path: the reference's sample cache (dataset.py:86-105 load_cached_sample; cache.py:50-112) ----
 * Reads n np.savez cache files (stored zip of left.npy / right.npy uint8 [H][W][3], disparity.npy f16 [H][W]) with
 * `threads` host threads into left/right [n][H][W][3] and disparity [n][H][W] (f16 bits). Returns 0, or 1 + the index
 * of the first file that is missing, compressed, or of another dtype/shape (message in err), or -1 for bad args. */
int sd_read_cache_batch(const char* const* paths, int n, int H, int W, uint8_t* left, uint8_t* right,
                        uint16_t* disparity, int threads, char* err, int errlen);

/* PNG frames of the un-cached source (reference dataset.py:23-30,184-212: PIL open + convert("RGB")): 8-bit RGB or
 * RGBA, not interlaced. sd_png_size reads the IHDR; sd_read_png_batch decodes n frames of H x W with `threads` host
 * threads into out [n][H][W][3]. Returns as sd_read_cache_batch (other PNG kinds: an error, for a PIL fallback). */
int sd_png_size(const char* path, int* height, int* width);
int sd_read_png_batch(const char* const* paths, int n, int H, int W, uint8_t* out, int threads, char* err, int errlen);

/* ---- BatchNorm2d train/eval (model.py:37,40; native_batch_norm / _backward) ---- */
int sd_bn_fwd_finalize(const float* stats, int rows, int C, double count, const float* gamma, const float* beta,
                       float* running_mean, float* running_var, int64_t* num_batches_tracked, float momentum,
                       float eps, float* mean, float* invstd, float* scale, float* shift, sd_stream s);
int sd_bn_eval_coeffs(const float* running_mean, const float* running_var, const float* gamma, const float* beta,
                      int C, float eps, float* mean, float* invstd, float* scale, float* shift, sd_stream s);
/* rows of float2 partials sd_bn_bwd_reduce / sd_chan_sum write */
int sd_chan_reduce_rows(int64_t pixels, int C);
/* partial (sum dz, sum dz*xhat), dz = da * [scale*y+shift > 0], xhat = (y-mean)*invstd */
int sd_bn_bwd_reduce(int dtype, const void* da, const void* y, const float* scale, const float* shift,
                     const float* mean, const float* invstd, int64_t pixels, int C, float* partials, sd_stream s);
/* -> dgamma, dbeta (fp32, into the flat grad buffer) and coef[C][3] = {gamma*invstd, sum dz/N, sum dz*xhat/N};
 * batch_stats = 0 (forward used running stats, eval mode): coef = {gamma*invstd, 0, 0}. */
int sd_bn_bwd_finalize(const float* partials, int rows, int C, double count, const float* gamma,
                       const float* invstd, int batch_stats, float* dgamma, float* dbeta, float* coef, sd_stream s);
/* SyncBatchNorm (SURVEY §8e "--sync-bn"; torch.nn.SyncBatchNorm semantics, replacing the per-rank reductions of
 * model.py:37,40 under DDP). Each rank reduces its float2 partial rows (the producer's STATS rows, or the
 * BatchNorm-backward partials) to fp64 sums[2C + 1]: per channel (sum, sumsq), then this rank's pixel count; the
 * host all-reduces the whole vector (SUM) across ranks, so the count that arrives is the global one whatever each
 * rank's batch size; the finalizes below read it from sums[2C]. The backward writes dgamma/dbeta from local_sums
 * (the gradient all-reduce adds the ranks' shares) and coef from global_sums. */
int sd_bn_rows_sum64(const float* rows, int nrows, int C, double pixels, double* sums, sd_stream s);
int sd_bn_fwd_finalize64(const double* sums, int C, const float* gamma, const float* beta,
                         float* running_mean, float* running_var, int64_t* num_batches_tracked, float momentum,
                         float eps, float* mean, float* invstd, float* scale, float* shift, sd_stream s);
int sd_bn_bwd_finalize64(const double* local_sums, const double* global_sums, int C, const float* gamma,
                         const float* invstd, int batch_stats, float* dgamma, float* dbeta, float* coef, sd_stream s);
/* dy = coef0 * (dz - coef1 - xhat*coef2) */
int sd_bn_bwd_apply(int dtype, const void* da, const void* y, const float* scale, const float* shift,
                    const float* mean, const float* invstd, const float* coef, int64_t pixels, int C, void* dy,
                    sd_stream s);
/* MaxPool2d(2) backward (first max in row-major window order, as ATen CPU) + skip-gradient add:
 * da[b,h,w,c] = dskip[b,h,w,c] + (argmax ? dpool[b,h/2,w/2,c] : 0); dskip may be NULL.
 * partials != NULL: also the BatchNorm-backward partial sums of this layer (what sd_bn_bwd_reduce
 * computes from da and y, here from registers), sd_pool_bwd_rows() rows of float2[C], for
 * sd_bn_bwd_finalize; needs mean/invstd and C/8 dividing 256. */
int sd_pool_bwd_add(int dtype, const void* y, const float* scale, const float* shift, const void* dskip,
                    const void* dpool, int batch, int H, int W, int C, void* da, const float* mean,
                    const float* invstd, float* partials, sd_stream s);
int sd_pool_bwd_rows(int batch, int H, int W, int C);
/* bf16: materialise MaxPool2d(2)(relu(scale*y + shift)) [b][H/2][W/2][C] (model.py:59,83-86) so the
 * next conv's gather is a plain read (the fp32 parity path pools inside the gather instead) */
int sd_bnrelu_pool(int dtype, const void* y, const float* scale, const float* shift, int batch, int H, int W, int C,
                   void* out, sd_stream s);
/* column sums over pixels (ConvTranspose2d bias grad): partials then out[C] = sum (fp32) */
int sd_chan_sum(int dtype, const void* x, int64_t pixels, int C, float* partials, float* out, sd_stream s);
/* out[c] = sum over rows of stats[r][c].sum (float2 rows of ld columns, c < C; fp64 accumulation): the column
 * sums of an SD_EPI_SPLIT_STATS (or STATS) launch, e.g. the ConvTranspose2d bias gradient (model.py:67-73) */
int sd_stat_rows_sum(const float* stats, int rows, int ld, int C, float* out, sd_stream s);

/* ---- heads + loss (model.py:76-77,98,103; train.py:329-356) ----
 * act = max(scale*y + shift, 0) [pixels][C] (dec1 output), head weights wd/wl [C], biases bd/bl [1].
 * INFER : disp = softplus(act.wd + bd), logvar = clamp(act.wl + bl, -6, 3)
 * LOSS  : + masked heteroscedastic NLL with n = *count valid pixels (mask & isfinite(target)):
 *         da[pixels][C] (dtype) = d loss / d act; partials for head grads and metric sums
 * GRADS : da from given dense gdisp/glogvar (autograd path) */
/* valid pixels of a batch (train.py:329-330: valid_mask & isfinite(target)) into count[0..ncount-1] (1-4 counters, all
 * set to the same value: this rank's count and the loss normaliser that DDP all-reduces, without a copy launch).
 * clear == NULL: count is zeroed first (a memset); else count must already be zero and the kernel zeroes
 * clear[0..ncount-1] for the caller's next call (double-buffered counters: one launch per batch). */
int sd_count_valid(const float* target, const uint8_t* mask, int64_t pixels, int* count, int ncount, int* clear,
                   sd_stream s);
/* the train step's prologue in ONE launch (train.py:320-330 before the forward): sd_pack_weights(dtype, jobs, njobs,
 * wpack), sd_pack_input(dtype, x, batch, cin, H, W, cpad, xout) and sd_count_valid(target, mask, pixels, count, ncount,
 * clear) with a non-NULL clear, a 4-B aligned mask and 16-B aligned targets; the same results as the three calls */
int sd_step_prologue(int dtype, const sd_pack_job* jobs, int njobs, void* wpack, const float* x, int batch, int cin,
                     int H, int W, int cpad, void* xout, const float* target, const uint8_t* mask, int64_t pixels,
                     int* count, int ncount, int* clear, sd_stream s);
int sd_heads_rows(int64_t pixels);
int sd_heads(int dtype, int mode, const void* y, const float* scale, const float* shift, int64_t pixels, int C,
             const float* wd, const float* bd, const float* wl, const float* bl, float* disp, float* logvar,
             const float* target, const uint8_t* mask, const int* count, const float* gdisp, const float* glogvar,
             void* da, float* partials, sd_stream s);
/* sd_heads (LOSS / GRADS) that also writes the BatchNorm-backward partial sums of the dec1 layer it
 * reads (replaces sd_bn_bwd_reduce over da and y, model.py:40-41 backward): bnpart[sd_heads_rows][C]
 * float2 = (sum dz, sum dz*xhat), dz = da (as stored) where y*scale+shift > 0, xhat = (y-mean)*invstd */
int sd_heads_bnsum(int dtype, int mode, const void* y, const float* scale, const float* shift, int64_t pixels, int C,
                   const float* wd, const float* bd, const float* wl, const float* bl, float* disp, float* logvar,
                   const float* target, const uint8_t* mask, const int* count, const float* gdisp,
                   const float* glogvar, void* da, float* partials, const float* mean, const float* invstd,
                   float* bnpart, sd_stream s);
/* reduce heads partials: head grads into dwd[C], dbd[1], dwl[C], dbl[1] (skipped if NULL) and
 * metric sums (sum nll, sum |d|, sum d^2, sum exp(lv/2), n) added into metrics[5] (fp64). */
int sd_heads_finalize(const float* partials, int rows, int C, float* dwd, float* dbd, float* dwl, float* dbl,
                      double* metrics, const int* count, sd_stream s);

/* ---- fp8 (OCP e4m3) inference forward of the 3x3 convolutions (eval-mode model.py:36-41 as the live app
 *      runs it, depth_live_dl.py:516-529) ----
 * Activations stay bf16 NHWC. Each source of `a` carries its folded quantisation affine in scale/shift:
 * q = e4m3(clamp(xform(x*scale + shift), +-448)), xform = ReLU for SD_BNRELU, none for SD_AFFINE
 * (sd_fp8_qparams computes them). Weights: sd_pack_conv3_w_fp8, e4m3 [co][kpad] (k = tap*ctap + c,
 * ctap = ctot rounded up to 16) with one fp32 scale per output channel.
 * out[m][n] (bf16) = act_scale[0] * wscale[n] * sum_k q[m][k] * wq[n][k]   (v_mfma_scale_f32_32x32x64_f8f6f4)
 * minmax: sd_conv3x3_fp8_rows() rows of float2[N] = (min, max) of the stored outputs, per block. */
int sd_pack_conv3_w_fp8(const float* w, int co, int ci, int ci_pad, int kpad, void* out, float* scale, sd_stream s);
int sd_conv3x3_fp8(const sd_src* a, int batch, int H, int W, const void* wq, const float* wscale,
                   const float* act_scale, int N, int kpad, void* out, float* minmax, sd_stream s);
int sd_conv3x3_fp8_rows(int batch, int H, int W, int N);
const char* sd_conv3x3_fp8_kernel_name(int N);
/* per-channel (min, max) rows of a bf16 NHWC tensor [pixels][C] (sources no fp8 conv produced: the packed
 * input, ConvTranspose outputs): sd_chan_minmax_rows() rows of float2[C] */
int sd_chan_minmax_rows(int64_t pixels, int C);
int sd_chan_minmax(const void* x, int64_t pixels, int C, float* rows, sd_stream s);
/* Dynamic activation scale of one conv input (1 or 2 concatenated sources): amax over the sources of
 * xform(scale*x + shift) from their (min, max) rows (identity affine when scale == NULL),
 * act_scale[0] = s_a = amax / 448, and per source the folded affine for the fp8 gather:
 * qscale = scale / s_a, qshift = shift / s_a (or 1/s_a, 0 when scale == NULL or ident: the consumer
 * reads the already-transformed tensor, e.g. the materialised MaxPool of relu(bn(y))). */
typedef struct sd_qsrc {
    const float* rows; /* [nrows][C] float2 (min, max) */
    int nrows;
    int C;
    const float* scale; /* per-channel affine before the quantisation, NULL = identity */
    const float* shift;
    int relu;
    int ident;
    float* qscale; /* out [C] */
    float* qshift; /* out [C] */
} sd_qsrc;
int sd_fp8_qparams(const sd_qsrc* src, int nsrc, float* act_scale, sd_stream s);
/* The same conv with STATIC scales (the engine's forwards after its calibration forward, while the model state is
 * unchanged): act_scale and the sources' folded affines are the ones sd_fp8_qparams left; no min/max rows are
 * written. Same operands and result contract as sd_conv3x3_fp8 otherwise (N = 32 or a multiple of 64, <= 512 input
 * channels; a concatenation's first source a multiple of 16 channels). */
int sd_conv3x3_q8(const sd_src* a, int batch, int H, int W, const void* wq, const float* wscale,
                  const float* act_scale, int N, int kpad, void* out, sd_stream s);
const char* sd_conv3x3_q8_kernel_name(int batch, int H, int W, int N, int c0, int c1);

/* ---- fused backward of a full-resolution 32 -> 32 conv + BatchNorm + ReLU layer (model.py:36-41: enc1.1, dec1.1)
 * One pass over the layer: dy = BatchNorm-backward(da, y) (scale, shift, mean, invstd: this layer's forward
 * coefficients, coef: its [C][3] backward coefficients from sd_bn_bwd_finalize), never stored; the weight gradient as
 * split-K slabs slab[splits][32][288] (k = tap*32 + ci, reduced by sd_wgrad_reduce with SD_W_CONV3); dx = the dgrad
 * (wd: sd_pack_conv3_w dgrad layout, kpad >= 288) into dx, which is da of the previous BatchNorm layer, whose raw
 * output yp and coefficients (pscale, pshift: x = relu(pscale*yp + pshift); pmean, pinvstd) it takes; and that
 * layer's BatchNorm-backward sums (sum dz, sum dz*xhat) as partials[splits][32] float2, for sd_bn_bwd_finalize.
 * Replaces sd_wgrad_gemm_bnbwd + sd_conv_gemm_bnsum for these layers. splits = sd_conv3x3_bwd_fused_splits(...). */
int sd_conv3x3_bwd_fused_ok(int C, int Cx, int H, int W);
int sd_conv3x3_bwd_fused_splits(int batch, int H, int W);
int sd_conv3x3_bwd_fused(const void* da, const void* y, const float* scale, const float* shift, const float* mean,
                         const float* invstd, const float* coef, const void* yp, const float* pscale,
                         const float* pshift, const float* pmean, const float* pinvstd, const void* wd, int kpad,
                         int batch, int H, int W, void* dx, float* slab, float* partials, sd_stream s);
/* The same for the full-resolution decoder conv0 (model.py:89-95, dec1.0: cat(u, relu(sscale*xs + sshift)), 32 + 32
 * -> 32 channels): dy from (da, y) as above; the weight gradient as slab[splits][32][576] (k = tap*64 + ci, ci < 32 the
 * u half; sd_wgrad_reduce with SD_W_CONV3, ci_real 64); the 64-channel dgrad (wd: [64][kpad], kpad >= 288) stored
 * split, du = its first 32 channels (d(u), the ConvTranspose2d output gradient), dskip the other 32; and the column
 * sums of du (the ConvTranspose2d bias gradient) as partials[splits][32] float2 (sum, 0) for sd_stat_rows_sum(ld 32).
 * Replaces sd_wgrad_gemm_bnbwd (two 32-channel x blocks) + the SD_EPI_SPLIT_STATS dgrad. */
int sd_conv3x3_bwd_fused_dec_ok(int C, int Cu, int Cs, int H, int W);
int sd_conv3x3_bwd_fused_dec(const void* da, const void* y, const float* scale, const float* shift, const float* mean,
                             const float* invstd, const float* coef, const void* xu, const void* xs,
                             const float* sscale, const float* sshift, const void* wd, int kpad, int batch, int H,
                             int W, void* du, void* dskip, float* slab, float* partials, sd_stream s);

/* ---- AdamW (train.py:343,578; torch 2.10 single-tensor AdamW, decoupled weight decay) ----
 * One flat fp32 parameter/gradient/state buffer (all tensors share lr/betas/eps/wd).
 * The step is skipped (and *step not advanced) when *count == 0 (train.py:331-332). One launch: scratch[0] is the
 * kernel's block counter (zero before the first call; every call leaves it zero). */
int sd_adamw(float* p, const float* g, float* m, float* v, int64_t n, double lr, double weight_decay, double beta1,
             double beta2, double eps, int* step, const int* count, float* scratch /* 4 floats */, sd_stream s);

/* ---- data path (dataset.py:184-212): bilinear resize, align_corners=False, no antialias ----
 * in [planes][Hi][Wi] f32 -> out [planes][Ho][Wo] f32, times `mul` (disparity width scaling). */
int sd_resize_bilinear(const float* in, int planes, int Hi, int Wi, float* out, int Ho, int Wo, float mul, sd_stream s);

/* ---- on-device sample preparation (replaces FoundationStereoDataset.__getitem__'s tensor work,
 * dataset.py:184-212,305-311, which the reference runs in DataLoader workers) ----
 * Raw samples, uint8 HWC at the source resolution as PIL decodes them (RGB order):
 *   left, right [B][Hs][Ws][3]; disparity RGB24 [B][Hs][Ws][3] (depth_uint8_decoding, dataset.py:23-30)
 * -> input  [B][6][Ho][Wo] f32: left RGB/255 then right, bilinear (align_corners=False), dataset.py:184-193
 *    target [B][1][Ho][Wo] f32: (R*255*255 + G*255 + B)/1000, bilinear, times Wo/Ws, dataset.py:195-212
 *    valid  [B][1][Ho][Wo] u8 : target > 0, dataset.py:306
 * Optional asymmetric colour augmentation (dataset.py:248-270) is applied afterwards by sd_augment_rgb. */
int sd_stereo_preprocess(const uint8_t* left, const uint8_t* right, const uint8_t* disp_rgb, int batch, int Hs,
                         int Ws, int Ho, int Wo, float* input, float* target, uint8_t* valid, sd_stream s);
/* Cached samples (load_cached_sample, dataset.py:86-105): left/right uint8 [B][Ho][Wo][3] and disparity
 * f16 [B][Ho][Wo] already at the training resolution -> the same three outputs. */
int sd_stereo_from_cache(const uint8_t* left, const uint8_t* right, const uint16_t* disp_f16, int batch, int Ho,
                         int Wo, float* input, float* target, uint8_t* valid, sd_stream s);
/* Asymmetric colour augmentation (FoundationStereoDataset._augment_rgb, dataset.py:248-270, torchvision 0.25
 * functional ops), in place on input [B][6][H][W] f32 = 2B RGB images (left, right of each pair).
 * params [2B][7] f32 per image: brightness, contrast, saturation factors, hue shift, gamma, blur sigma
 * (0 = no blur), noise std. blur_ksize odd in [3, 31]. Noise: counter-based N(0,1) keyed by `seed`.
 * work: 8-B aligned scratch of B*6*H*W + 128*B floats (the images, then 64 fp64 contrast partial sums per pair). */
int sd_augment_rgb(float* input, int batch, int H, int W, const float* params, int blur_ksize, uint64_t seed,
                   float* work, sd_stream s);

#ifdef __cplusplus
}
#endif
#endif /* STEREO_HIP_H */
