"""Per-kernel parity through the C ABI vs plain PyTorch fp32 CPU references (needs an MI355X).

fp32 mode (exact-f32 MFMA): max |Δ| <= 1e-4 * (1 + max|ref|).  bf16 mode: inputs are first
rounded to bf16 on both sides; tolerance 2e-2 relative to max|ref| (bf16 output rounding + K-sum order).
"""

import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")


def L():
    from stereo_depth_estimation_amd import _lib

    return _lib


def _tol(ref, prec):
    m = float(ref.abs().max())
    return (1e-4 if prec == "fp32" else 5e-3) * (1 + m)


def _adt(prec):
    return torch.float32 if prec == "fp32" else torch.bfloat16


def _sd(prec):
    return L().SD_F32 if prec == "fp32" else L().SD_BF16


def _nhwc(x, prec):
    return x.permute(0, 2, 3, 1).contiguous().to(DEV, _adt(prec))


def _from_nhwc(y, B, H, W, C):
    return y.float().cpu().reshape(B, H, W, C).permute(0, 3, 1, 2)


def _pack3(w, ci_pad, dgrad, prec):
    lib = L()
    co, ci = w.shape[:2]
    kpad = ((9 * (co if dgrad else ci_pad) + 63) // 64) * 64
    out = torch.empty((ci if dgrad else co) * kpad, dtype=_adt(prec), device=DEV)
    wd = w.contiguous().to(DEV)
    lib.call("sd_pack_conv3_w", _sd(prec), wd.data_ptr(), co, ci, ci_pad, int(dgrad), kpad, out.data_ptr(), lib.stream_handle())
    return out, kpad


@pytest.mark.parametrize("prec", ["fp32", "bf16"])
@pytest.mark.parametrize("B,H,W,ci,co,pool,bn", [(2, 12, 20, 16, 32, False, False), (2, 8, 16, 32, 64, True, True),
                                                 (1, 16, 16, 64, 128, False, True), (3, 6, 10, 24, 8, False, False),
                                                 # bf16 halo-kernel tile shapes: whole 15x20 image (10 row tiles),
                                                 # 6x40 tiles, 5x50 rows with a ragged last tile, ragged 8x32
                                                 (2, 15, 20, 40, 128, False, True), (1, 30, 40, 64, 192, False, False),
                                                 (1, 26, 50, 16, 64, True, True), (1, 9, 300, 8, 64, False, False),
                                                 # N=32 16x32 tiles; > 256 tiles so blocks reuse the weights
                                                 (1, 32, 64, 32, 32, False, True), (2, 128, 640, 8, 32, False, True),
                                                 # 8-channel input (enc1.0): CK=8 chunks, 8x32 and ragged tiles
                                                 (2, 32, 64, 8, 32, False, True), (2, 30, 50, 8, 32, False, True)])
def test_conv3x3_fwd_with_bn_pool_gather_and_stats(prec, B, H, W, ci, co, pool, bn):
    lib = L()
    torch.manual_seed(0)
    Hs, Ws = (2 * H, 2 * W) if pool else (H, W)
    y = torch.randn(B, ci, Hs, Ws)
    sc, sh = torch.rand(ci) + 0.5, torch.randn(ci) * 0.2
    sc[::3] *= -1
    w = torch.randn(co, ci, 3, 3) / (3 * ci ** 0.5)
    yq = y.to(_adt(prec)).float()
    wq = w.to(_adt(prec)).float()
    x = torch.relu(yq * sc[None, :, None, None] + sh[None, :, None, None]) if bn else yq
    if pool:
        x = F.max_pool2d(x, 2)
    if prec == "bf16":
        x = x.to(torch.bfloat16).float()
    ref = F.conv2d(x, wq, padding=1)
    wp, kpad = _pack3(w, ci, False, prec)
    scd, shd = sc.to(DEV), sh.to(DEV)
    yd = _nhwc(y, prec)
    src = lib.make_src(yd, ci, Hs, Ws, taps=9, pool=pool, bn0=(scd, shd) if bn else None)
    out = torch.empty(B * H * W, co, dtype=_adt(prec), device=DEV)
    if prec == "bf16" and pool:
        # bf16 pooled gather = generic kernel (STORE only); the fast path reads a materialised pool
        lib.call("sd_conv_gemm", _sd(prec), src, B, H, W, wp.data_ptr(), co, kpad, lib.SD_EPI_STORE, out.data_ptr(),
                 None, 0, None, None, lib.stream_handle())
        assert float((_from_nhwc(out, B, H, W, co) - ref).abs().max()) <= _tol(ref, prec)
        pooled = torch.empty(B * H * W, ci, dtype=torch.bfloat16, device=DEV)
        lib.call("sd_bnrelu_pool", lib.SD_BF16, yd.data_ptr(), scd.data_ptr(), shd.data_ptr(), B, Hs, Ws, ci,
                 pooled.data_ptr(), lib.stream_handle())
        xp = torch.relu(yq * sc[None, :, None, None] + sh[None, :, None, None])
        xp = F.max_pool2d(xp, 2).to(torch.bfloat16).float()
        assert float((_from_nhwc(pooled, B, H, W, ci) - xp).abs().max()) <= 1e-2 * (1 + float(xp.abs().max()))
        src = lib.make_src(pooled, ci, H, W, taps=9)
    rows = lib.call("sd_conv_gemm_stat_rows", _sd(prec), B, H, W, co)
    stats = torch.empty(rows, co, 2, device=DEV)
    lib.call("sd_conv_gemm", _sd(prec), src, B, H, W, wp.data_ptr(), co, kpad, lib.SD_EPI_STATS, out.data_ptr(),
             None, 0, None, stats.data_ptr(), lib.stream_handle())
    got = _from_nhwc(out, B, H, W, co)
    assert float((got - ref).abs().max()) <= _tol(ref, prec)
    st = stats.double().sum(0).cpu()
    r64 = ref.double()
    # bf16: the statistics are of the bf16-rounded stored values (what the consumer reads), so the
    # per-channel sum differs from the fp32 reference by ~sqrt(n) rounding errors of ~2^-9
    n = B * H * W
    atol = (1e-3 if prec == "fp32" else 5e-3 * n ** 0.5) * (1 + float(r64.abs().max()))
    assert torch.allclose(st[:, 0], r64.sum((0, 2, 3)), rtol=1e-3, atol=atol)


@pytest.mark.parametrize("prec", ["fp32", "bf16"])
@pytest.mark.parametrize("B,H,W,c0,c1,co", [(2, 8, 12, 16, 16, 16), (2, 15, 20, 64, 64, 64),
                                              # split points at 8-channel (not 16-channel) boundaries: the
                                              # 16-B epilogue pieces of lanes l / l+32 on either side
                                              (1, 16, 32, 8, 24, 32), (1, 16, 64, 24, 40, 64)])
def test_conv3x3_dual_source_and_dgrad_split(prec, B, H, W, c0, c1, co):
    lib = L()
    torch.manual_seed(1)
    u = torch.randn(B, c0, H, W).to(_adt(prec)).float()
    s = torch.randn(B, c1, H, W).to(_adt(prec)).float()
    sc, sh = torch.rand(c1) + 0.5, torch.randn(c1) * 0.1
    w = (torch.randn(co, c0 + c1, 3, 3) / 12).to(_adt(prec)).float()
    xs = torch.relu(s * sc[None, :, None, None] + sh[None, :, None, None])
    x = torch.cat([u, xs if prec == "fp32" else xs.to(torch.bfloat16).float()], 1).requires_grad_(True)
    ref = F.conv2d(x, w, padding=1)
    wp, kpad = _pack3(w, c0 + c1, False, prec)
    ud, sd_, scd, shd = _nhwc(u, prec), _nhwc(s, prec), sc.to(DEV), sh.to(DEV)
    src = lib.make_src(ud, c0, H, W, taps=9, src1=sd_, c1=c1, bn1=(scd, shd))
    out = torch.empty(B * H * W, co, dtype=_adt(prec), device=DEV)
    lib.call("sd_conv_gemm", _sd(prec), src, B, H, W, wp.data_ptr(), co, kpad, lib.SD_EPI_STORE, out.data_ptr(), None,
             0, None, None, lib.stream_handle())
    assert float((_from_nhwc(out, B, H, W, co) - ref).abs().max()) <= _tol(ref, prec)
    # dgrad with split epilogue (cat backward)
    dy = torch.randn(B, co, H, W).to(_adt(prec)).float()
    ref.backward(dy)
    wd, kpd = _pack3(w, c0 + c1, True, prec)
    du = torch.empty(B * H * W, c0, dtype=_adt(prec), device=DEV)
    ds = torch.empty(B * H * W, c1, dtype=_adt(prec), device=DEV)
    dyd = _nhwc(dy, prec)
    dsrc = lib.make_src(dyd, co, H, W, taps=9)
    lib.call("sd_conv_gemm", _sd(prec), dsrc, B, H, W, wd.data_ptr(), c0 + c1, kpd, lib.SD_EPI_SPLIT, du.data_ptr(),
             ds.data_ptr(), c0, None, None, lib.stream_handle())
    gx = x.grad
    assert float((_from_nhwc(du, B, H, W, c0) - gx[:, :c0]).abs().max()) <= _tol(gx, prec)
    assert float((_from_nhwc(ds, B, H, W, c1) - gx[:, c0:]).abs().max()) <= _tol(gx, prec)
    N = c0 + c1
    if prec == "bf16" and (N == 32 or N % 64 == 0):
        # SPLIT_STATS: the same stores, plus per-column sums of the stored values (ConvTranspose bias gradient)
        du2, ds2 = torch.empty_like(du), torch.empty_like(ds)
        rows = lib.call("sd_conv_gemm_stat_rows", lib.SD_BF16, B, H, W, N)
        st = torch.empty(rows, N, 2, device=DEV)
        lib.call("sd_conv_gemm", lib.SD_BF16, dsrc, B, H, W, wd.data_ptr(), N, kpd, lib.SD_EPI_SPLIT_STATS,
                 du2.data_ptr(), ds2.data_ptr(), c0, None, st.data_ptr(), lib.stream_handle())
        assert torch.equal(du2, du) and torch.equal(ds2, ds)
        bias_grad = torch.empty(c0, device=DEV)
        lib.call("sd_stat_rows_sum", st.data_ptr(), rows, N, c0, bias_grad.data_ptr(), lib.stream_handle())
        ref_sum = du.double().sum(0).float()
        assert torch.allclose(bias_grad, ref_sum, rtol=1e-4, atol=1e-3)
        # the same sums as an SD_W_ROWSUM job of the batched reduce, beside a weight-gradient job: bit-identical
        slab = torch.randn(3, 8, 9 * 8, device=DEV)
        dw_one, dw_bat, bias_bat = torch.empty(8, 8, 9, device=DEV), torch.empty(8, 8, 9, device=DEV), torch.empty(c0, device=DEV)
        lib.call("sd_wgrad_reduce", slab.data_ptr(), 3, 8, 72, lib.SD_W_CONV3, 8, dw_one.data_ptr(), lib.stream_handle())
        jobs = (lib.SdWredJob * 2)(lib.SdWredJob(slab.data_ptr(), 3, 8, 72, lib.SD_W_CONV3, 8, dw_bat.data_ptr()),
                                   lib.SdWredJob(st.data_ptr(), rows, 1, N, lib.SD_W_ROWSUM, c0, bias_bat.data_ptr()))
        lib.call("sd_wgrad_reduce_batch", jobs, 2, lib.stream_handle())
        assert torch.equal(bias_bat, bias_grad) and torch.equal(dw_bat, dw_one)


@pytest.mark.parametrize("prec", ["fp32", "bf16"])
@pytest.mark.parametrize("B,H,W,ci,co", [(2, 10, 14, 24, 32),
                                         # bf16 halo wgrad: 64-row dy blocks, flattened tiles of any shape
                                         (2, 15, 20, 64, 64), (1, 30, 40, 40, 128), (1, 13, 50, 16, 192),
                                         (1, 9, 300, 8, 64),
                                         # warp-specialised wgrad (M % 64, x channels % 64): 2 x-channel blocks,
                                         # 2 dy blocks, ragged tiles, many tiles per split
                                         (2, 30, 40, 128, 64), (1, 13, 50, 64, 128), (3, 17, 33, 64, 64),
                                         (1, 120, 160, 64, 64),
                                         # M = 32 / 32-channel x blocks (the full-resolution layers)
                                         (2, 12, 40, 32, 32), (1, 24, 64, 64, 32), (2, 15, 20, 32, 64),
                                         (1, 48, 64, 32, 32)])
def test_conv3x3_wgrad(prec, B, H, W, ci, co):
    lib = L()
    torch.manual_seed(2)
    x = torch.randn(B, ci, H, W).to(_adt(prec)).float()
    dy = torch.randn(B, co, H, W).to(_adt(prec)).float()
    w = torch.zeros(co, ci, 3, 3, requires_grad=True)
    F.conv2d(x, w, padding=1).backward(dy)
    dyd, xd = _nhwc(dy, prec), _nhwc(x, prec)
    a = lib.make_src(dyd, co, H, W, taps=1)
    b = lib.make_src(xd, ci, H, W, taps=9)
    sp = lib.call("sd_wgrad_splits", _sd(prec), B, H, W, co, 9 * ci)
    slab = torch.empty(sp * co * 9 * ci, device=DEV)
    dw = torch.empty(co, ci, 3, 3, device=DEV)
    lib.call("sd_wgrad_gemm", _sd(prec), a, b, B, H, W, co, 9 * ci, slab.data_ptr(), sp, lib.stream_handle())
    lib.call("sd_wgrad_reduce", slab.data_ptr(), sp, co, 9 * ci, lib.SD_W_CONV3, ci, dw.data_ptr(), lib.stream_handle())
    ref = w.grad
    assert float((dw.cpu() - ref).abs().max()) <= (1e-4 if prec == "fp32" else 1e-2) * (1 + float(ref.abs().max()))


@pytest.mark.parametrize("B,H,W,ci,co", [(2, 30, 40, 64, 64), (1, 15, 20, 128, 128), (2, 10, 14, 32, 64),
                                         (1, 24, 64, 32, 32), (1, 16, 64, 64, 32)])
def test_conv3x3_wgrad_bn_relu_source(B, H, W, ci, co):
    """bf16 wgrad whose x operand is relu(bn(y)) applied while the halo is staged (the training path)."""
    lib = L()
    torch.manual_seed(3)
    y = torch.randn(B, ci, H, W).to(torch.bfloat16).float()
    sc = (torch.rand(ci) + 0.5) * torch.where(torch.rand(ci) < 0.2, -1.0, 1.0)
    sh = torch.randn(ci) * 0.3
    x = torch.relu(y * sc.view(1, -1, 1, 1) + sh.view(1, -1, 1, 1)).to(torch.bfloat16).float()
    dy = torch.randn(B, co, H, W).to(torch.bfloat16).float()
    w = torch.zeros(co, ci, 3, 3, requires_grad=True)
    F.conv2d(x, w, padding=1).backward(dy)
    a = lib.make_src(_nhwc(dy, "bf16"), co, H, W, taps=1)
    b = lib.make_src(_nhwc(y, "bf16"), ci, H, W, taps=9, bn0=(sc.to(DEV), sh.to(DEV)))
    sp = lib.call("sd_wgrad_splits", lib.SD_BF16, B, H, W, co, 9 * ci)
    slab = torch.empty(sp * co * 9 * ci, device=DEV)
    dw = torch.empty(co, ci, 3, 3, device=DEV)
    lib.call("sd_wgrad_gemm", lib.SD_BF16, a, b, B, H, W, co, 9 * ci, slab.data_ptr(), sp, lib.stream_handle())
    lib.call("sd_wgrad_reduce", slab.data_ptr(), sp, co, 9 * ci, lib.SD_W_CONV3, ci, dw.data_ptr(), lib.stream_handle())
    ref = w.grad
    assert float((dw.cpu() - ref).abs().max()) <= 1e-2 * (1 + float(ref.abs().max()))


@pytest.mark.parametrize("B,H,W,ci,co", [(2, 30, 40, 128, 64), (1, 15, 20, 128, 128), (2, 10, 14, 32, 64),
                                         (1, 24, 64, 32, 32), (1, 16, 64, 64, 32), (3, 17, 33, 64, 64),
                                         (1, 48, 64, 32, 32), (2, 15, 20, 256, 64),
                                         # enc1.0: 8-channel x, no dgrad (dy not written; k_halo_wgrad<32, true, true>)
                                         (2, 32, 64, 8, 32), (1, 30, 50, 8, 32), (3, 70, 90, 8, 32)])
def test_conv3x3_wgrad_fused_bn_backward(monkeypatch, B, H, W, ci, co):
    """sd_wgrad_gemm_bnbwd: dy = BatchNorm-backward apply of (da, y) formed while staging (written out for the
    dgrad) and the weight gradient on it, vs sd_bn_bwd_apply's formula in fp32 then F.conv2d backward. The 8-channel
    x layout (two tiles in flight) writes the same slab bits as the 32-channel chunk layout (SD_WG_X8=0)."""
    lib = L()
    torch.manual_seed(5)
    yx = torch.randn(B, ci, H, W).to(torch.bfloat16).float()
    scx = (torch.rand(ci) + 0.5) * torch.where(torch.rand(ci) < 0.2, -1.0, 1.0)
    shx = torch.randn(ci) * 0.3
    x = torch.relu(yx * scx.view(1, -1, 1, 1) + shx.view(1, -1, 1, 1)).to(torch.bfloat16).float()
    # BatchNorm backward operands of the conv's output layer: raw output y, upstream gradient da
    y = (torch.randn(B, co, H, W) * 2 + 0.5).to(torch.bfloat16).float()
    da = torch.randn(B, co, H, W).to(torch.bfloat16).float()
    mean, invstd = torch.randn(co) * 0.5, torch.rand(co) + 0.5
    gamma = (torch.rand(co) + 0.5) * torch.where(torch.rand(co) < 0.2, -1.0, 1.0)
    sc = gamma * invstd
    sh = torch.randn(co) * 0.2 - mean * sc
    coef = torch.stack([sc, torch.randn(co) * 0.1, torch.randn(co) * 0.1], 1).contiguous()
    v = lambda t: t.view(1, -1, 1, 1)  # noqa: E731
    dz = torch.where(y * v(sc) + v(sh) > 0, da, torch.zeros_like(da))
    dy_ref = v(coef[:, 0]) * (dz - v(coef[:, 1]) - (y - v(mean)) * v(invstd) * v(coef[:, 2]))
    w = torch.zeros(co, ci, 3, 3, requires_grad=True)
    F.conv2d(x, w, padding=1).backward(dy_ref)
    dyd = torch.full((B * H * W, co), float("nan"), dtype=torch.bfloat16, device=DEV)
    dev = [t.to(DEV).contiguous() for t in (sc, sh, mean, invstd, coef)]
    write_dy = ci % 32 == 0
    a = lib.make_src(dyd if write_dy else None, co, H, W, taps=1)
    b = lib.make_src(_nhwc(yx, "bf16"), ci, H, W, taps=9, bn0=(scx.to(DEV), shx.to(DEV)))
    blocks = (ci // 64 if ci % 64 == 0 else ci // 32) if write_dy else 1
    assert lib.call("sd_wgrad_bnbwd_ok", lib.SD_BF16, a, b, co, 9 * ci) == blocks
    if not write_dy:  # that kernel has no dy destination
        assert lib.call("sd_wgrad_bnbwd_ok", lib.SD_BF16, lib.make_src(dyd, co, H, W, taps=1), b, co, 9 * ci) == 0
    sp = lib.call("sd_wgrad_splits", lib.SD_BF16, B, H, W, co, 9 * ci)
    slab = torch.empty(sp * co * 9 * ci, device=DEV)
    dw = torch.empty(co, ci, 3, 3, device=DEV)
    dad, yd = _nhwc(da, "bf16"), _nhwc(y, "bf16")
    lib.call("sd_wgrad_gemm_bnbwd", lib.SD_BF16, a, b, B, H, W, co, 9 * ci, dad.data_ptr(), yd.data_ptr(),
             *[t.data_ptr() for t in dev], slab.data_ptr(), sp, lib.stream_handle())
    if ci <= 8:
        assert lib.kernel_name("sd_wgrad_bnbwd_kernel_name", a, b, co, 9 * ci) == "k_halo_wgrad<32, true, true>"
        monkeypatch.setenv("SD_WG_X8", "0")
        slab0 = torch.empty_like(slab)
        lib.call("sd_wgrad_gemm_bnbwd", lib.SD_BF16, a, b, B, H, W, co, 9 * ci, dad.data_ptr(), yd.data_ptr(),
                 *[t.data_ptr() for t in dev], slab0.data_ptr(), sp, lib.stream_handle())
        monkeypatch.delenv("SD_WG_X8")
        torch.cuda.synchronize()
        assert torch.equal(slab, slab0)
    lib.call("sd_wgrad_reduce", slab.data_ptr(), sp, co, 9 * ci, lib.SD_W_CONV3, ci, dw.data_ptr(), lib.stream_handle())
    got_dy = _from_nhwc(dyd, B, H, W, co)
    if write_dy:  # every dy element written once (no NaN left), each within bf16 rounding of the fp32 formula
        assert not torch.isnan(got_dy).any()
        assert float(((got_dy - dy_ref).abs() - 2 ** -8 * dy_ref.abs()).max()) <= 1e-5 * (1 + float(dy_ref.abs().max()))
    else:
        assert torch.isnan(got_dy).all()
    ref = w.grad
    assert float((dw.cpu() - ref).abs().max()) <= 1e-2 * (1 + float(ref.abs().max()))


@pytest.mark.parametrize("B,H,W,c0,c1,co", [(2, 30, 40, 64, 0, 128), (1, 24, 64, 96, 0, 128), (1, 15, 20, 128, 0, 256),
                                             (2, 17, 33, 64, 0, 128), (2, 20, 30, 32, 96, 128), (1, 30, 40, 128, 128, 256),
                                             (1, 15, 20, 256, 256, 512)])
def test_conv3x3_wgrad_co128_blocks_bit_identical(monkeypatch, B, H, W, c0, c1, co):
    """Plain weight gradients with M % 128 == 0 run 128 dy x 32 x-channel blocks (default; SD_WS_CO128=0: 64 x 64).
    Every MFMA wave keeps its 64 dy rows x 16 x channels x 9 taps and the split-K tile ranges are the same, so each dW
    element is the same MFMA chain over the same pixels: the reduced dW are bit-identical. Single and concatenated
    (dual-source, 32-aligned boundary) x, both halo layouts, ragged tiles; and against fp64."""
    lib = L()
    torch.manual_seed(13)
    ys = [torch.randn(B, c, H, W).to(torch.bfloat16).float() for c in (c0, c1) if c]
    bns = [((torch.rand(y.shape[1]) + 0.5) * torch.where(torch.rand(y.shape[1]) < 0.2, -1.0, 1.0),
            torch.randn(y.shape[1]) * 0.3) for y in ys]
    x = torch.cat([torch.relu(torch.addcmul(h.view(1, -1, 1, 1), y, s.view(1, -1, 1, 1))).to(torch.bfloat16).double()
                   for y, (s, h) in zip(ys, bns)], 1)
    ci = c0 + c1
    dy = torch.randn(B, co, H, W).to(torch.bfloat16).float()
    kw = dict(src1=_nhwc(ys[1], "bf16"), c1=c1, bn1=tuple(t.to(DEV) for t in bns[1])) if c1 else {}
    b = lib.make_src(_nhwc(ys[0], "bf16"), c0, H, W, taps=9, bn0=tuple(t.to(DEV) for t in bns[0]), **kw)
    a = lib.make_src(_nhwc(dy, "bf16"), co, H, W, taps=1)
    sp = lib.call("sd_wgrad_splits", lib.SD_BF16, B, H, W, co, 9 * ci)
    out = {}
    for mode in ("1", "0"):
        monkeypatch.setenv("SD_WS_CO128", mode)
        name = lib.kernel_name("sd_wgrad_kernel_name", lib.SD_BF16, a, b, co, 9 * ci)
        assert name.startswith("k_halo_wgrad_ws<128, 32," if mode == "1" else "k_halo_wgrad_ws<64, "), name
        slab = torch.empty(sp * co * 9 * ci, device=DEV)
        dw = torch.empty(co, ci, 3, 3, device=DEV)
        lib.call("sd_wgrad_gemm", lib.SD_BF16, a, b, B, H, W, co, 9 * ci, slab.data_ptr(), sp, lib.stream_handle())
        lib.call("sd_wgrad_reduce", slab.data_ptr(), sp, co, 9 * ci, lib.SD_W_CONV3, ci, dw.data_ptr(),
                 lib.stream_handle())
        torch.cuda.synchronize()
        out[mode] = dw.cpu()
    assert torch.equal(out["1"], out["0"]), float((out["1"] - out["0"]).abs().max())
    ref = torch.nn.grad.conv2d_weight(x, (co, ci, 3, 3), dy.double(), padding=1).float()
    assert float((out["1"] - ref).abs().max()) <= 1e-3 * float(ref.abs().max())


@pytest.mark.parametrize("B,H,W,ci,co", [(2, 30, 40, 64, 64), (1, 15, 20, 128, 128), (3, 17, 33, 64, 64),
                                         (1, 24, 64, 64, 128), (2, 60, 80, 128, 64)])
@pytest.mark.parametrize("fused", [False, True])
def test_conv3x3_wgrad_mfma32_matches_mfma16(monkeypatch, B, H, W, ci, co, fused):
    """The 64 x 64-block weight gradient on v_mfma_f32_32x32x16_bf16 (SD_WS_MF32=1, opt-in) against its default
    v_mfma_f32_16x16x32_bf16 form on the same bf16 operands: both accumulate the same 16-pixel chunks in the same order
    (the 16x16x32 k-step's two k halves are pixels 0-15 and 16-31), so the reduced dW and the fused BatchNorm-backward
    dy stores are bit-identical (measured at every step shape, tools/conv_micro.py --wgrad-step); both against fp64."""
    lib = L()
    monkeypatch.setenv("SD_WS_CO128", "0")  # the 64 x 64 blocks at M % 128 == 0 too
    torch.manual_seed(11)
    yx = torch.randn(B, ci, H, W).to(torch.bfloat16).float()
    scx = (torch.rand(ci) + 0.5) * torch.where(torch.rand(ci) < 0.2, -1.0, 1.0)
    shx = torch.randn(ci) * 0.3
    x = torch.relu(yx * scx.view(1, -1, 1, 1) + shx.view(1, -1, 1, 1)).to(torch.bfloat16).double()
    b = lib.make_src(_nhwc(yx, "bf16"), ci, H, W, taps=9, bn0=(scx.to(DEV), shx.to(DEV)))
    sp = lib.call("sd_wgrad_splits", lib.SD_BF16, B, H, W, co, 9 * ci)
    if fused:
        y = (torch.randn(B, co, H, W) * 2 + 0.5).to(torch.bfloat16).float()
        da = torch.randn(B, co, H, W).to(torch.bfloat16).float()
        sc, sh = torch.rand(co) + 0.5, torch.randn(co) * 0.2
        mean, invstd = torch.randn(co) * 0.5, torch.rand(co) + 0.5
        coef = torch.stack([sc, torch.randn(co) * 0.1, torch.randn(co) * 0.1], 1).contiguous()
        dev = [t.to(DEV).contiguous() for t in (sc, sh, mean, invstd, coef)]
        dad, yd = _nhwc(da, "bf16"), _nhwc(y, "bf16")
    else:
        dy = torch.randn(B, co, H, W).to(torch.bfloat16).float()
    out = {}
    for mode in ("1", "0"):
        monkeypatch.setenv("SD_WS_MF32", mode)
        slab = torch.empty(sp * co * 9 * ci, device=DEV)
        dw = torch.empty(co, ci, 3, 3, device=DEV)
        if fused:
            dyd = torch.full((B * H * W, co), float("nan"), dtype=torch.bfloat16, device=DEV)
            a = lib.make_src(dyd, co, H, W, taps=1)
            lib.call("sd_wgrad_gemm_bnbwd", lib.SD_BF16, a, b, B, H, W, co, 9 * ci, dad.data_ptr(), yd.data_ptr(),
                     *[t.data_ptr() for t in dev], slab.data_ptr(), sp, lib.stream_handle())
        else:
            dyd = _nhwc(dy, "bf16")
            a = lib.make_src(dyd, co, H, W, taps=1)
            lib.call("sd_wgrad_gemm", lib.SD_BF16, a, b, B, H, W, co, 9 * ci, slab.data_ptr(), sp, lib.stream_handle())
        name = lib.kernel_name("sd_wgrad_kernel_name", lib.SD_BF16, a, b, co, 9 * ci)
        assert name.endswith(", true>") == (mode == "1"), name
        lib.call("sd_wgrad_reduce", slab.data_ptr(), sp, co, 9 * ci, lib.SD_W_CONV3, ci, dw.data_ptr(),
                 lib.stream_handle())
        torch.cuda.synchronize()
        out[mode] = (dw.cpu(), dyd.cpu().clone())
    dw1, dw0 = out["1"][0], out["0"][0]
    if fused:
        assert torch.equal(out["1"][1], out["0"][1])
        dyr = _from_nhwc(out["1"][1].to(DEV), B, H, W, co).double()
    else:
        dyr = dy.double()
    ref = torch.nn.grad.conv2d_weight(x, (co, ci, 3, 3), dyr, padding=1).float()
    scale = float(ref.abs().max())
    assert torch.equal(dw1, dw0), float((dw1 - dw0).abs().max()) / scale
    # x here is relu(y*sc + sh) with a separate multiply and add, the kernel's one fma: a rare x differs by a bf16 ulp
    assert float((dw1 - ref).abs().max()) <= 1e-3 * scale


@pytest.mark.parametrize("prec", ["fp32", "bf16"])
@pytest.mark.parametrize("B,h,w_,ci,co", [(2, 5, 7, 32, 16), (2, 12, 20, 64, 32), (1, 15, 20, 128, 64),
                                          # k_convt (forward, K <= 128): many 128-pixel tiles per block, ragged
                                          # last tile; K 256 / 512: the tiled GEMM
                                          (3, 60, 90, 64, 32), (2, 9, 13, 256, 128), (1, 6, 10, 512, 256)])
def test_convT_fwd_dgrad_wgrad_bias(prec, B, h, w_, ci, co):
    lib = L()
    torch.manual_seed(3)
    xr = torch.randn(B, ci, h, w_).to(_adt(prec)).float()
    sc, sh = torch.rand(ci) + 0.5, torch.randn(ci) * 0.1
    x = torch.relu(xr * sc[None, :, None, None] + sh[None, :, None, None])
    if prec == "bf16":
        x = x.to(torch.bfloat16).float()
    wt = (torch.randn(ci, co, 2, 2) / 8).to(_adt(prec)).float().requires_grad_(True)
    bias = torch.randn(co).requires_grad_(True)
    xg = x.clone().requires_grad_(True)
    ref = F.conv_transpose2d(xg, wt, bias, stride=2)
    s = lib.stream_handle()
    kf = ((ci + 63) // 64) * 64
    wpf = torch.empty(4 * co * kf, dtype=_adt(prec), device=DEV)
    wtd = wt.detach().contiguous().to(DEV)
    lib.call("sd_pack_convT_w", _sd(prec), wtd.data_ptr(), ci, co, 0, kf, wpf.data_ptr(), s)
    xrd, scd, shd = _nhwc(xr, prec), sc.to(DEV), sh.to(DEV)
    src = lib.make_src(xrd, ci, h, w_, taps=1, bn0=(scd, shd))
    out = torch.empty(B * 4 * h * w_, co, dtype=_adt(prec), device=DEV)
    bd = bias.detach().to(DEV)
    lib.call("sd_conv_gemm", _sd(prec), src, B, h, w_, wpf.data_ptr(), 4 * co, kf, lib.SD_EPI_PIXSHUF, out.data_ptr(),
             None, 0, bd.data_ptr(), None, s)
    assert float((_from_nhwc(out, B, 2 * h, 2 * w_, co) - ref.detach()).abs().max()) <= _tol(ref, prec)
    dout = torch.randn(B, co, 2 * h, 2 * w_).to(_adt(prec)).float()
    ref.backward(dout)
    dout_d = _nhwc(dout, prec)
    # dgrad
    kd = ((4 * co + 63) // 64) * 64
    wpd = torch.empty(ci * kd, dtype=_adt(prec), device=DEV)
    lib.call("sd_pack_convT_w", _sd(prec), wtd.data_ptr(), ci, co, 1, kd, wpd.data_ptr(), s)
    dsrc = lib.make_src(dout_d, co, 2 * h, 2 * w_, taps=4)
    dx = torch.empty(B * h * w_, ci, dtype=_adt(prec), device=DEV)
    lib.call("sd_conv_gemm", _sd(prec), dsrc, B, h, w_, wpd.data_ptr(), ci, kd, lib.SD_EPI_STORE, dx.data_ptr(), None, 0,
             None, None, s)
    assert float((_from_nhwc(dx, B, h, w_, ci) - xg.grad).abs().max()) <= _tol(xg.grad, prec)
    # wgrad
    sp = lib.call("sd_wgrad_splits", _sd(prec), B, h, w_, ci, 4 * co)
    slab = torch.empty(sp * ci * 4 * co, device=DEV)
    dw = torch.empty(ci, co, 2, 2, device=DEV)
    lib.call("sd_wgrad_gemm", _sd(prec), src, dsrc, B, h, w_, ci, 4 * co, slab.data_ptr(), sp, s)
    lib.call("sd_wgrad_reduce", slab.data_ptr(), sp, ci, 4 * co, lib.SD_W_CONVT, ci, dw.data_ptr(), s)
    assert float((dw.cpu() - wt.grad).abs().max()) <= (1e-4 if prec == "fp32" else 1e-2) * (1 + float(wt.grad.abs().max()))
    # bias grad
    part = torch.empty(lib.call("sd_chan_reduce_rows", B * 4 * h * w_, co) * co * 2, device=DEV)
    db = torch.empty(co, device=DEV)
    lib.call("sd_chan_sum", _sd(prec), dout_d.data_ptr(), B * 4 * h * w_, co, part.data_ptr(), db.data_ptr(), s)
    # fp32 sums of B*4*h*w values: the tolerance grows with sqrt(count)
    assert torch.allclose(db.cpu(), bias.grad, atol=1e-3 * (1 + (B * 4 * h * w_) ** 0.5 / 100))


@pytest.mark.parametrize("case,B,h,w_,ci,co", [
    ("fwd", 64, 15, 20, 512, 256),   # up4 forward shape, identity source, K = 512: stays on the tiled kernel
    ("fwd", 63, 15, 20, 1024, 256),  # K = 1024, PIXSHUF + bias, ragged M (18900 rows): the ring
    ("fwd_bn", 64, 15, 20, 512, 256),  # BN+ReLU source: stays on the tiled kernel
    ("dgrad", 64, 15, 20, 512, 256),  # up4 dgrad: 4 sub-pixel taps of 256 channels, K = 1024
    ("dgrad", 64, 30, 40, 256, 128),  # up3 dgrad: K = 512 (8 K tiles), stays on the tiled kernel
    ("dgrad", 8, 64, 64, 128, 256),   # 8 x 64 x 64 rows, K = 1024, N = 128: 256 tiles, one per block
    ("dgrad", 2, 64, 64, 128, 512),   # K = 2048 over 64 tiles: stays on the tiled kernel (< 256 tiles)
])
def test_conv_fwd_tilings_bit_identical(monkeypatch, case, B, h, w_, ci, co):
    """The FA GEMMs' three forms store the same bits: k_conv_fwd_bf16 at 64 x 128 (SD_FWD_BM=64) and at 128 x 128 (the
    default at large M), and the opt-in k_conv_fwd_ring (persistent, LDS-DMA ring) — one MFMA order over the same
    fragments (model.py:67-73: the ConvTranspose2d forward and its data gradient)."""
    lib = L()
    torch.manual_seed(21)
    s = lib.stream_handle()
    wt = (torch.randn(ci, co, 2, 2) / (2 * ci ** 0.5)).to(torch.bfloat16).float()
    if case.startswith("fwd"):
        xr = torch.randn(B, ci, h, w_).to(torch.bfloat16).float()
        bn = case == "fwd_bn"
        sc, sh = (torch.rand(ci) + 0.5, torch.randn(ci) * 0.3) if bn else (torch.ones(ci), torch.zeros(ci))
        bias = torch.randn(co)
        kp = ((ci + 63) // 64) * 64
        wp = torch.empty(4 * co * kp, dtype=torch.bfloat16, device=DEV)
        lib.call("sd_pack_convT_w", lib.SD_BF16, wt.contiguous().to(DEV).data_ptr(), ci, co, 0, kp, wp.data_ptr(), s)
        keep = [_nhwc(xr, "bf16"), sc.to(DEV), sh.to(DEV), bias.to(DEV)]
        src = lib.make_src(keep[0], ci, h, w_, taps=1, bn0=(keep[1], keep[2]) if bn else None)
        N, epi, rows, bptr = 4 * co, lib.SD_EPI_PIXSHUF, B * 4 * h * w_, keep[3].data_ptr()
        x = torch.relu(xr * sc[None, :, None, None] + sh[None, :, None, None]).to(torch.bfloat16).float() if bn else xr
        ref = F.conv_transpose2d(x.to(DEV), wt.to(DEV), bias.to(DEV), stride=2).cpu()
        shape = (B, 2 * h, 2 * w_, co)
    else:
        dy = torch.randn(B, co, 2 * h, 2 * w_).to(torch.bfloat16).float()
        kp = ((4 * co + 63) // 64) * 64
        wp = torch.empty(ci * kp, dtype=torch.bfloat16, device=DEV)
        lib.call("sd_pack_convT_w", lib.SD_BF16, wt.contiguous().to(DEV).data_ptr(), ci, co, 1, kp, wp.data_ptr(), s)
        keep = [_nhwc(dy, "bf16")]
        src = lib.make_src(keep[0], co, 2 * h, 2 * w_, taps=4)
        N, epi, rows, bptr = ci, lib.SD_EPI_STORE, B * h * w_, None
        ref = F.conv2d(dy.to(DEV), wt.to(DEV), stride=2).cpu()  # ConvTranspose2d's data gradient
        shape = (B, h, w_, ci)
    outs = {}
    M = B * h * w_
    ring = case != "fwd_bn" and (4 * co if case == "dgrad" else ci) >= 1024 and (M + 127) // 128 * ((N + 127) // 128) >= 256
    big = "k_conv_fwd_bf16<128, 128, 2, 2, true, 1>" if M >= 128 * 96 else "k_conv_fwd_bf16<64, 128, 2, 2, true, 1>"
    modes = (("64", "0", "k_conv_fwd_bf16<64, 128, 2, 2, true, 1>"), ("", "0", big),
             ("", "1", "k_conv_fwd_ring" if ring else big))
    for bm, rg, kname in modes:
        monkeypatch.setenv("SD_FWD_BM", bm)
        monkeypatch.setenv("SD_FWD_RING", rg)
        assert lib.kernel_name("sd_conv_gemm_kernel_name", lib.SD_BF16, src, B, h, w_, N, epi) == kname
        out = torch.full((rows, shape[3]), float("nan"), dtype=torch.bfloat16, device=DEV)
        lib.call("sd_conv_gemm", lib.SD_BF16, src, B, h, w_, wp.data_ptr(), N, kp, epi, out.data_ptr(), None, 0, bptr,
                 None, s)
        torch.cuda.synchronize()
        outs[bm + rg] = out
    assert torch.equal(outs["0"], outs["640"]) and torch.equal(outs["1"], outs["640"])
    got = outs["0"].float().cpu().reshape(shape).permute(0, 3, 1, 2)
    assert float((got - ref).abs().max()) <= _tol(ref, "bf16")


def test_pool_bwd_first_max_tie_break_and_skip_add():
    lib = L()
    B, H, W, C = 1, 4, 4, 8
    y = torch.zeros(B, H, W, C)
    y[0, 0, 1, 0] = 5.0  # max at window position 1
    y[0, 2, 2, 1] = -3.0  # all-relu-zero window: ties -> first (position 0)
    sc, sh = torch.ones(C), torch.zeros(C)
    dpool = torch.arange(B * 2 * 2 * C, dtype=torch.float32).reshape(B, 2, 2, C) + 1
    dskip = torch.full((B, H, W, C), 0.5)
    da = torch.empty(B, H, W, C, device=DEV)
    keep = [t.to(DEV) for t in (y, sc, sh, dskip, dpool)]
    lib.call("sd_pool_bwd_add", lib.SD_F32, *[t.data_ptr() for t in keep], B, H, W, C, da.data_ptr(),
             None, None, None, lib.stream_handle())
    # reference: torch max_pool2d backward on relu(y) (NCHW)
    x = torch.relu(y).permute(0, 3, 1, 2).contiguous().requires_grad_(True)
    F.max_pool2d(x, 2).backward(dpool.permute(0, 3, 1, 2))
    ref = x.grad.permute(0, 2, 3, 1) + dskip
    assert torch.equal(da.cpu(), ref)


def test_bilinear_resize_matches_interpolate():
    lib = L()
    torch.manual_seed(4)
    x = torch.rand(3, 45, 61)
    xd = x.to(DEV)
    for ho, wo in ((24, 32), (240, 320), (45, 61), (7, 100)):
        out = torch.empty(3, ho, wo, device=DEV)
        lib.call("sd_resize_bilinear", xd.data_ptr(), 3, 45, 61, out.data_ptr(), ho, wo, 1.0, lib.stream_handle())
        ref = F.interpolate(x[None], size=(ho, wo), mode="bilinear", align_corners=False)[0]
        assert float((out.cpu() - ref).abs().max()) < 1e-5


@pytest.mark.parametrize("prec", ["fp32", "bf16"])
@pytest.mark.parametrize("B,H,W,C", [(2, 8, 12, 32), (1, 16, 20, 256), (3, 6, 4, 64)])
def test_pool_bwd_fused_bn_sums_match_reduce(prec, B, H, W, C):
    """sd_pool_bwd_add's fused BatchNorm-backward sums == sd_bn_bwd_reduce on the da it wrote."""
    lib = L()
    torch.manual_seed(5)
    dt = _adt(prec)
    y = torch.randn(B * H * W, C).to(dt).to(DEV)
    sc, sh = (torch.rand(C) + 0.5).to(DEV), (torch.randn(C) * 0.3).to(DEV)
    sc[::4] *= -1
    mean, invstd = (torch.randn(C) * 0.1).to(DEV), (torch.rand(C) + 0.5).to(DEV)
    dskip = torch.randn(B * H * W, C).to(dt).to(DEV)
    dpool = torch.randn(B * (H // 2) * (W // 2), C).to(dt).to(DEV)
    s = lib.stream_handle()
    rows = lib.call("sd_pool_bwd_rows", B, H, W, C)
    da1 = torch.empty(B * H * W, C, dtype=dt, device=DEV)
    da2 = torch.empty_like(da1)
    part = torch.empty(rows, C, 2, device=DEV)
    lib.call("sd_pool_bwd_add", _sd(prec), y.data_ptr(), sc.data_ptr(), sh.data_ptr(), dskip.data_ptr(),
             dpool.data_ptr(), B, H, W, C, da1.data_ptr(), mean.data_ptr(), invstd.data_ptr(), part.data_ptr(), s)
    lib.call("sd_pool_bwd_add", _sd(prec), y.data_ptr(), sc.data_ptr(), sh.data_ptr(), dskip.data_ptr(),
             dpool.data_ptr(), B, H, W, C, da2.data_ptr(), None, None, None, s)
    rrows = lib.call("sd_chan_reduce_rows", B * H * W, C)
    ref = torch.empty(rrows, C, 2, device=DEV)
    lib.call("sd_bn_bwd_reduce", _sd(prec), da1.data_ptr(), y.data_ptr(), sc.data_ptr(), sh.data_ptr(),
             mean.data_ptr(), invstd.data_ptr(), B * H * W, C, ref.data_ptr(), s)
    torch.cuda.synchronize()
    assert torch.equal(da1, da2)
    got, want = part.double().sum(0), ref.double().sum(0)
    assert torch.allclose(got, want, rtol=1e-4, atol=1e-3 * (1 + float(want.abs().max())))


@pytest.mark.parametrize("prec", ["fp32", "bf16"])
def test_pack_weights_multi_equals_per_tensor_packs(prec):
    """sd_pack_weights (one launch, all kinds) writes exactly what the per-tensor packs write."""
    lib = L()
    s = lib.stream_handle()
    torch.manual_seed(5)
    convs = [(32, 6, 8), (64, 32, 32), (128, 256, 256), (512, 16, 16)]  # (co, ci, ci_pad)
    ups = [(64, 32), (512, 256)]  # (ci, co)
    ws3 = [torch.randn(co, ci, 3, 3, device=DEV) for co, ci, _ in convs]
    wsT = [torch.randn(ci, co, 2, 2, device=DEV) for ci, co in ups]
    jobs, refs, off = [], [], 0
    for w, (co, ci, cp) in zip(ws3, convs):
        for kind, dgrad in ((lib.SD_PACK_CONV3_FWD, 0), (lib.SD_PACK_CONV3_DGRAD, 1)):
            if dgrad and cp != ci:
                continue
            kpad = ((9 * (co if dgrad else cp) + 63) // 64) * 64
            n = (ci if dgrad else co) * kpad
            ref = torch.empty(n, dtype=_adt(prec), device=DEV)
            lib.call("sd_pack_conv3_w", _sd(prec), w.data_ptr(), co, ci, cp, dgrad, kpad, ref.data_ptr(), s)
            jobs.append(lib.SdPackJob(w.data_ptr(), kind, co, ci, cp, kpad, off))
            refs.append((off, ref))
            off += n + 64  # gaps stay untouched
    for w, (ci, co) in zip(wsT, ups):
        for kind, dgrad in ((lib.SD_PACK_CONVT_FWD, 0), (lib.SD_PACK_CONVT_DGRAD, 1)):
            kpad = ((4 * co if dgrad else ci) + 63) // 64 * 64
            n = (ci if dgrad else 4 * co) * kpad
            ref = torch.empty(n, dtype=_adt(prec), device=DEV)
            lib.call("sd_pack_convT_w", _sd(prec), w.data_ptr(), ci, co, dgrad, kpad, ref.data_ptr(), s)
            jobs.append(lib.SdPackJob(w.data_ptr(), kind, co, ci, ci, kpad, off))
            refs.append((off, ref))
            off += n
    out = torch.full((off,), 7.0, dtype=_adt(prec), device=DEV)
    arr = (lib.SdPackJob * len(jobs))(*jobs)
    lib.call("sd_pack_weights", _sd(prec), arr, len(jobs), out.data_ptr(), s)
    torch.cuda.synchronize()
    covered = torch.zeros(off, dtype=torch.bool)
    for o, ref in refs:
        assert torch.equal(out[o:o + ref.numel()].cpu(), ref.cpu())
        covered[o:o + ref.numel()] = True
    assert bool((out.cpu()[~covered] == 7.0).all())


@pytest.mark.parametrize("ck", ["16", "32"])
@pytest.mark.parametrize("B,H,W,ci,co", [(1, 32, 64, 48, 64), (2, 24, 96, 64, 128), (1, 60, 80, 72, 128),
                                         (1, 45, 60, 24, 64), (2, 20, 30, 200, 64), (1, 64, 64, 16, 192),
                                         (1, 36, 64, 72, 64)])
def test_conv3x3_halo_tilings_store_and_stats(monkeypatch, ck, B, H, W, ci, co):
    """bf16 halo conv at every tiling (the default CK=32 chunks with RT=2..3 column tiles per wave: 8x32,
    12x32 (H % 12 == 0), 6x40, whole images; and
    CK=16 with RT up to 4 via SD_HALO_CK=16), STORE and STATS epilogues, partial chunks."""
    monkeypatch.setenv("SD_HALO_CK", ck)
    lib = L()
    torch.manual_seed(3)
    y = torch.randn(B, ci, H, W).to(torch.bfloat16).float()
    sc, sh = torch.rand(ci) + 0.5, torch.randn(ci) * 0.2
    w = (torch.randn(co, ci, 3, 3) / (3 * ci ** 0.5)).to(torch.bfloat16).float()
    x = torch.relu(y * sc[None, :, None, None] + sh[None, :, None, None]).to(torch.bfloat16).float()
    wp, kpad = _pack3(w, ci, False, "bf16")
    yd = _nhwc(y, "bf16")
    for epi in (lib.SD_EPI_STORE, lib.SD_EPI_STATS):
        bn = epi == lib.SD_EPI_STATS
        src = lib.make_src(yd, ci, H, W, taps=9, bn0=(sc.to(DEV), sh.to(DEV)) if bn else None)
        ref = F.conv2d(x if bn else y, w, padding=1)
        out = torch.full((B * H * W, co), float("nan"), dtype=torch.bfloat16, device=DEV)
        rows = lib.call("sd_conv_gemm_stat_rows", lib.SD_BF16, B, H, W, co)
        stats = torch.empty(rows, co, 2, device=DEV)
        lib.call("sd_conv_gemm", lib.SD_BF16, src, B, H, W, wp.data_ptr(), co, kpad, epi, out.data_ptr(), None, 0,
                 None, stats.data_ptr() if bn else None, lib.stream_handle())
        got = _from_nhwc(out, B, H, W, co)
        name = lib.kernel_name("sd_conv_gemm_kernel_name", lib.SD_BF16, src, B, H, W, co, epi)
        assert float((got - ref).abs().max()) <= _tol(ref, "bf16"), (name, int(torch.isnan(got).sum()),
                                                                       float((got == 0).float().mean()))
        if bn:  # statistics of exactly the stored bf16 values
            st = stats.double().sum(0).cpu()
            g64 = got.double()
            assert torch.allclose(st[:, 0], g64.sum((0, 2, 3)), rtol=1e-5, atol=1e-3)
            assert torch.allclose(st[:, 1], (g64 * g64).sum((0, 2, 3)), rtol=1e-5, atol=1e-3)


@pytest.mark.parametrize("prec", ["fp32", "bf16"])
@pytest.mark.parametrize("C,P", [(32, 5000), (16, 777), (64, 4096)])
def test_heads_bnsum_matches_heads_then_reduce(prec, C, P):
    """sd_heads_bnsum == sd_heads (same da bits, head-grad partials, metrics) followed by
    sd_bn_bwd_reduce over the da it stored (sums equal after adding the rows)."""
    lib = L()
    torch.manual_seed(13)
    dt = _adt(prec)
    s = lib.stream_handle()
    y = torch.randn(P, C).to(dt).to(DEV)
    sc, sh = (torch.rand(C) + 0.5).to(DEV), (torch.randn(C) * 0.3).to(DEV)
    sc[::4] *= -1
    mean, invstd = (torch.randn(C) * 0.2).to(DEV), (torch.rand(C) + 0.5).to(DEV)
    wd, wl = (torch.randn(C) * 0.3).to(DEV), (torch.randn(C) * 0.3).to(DEV)
    bd, bl = torch.tensor([0.5], device=DEV), torch.tensor([-0.2], device=DEV)
    target = (torch.rand(P) * 4).to(DEV)
    target[::7] = float("nan")
    valid = (torch.rand(P) > 0.1).to(torch.uint8).to(DEV)
    count = torch.tensor([int(((valid != 0) & torch.isfinite(target)).sum())], dtype=torch.int32, device=DEV)
    rows = lib.call("sd_heads_rows", P)
    NV = 2 * C + 7
    outs = []
    for fused in (True, False):
        da = torch.full((P, C), float("nan"), dtype=dt, device=DEV)
        part = torch.zeros(rows * NV, device=DEV)
        args = (_sd(prec), lib.SD_HEADS_LOSS, y.data_ptr(), sc.data_ptr(), sh.data_ptr(), P, C, wd.data_ptr(),
                bd.data_ptr(), wl.data_ptr(), bl.data_ptr(), None, None, target.data_ptr(), valid.data_ptr(),
                count.data_ptr(), None, None, da.data_ptr(), part.data_ptr())
        if fused:
            bnp = torch.empty(rows, C, 2, device=DEV)
            lib.call("sd_heads_bnsum", *args, mean.data_ptr(), invstd.data_ptr(), bnp.data_ptr(), s)
            bn = bnp.double().sum(0)
        else:
            lib.call("sd_heads", *args, s)
            rr = lib.call("sd_chan_reduce_rows", P, C)
            ref = torch.empty(rr, C, 2, device=DEV)
            lib.call("sd_bn_bwd_reduce", _sd(prec), da.data_ptr(), y.data_ptr(), sc.data_ptr(), sh.data_ptr(),
                     mean.data_ptr(), invstd.data_ptr(), P, C, ref.data_ptr(), s)
            bn = ref.double().sum(0)
        torch.cuda.synchronize()
        outs.append((da.clone(), part.view(rows, NV).double().sum(0), bn))
    (da1, p1, bn1), (da2, p2, bn2) = outs
    # the two instances may contract the gradient products differently: at most 1 bf16 ulp apart
    d = (da1.float() - da2.float()).abs()
    assert float((d > 2 ** -7 * da2.float().abs()).float().mean()) == 0.0
    assert torch.allclose(p1, p2, rtol=1e-5, atol=1e-5)
    assert torch.allclose(bn1, bn2, rtol=1e-4, atol=1e-4 * (1 + float(bn2.abs().max())))


@pytest.mark.parametrize("kmax,kname", [("256", "k_convt<1, "), ("128", "k_conv_fwd_bf16<")])
def test_convT_fwd_k256_both_routes(monkeypatch, kmax, kname):
    """The up3-shaped ConvTranspose2d forward (K = 256, BN+ReLU source, M = 19200 GEMM rows) through k_convt (the weight
    slice in LDS; the default at M >= 16384) and through the tiled GEMM (SD_CONVT_KMAX=128; the default below that M),
    both against the fp32 reference."""
    lib = L()
    monkeypatch.setenv("SD_CONVT_KMAX", kmax)
    torch.manual_seed(12)
    B, h, w_, ci, co = 16, 30, 40, 256, 128
    xr = torch.randn(B, ci, h, w_).to(torch.bfloat16).float()
    sc, sh = torch.rand(ci) + 0.5, torch.randn(ci) * 0.3
    x = torch.relu(xr * sc[None, :, None, None] + sh[None, :, None, None]).to(torch.bfloat16).float()
    wt = (torch.randn(ci, co, 2, 2) / 16).to(torch.bfloat16).float()
    bias = torch.randn(co)
    ref = F.conv_transpose2d(x.to(DEV), wt.to(DEV), bias.to(DEV), stride=2).cpu()
    s = lib.stream_handle()
    wpf = torch.empty(4 * co * ci, dtype=torch.bfloat16, device=DEV)
    lib.call("sd_pack_convT_w", lib.SD_BF16, wt.contiguous().to(DEV).data_ptr(), ci, co, 0, ci, wpf.data_ptr(), s)
    keep = [_nhwc(xr, "bf16"), sc.to(DEV), sh.to(DEV), bias.to(DEV)]
    src = lib.make_src(keep[0], ci, h, w_, taps=1, bn0=(keep[1], keep[2]))
    assert lib.kernel_name("sd_conv_gemm_kernel_name", lib.SD_BF16, src, B, h, w_, 4 * co,
                           lib.SD_EPI_PIXSHUF).startswith(kname)
    out = torch.empty(B * 4 * h * w_, co, dtype=torch.bfloat16, device=DEV)
    lib.call("sd_conv_gemm", lib.SD_BF16, src, B, h, w_, wpf.data_ptr(), 4 * co, ci, lib.SD_EPI_PIXSHUF,
             out.data_ptr(), None, 0, keep[3].data_ptr(), None, s)
    assert float((_from_nhwc(out, B, 2 * h, 2 * w_, co) - ref).abs().max()) <= _tol(ref, "bf16")


def test_convT_fwd_identity_source():
    """bf16 ConvTranspose2d forward from an untransformed source (k_convt<0, ...>: no BN transform)."""
    lib = L()
    torch.manual_seed(4)
    B, h, w_, ci, co = 2, 7, 30, 64, 32
    x = torch.randn(B, ci, h, w_).to(torch.bfloat16).float()
    wt = (torch.randn(ci, co, 2, 2) / 8).to(torch.bfloat16).float()
    bias = torch.randn(co)
    ref = F.conv_transpose2d(x, wt, bias, stride=2)
    s = lib.stream_handle()
    wpf = torch.empty(4 * co * 64, dtype=torch.bfloat16, device=DEV)
    lib.call("sd_pack_convT_w", lib.SD_BF16, wt.contiguous().to(DEV).data_ptr(), ci, co, 0, 64, wpf.data_ptr(), s)
    src = lib.make_src(_nhwc(x, "bf16"), ci, h, w_, taps=1)
    assert lib.kernel_name("sd_conv_gemm_kernel_name", lib.SD_BF16, src, B, h, w_, 4 * co,
                           lib.SD_EPI_PIXSHUF).startswith("k_convt<0, ")  # CT_FWD: no BN transform
    out = torch.empty(B * 4 * h * w_, co, dtype=torch.bfloat16, device=DEV)
    bd = bias.to(DEV)
    lib.call("sd_conv_gemm", lib.SD_BF16, src, B, h, w_, wpf.data_ptr(), 4 * co, 64, lib.SD_EPI_PIXSHUF,
             out.data_ptr(), None, 0, bd.data_ptr(), None, s)
    assert float((_from_nhwc(out, B, 2 * h, 2 * w_, co) - ref).abs().max()) <= _tol(ref, "bf16")


@pytest.mark.parametrize("B,H,W,ci,co", [(2, 32, 64, 32, 32), (1, 48, 64, 32, 32), (2, 30, 40, 64, 64),
                                         (1, 16, 64, 128, 64), (2, 24, 32, 64, 128), (1, 26, 50, 32, 64)])
def test_conv_gemm_bnsum_matches_store_plus_reduce(B, H, W, ci, co):
    """sd_conv_gemm_bnsum: the dgrad-style conv stores exactly what sd_conv_gemm(STORE) stores, and its partial rows
    sum to sd_bn_bwd_reduce's BatchNorm-backward sums over (out, y)."""
    lib = L()
    torch.manual_seed(8)
    s = lib.stream_handle()
    x = torch.randn(B, ci, H, W)
    w = torch.randn(co, ci, 3, 3) / (3 * ci ** 0.5)
    wp, kpad = _pack3(w, ci, False, "bf16")
    src = lib.make_src(_nhwc(x, "bf16"), ci, H, W, taps=9)
    assert lib.call("sd_conv_gemm_bnsum_ok", lib.SD_BF16, src, co) == 1
    y = (torch.randn(B * H * W, co) * 2 + 0.3).to(DEV, torch.bfloat16)
    sc = ((torch.rand(co) + 0.5) * torch.where(torch.rand(co) < 0.2, -1.0, 1.0)).to(DEV)
    sh, mean, invstd = (torch.randn(co) * 0.3).to(DEV), (torch.randn(co) * 0.2).to(DEV), (torch.rand(co) + 0.5).to(DEV)
    out_ref = torch.empty(B * H * W, co, dtype=torch.bfloat16, device=DEV)
    lib.call("sd_conv_gemm", lib.SD_BF16, src, B, H, W, wp.data_ptr(), co, kpad, lib.SD_EPI_STORE, out_ref.data_ptr(),
             None, 0, None, None, s)
    rows_r = lib.call("sd_chan_reduce_rows", B * H * W, co)
    part_r = torch.empty(rows_r, co, 2, device=DEV)
    lib.call("sd_bn_bwd_reduce", lib.SD_BF16, out_ref.data_ptr(), y.data_ptr(), sc.data_ptr(), sh.data_ptr(),
             mean.data_ptr(), invstd.data_ptr(), B * H * W, co, part_r.data_ptr(), s)
    out = torch.empty_like(out_ref)
    rows = lib.call("sd_conv_gemm_bnsum_rows", src, B, H, W, co)
    part = torch.full((rows, co, 2), float("nan"), device=DEV)
    lib.call("sd_conv_gemm_bnsum", lib.SD_BF16, src, B, H, W, wp.data_ptr(), co, kpad, out.data_ptr(), y.data_ptr(),
             sc.data_ptr(), sh.data_ptr(), mean.data_ptr(), invstd.data_ptr(), part.data_ptr(), s)
    assert torch.equal(out, out_ref)
    got, ref = part.double().sum(0).cpu(), part_r.double().sum(0).cpu()
    scale = 1e-4 * (B * H * W) ** 0.5 * (1 + float(ref.abs().max()))
    assert torch.allclose(got, ref, rtol=1e-4, atol=scale)


@pytest.mark.parametrize("B,h,w_,ci,co", [(2, 12, 20, 64, 32), (1, 15, 20, 128, 64), (3, 17, 23, 64, 32),
                                          (2, 30, 40, 128, 64), (4, 60, 80, 64, 32)])
def test_convT_dgrad_bnsum_matches_store_plus_reduce(B, h, w_, ci, co):
    """ConvTranspose2d dgrad through k_convt (sub-pixel gather, weights resident in LDS): sd_conv_gemm_bnsum stores
    exactly what sd_conv_gemm(STORE) stores, that matches F.conv_transpose2d's input gradient, and its partial rows sum
    to sd_bn_bwd_reduce's BatchNorm-backward sums over (dx, y) (the BatchNorm of the conv feeding the ConvTranspose)."""
    lib = L()
    torch.manual_seed(9)
    s = lib.stream_handle()
    wt = (torch.randn(ci, co, 2, 2) / 8).to(torch.bfloat16).float().requires_grad_(True)
    x = torch.randn(B, ci, h, w_).requires_grad_(True)
    dout = torch.randn(B, co, 2 * h, 2 * w_).to(torch.bfloat16).float()
    F.conv_transpose2d(x, wt, None, stride=2).backward(dout)
    kd = ((4 * co + 63) // 64) * 64
    wpd = torch.empty(ci * kd, dtype=torch.bfloat16, device=DEV)
    lib.call("sd_pack_convT_w", lib.SD_BF16, wt.detach().contiguous().to(DEV).data_ptr(), ci, co, 1, kd, wpd.data_ptr(), s)
    dsrc = lib.make_src(_nhwc(dout, "bf16"), co, 2 * h, 2 * w_, taps=4)
    assert lib.kernel_name("sd_conv_gemm_kernel_name", lib.SD_BF16, dsrc, B, h, w_, ci,
                           lib.SD_EPI_STORE).startswith("k_convt<2, ")
    assert lib.call("sd_conv_gemm_bnsum_ok", lib.SD_BF16, dsrc, ci) == 1
    P = B * h * w_
    out_ref = torch.empty(P, ci, dtype=torch.bfloat16, device=DEV)
    lib.call("sd_conv_gemm", lib.SD_BF16, dsrc, B, h, w_, wpd.data_ptr(), ci, kd, lib.SD_EPI_STORE, out_ref.data_ptr(),
             None, 0, None, None, s)
    assert float((_from_nhwc(out_ref, B, h, w_, ci) - x.grad).abs().max()) <= _tol(x.grad, "bf16")
    y = (torch.randn(P, ci) * 2 + 0.3).to(DEV, torch.bfloat16)
    sc = ((torch.rand(ci) + 0.5) * torch.where(torch.rand(ci) < 0.2, -1.0, 1.0)).to(DEV)
    sh, mean, invstd = (torch.randn(ci) * 0.3).to(DEV), (torch.randn(ci) * 0.2).to(DEV), (torch.rand(ci) + 0.5).to(DEV)
    rows_r = lib.call("sd_chan_reduce_rows", P, ci)
    part_r = torch.empty(rows_r, ci, 2, device=DEV)
    lib.call("sd_bn_bwd_reduce", lib.SD_BF16, out_ref.data_ptr(), y.data_ptr(), sc.data_ptr(), sh.data_ptr(),
             mean.data_ptr(), invstd.data_ptr(), P, ci, part_r.data_ptr(), s)
    out = torch.empty_like(out_ref)
    rows = lib.call("sd_conv_gemm_bnsum_rows", dsrc, B, h, w_, ci)
    part = torch.full((rows, ci, 2), float("nan"), device=DEV)
    lib.call("sd_conv_gemm_bnsum", lib.SD_BF16, dsrc, B, h, w_, wpd.data_ptr(), ci, kd, out.data_ptr(), y.data_ptr(),
             sc.data_ptr(), sh.data_ptr(), mean.data_ptr(), invstd.data_ptr(), part.data_ptr(), s)
    assert lib.kernel_name("sd_conv_gemm_bnsum_kernel_name", dsrc, h, w_, ci).startswith("k_convt<3, ")
    assert torch.equal(out, out_ref)
    got, ref = part.double().sum(0).cpu(), part_r.double().sum(0).cpu()
    scale = 1e-4 * P ** 0.5 * (1 + float(ref.abs().max()))
    assert torch.allclose(got, ref, rtol=1e-4, atol=scale)


@pytest.mark.parametrize("B,H,W,c0,c1,co", [(2, 24, 64, 32, 32, 32), (1, 20, 30, 32, 32, 64), (2, 16, 40, 32, 96, 32)])
@pytest.mark.parametrize("fused", [False, True])
def test_conv3x3_wgrad_dual_source_spanning_block(B, H, W, c0, c1, co, fused):
    """Weight gradient over cat([up, skip]) (model.py:89-95) where a 64-channel x block spans both sources (dec1.0:
    32 + 32): each loader thread takes its 8 channels from its own source; plain and BatchNorm-backward-fused forms."""
    lib = L()
    torch.manual_seed(11)
    ys = [torch.randn(B, c, H, W).to(torch.bfloat16).float() for c in (c0, c1)]
    bns = [((torch.rand(c) + 0.5) * torch.where(torch.rand(c) < 0.2, -1.0, 1.0), torch.randn(c) * 0.3) for c in (c0, c1)]
    x = torch.cat([torch.relu(y * s.view(1, -1, 1, 1) + h.view(1, -1, 1, 1)).to(torch.bfloat16).float()
                   for y, (s, h) in zip(ys, bns)], 1)
    ci = c0 + c1
    dy = torch.randn(B, co, H, W).to(torch.bfloat16).float()
    b = lib.make_src(_nhwc(ys[0], "bf16"), c0, H, W, taps=9, bn0=tuple(t.to(DEV) for t in bns[0]),
                     src1=_nhwc(ys[1], "bf16"), c1=c1, bn1=tuple(t.to(DEV) for t in bns[1]))
    sp = lib.call("sd_wgrad_splits", lib.SD_BF16, B, H, W, co, 9 * ci)
    slab = torch.empty(sp * co * 9 * ci, device=DEV)
    dw = torch.empty(co, ci, 3, 3, device=DEV)
    s = lib.stream_handle()
    if fused:  # dy from (da, y) with coef = (scale, 0, 0) and y > 0 everywhere: dy = scale * da
        yo = (torch.rand(B, co, H, W) + 0.5).to(torch.bfloat16).float()
        sc = torch.rand(co) + 0.5
        dev = [t.to(DEV).contiguous() for t in (sc, torch.zeros(co), torch.zeros(co), torch.ones(co),
                                                torch.stack([sc, torch.zeros(co), torch.zeros(co)], 1))]
        dy = (sc.view(1, -1, 1, 1) * dy).to(torch.bfloat16).float()
        dyd = torch.full((B * H * W, co), float("nan"), dtype=torch.bfloat16, device=DEV)
        a = lib.make_src(dyd, co, H, W, taps=1)
        # 32-channel x blocks unless the source boundary is 64-aligned (SD_WS_CIB64=1: straddling SPAN blocks)
        assert lib.call("sd_wgrad_bnbwd_ok", lib.SD_BF16, a, b, co, 9 * ci) in (ci // 64, ci // 32)
        dad, yod = _nhwc(dy / sc.view(1, -1, 1, 1), "bf16"), _nhwc(yo, "bf16")  # held: no buffer reuse mid-call
        lib.call("sd_wgrad_gemm_bnbwd", lib.SD_BF16, a, b, B, H, W, co, 9 * ci, dad.data_ptr(), yod.data_ptr(),
                 *[t.data_ptr() for t in dev], slab.data_ptr(), sp, s)
    else:
        a = lib.make_src(_nhwc(dy, "bf16"), co, H, W, taps=1)
        lib.call("sd_wgrad_gemm", lib.SD_BF16, a, b, B, H, W, co, 9 * ci, slab.data_ptr(), sp, s)
    lib.call("sd_wgrad_reduce", slab.data_ptr(), sp, co, 9 * ci, lib.SD_W_CONV3, ci, dw.data_ptr(), s)
    w = torch.zeros(co, ci, 3, 3, requires_grad=True)
    F.conv2d(x, w, padding=1).backward(dy)
    ref = w.grad
    assert float((dw.cpu() - ref).abs().max()) <= 2e-2 * (1 + float(ref.abs().max()))
    if fused:
        assert not torch.isnan(_from_nhwc(dyd, B, H, W, co)).any()


# ---------------------------------------------------------------------------------------------- hi/lo split weights
def _pack_split(w, ci_pad):
    """SD_PACK_CONV3_FWD_SPLIT through sd_pack_weights: [co][kpad], k = tap*2*ci_pad + {hi ci | ci_pad + lo ci}."""
    lib = L()
    co, ci = w.shape[:2]
    kpad = ((18 * ci_pad + 63) // 64) * 64
    out = torch.empty(co * kpad, dtype=torch.bfloat16, device=DEV)
    wd = w.contiguous().to(DEV)
    job = (lib.SdPackJob * 1)(lib.SdPackJob(wd.data_ptr(), lib.SD_PACK_CONV3_FWD_SPLIT, co, ci, ci_pad, kpad, 0))
    lib.call("sd_pack_weights", lib.SD_BF16, job, 1, out.data_ptr(), lib.stream_handle())
    torch.cuda.synchronize()
    return out, kpad, wd


@pytest.mark.parametrize("H,W,c0,c1,co,wsplit,affine", [
    (30, 40, 256, 0, 256, True, True),     # bottleneck-side 30x40 layers: 16 hi/lo chunks over 4 N-blocks
    (15, 20, 256, 256, 512, True, True),   # decoder conv0 at 15x20: a concatenation, split across the two sources
    (60, 80, 128, 0, 128, False, False),   # plain bf16 weights, no affine, 32-channel N-blocks
    (15, 20, 512, 0, 512, False, True),
])
def test_conv3x3_ex_split_k_matches_unsplit(H, W, c0, c1, co, wsplit, affine):
    """sd_conv3x3_ex_ws at batch 1: groups of blocks over slices of the chunks (and hi/lo passes), partials added by a
    second launch; the same products as sd_conv3x3_ex up to fp32 summation order (within one bf16 rounding)."""
    lib = L()
    torch.manual_seed(11)
    ci = c0 + c1
    u = _nhwc(torch.randn(1, c0, H, W), "bf16")
    sk = _nhwc(torch.randn(1, c1, H, W), "bf16") if c1 else None
    sc, sh = (torch.rand(ci) + 0.5).to(DEV), (torch.randn(ci) * 0.2).to(DEV)
    w = torch.randn(co, ci, 3, 3) / (3 * ci ** 0.5)
    if wsplit:
        wp, kpad, _ = _pack_split(w, ci)
    else:
        wp, kpad = _pack3(w, ci, False, "bf16")
    src = lib.make_src(u, c0, H, W, taps=9, bn0=(sc[:c0].contiguous(), sh[:c0].contiguous()), src1=sk, c1=c1,
                       bn1=(sc[c0:].contiguous(), sh[c0:].contiguous()) if c1 else None)
    flags = lib.SD_CONV_WSPLIT if wsplit else 0
    osc, osh = (torch.rand(co) + 0.5).to(DEV), torch.randn(co).to(DEV)
    aff = (osc, osh) if affine else (None, None)
    nbytes = lib.call("sd_conv3x3_ex_ws_bytes", src, 1, H, W, co, lib.SD_EPI_STORE, flags)
    assert nbytes > 0, "the batch-1 deep shapes take the split-K path"
    ws = torch.empty(nbytes // 4, device=DEV)
    outs = []
    for wsp in (None, ws):
        out = torch.full((H * W, co), float("nan"), dtype=torch.bfloat16, device=DEV)
        lib.call("sd_conv3x3_ex_ws", src, 1, H, W, wp.data_ptr(), co, kpad, lib.SD_EPI_STORE, flags, lib.ptr(aff[0]),
                 lib.ptr(aff[1]), out.data_ptr(), None, lib.ptr(wsp), 0 if wsp is None else 4 * ws.numel(),
                 lib.stream_handle())
        outs.append(out.float())
    torch.cuda.synchronize()
    ref, got = outs
    assert torch.isfinite(got).all() and torch.isfinite(ref).all()
    assert float(((got - ref).abs() - 2.0 ** -7 * ref.abs()).max()) <= 1e-6 * float(ref.abs().max())
    assert float((got - ref).abs().mean()) <= 1e-3 * float(ref.abs().mean())


def test_pack_conv3_split_is_hi_plus_lo():
    torch.manual_seed(7)
    w = torch.randn(32, 24, 3, 3) / 7
    out, kpad, _ = _pack_split(w, 32)  # kpad = 576 = 18 * 32 exactly
    out40, kpad40, _ = _pack_split(torch.randn(16, 40, 3, 3), 40)  # kpad 768 > 720: zero K padding
    assert float(out40.float().cpu().reshape(16, kpad40)[:, 720:].abs().max()) == 0.0
    p = out.float().cpu().reshape(32, kpad)[:, :9 * 64].reshape(32, 9, 2, 32)
    hi, lo = p[:, :, 0, :24], p[:, :, 1, :24]
    ref = w.permute(0, 2, 3, 1).reshape(32, 9, 24)
    assert torch.equal(hi, ref.to(torch.bfloat16).float())  # hi = RNE(w)
    assert float(((hi + lo) - ref).abs().max()) <= 2.0 ** -16 * float(ref.abs().max())
    assert float(p[:, :, :, 24:].abs().max()) == 0.0  # channel padding stays zero
    tail = out.float().cpu().reshape(32, kpad)[:, 9 * 64:]
    assert tail.numel() == 0 or float(tail.abs().max()) == 0.0  # K padding past the 9 taps stays zero


@pytest.mark.parametrize("B,H,W,c0,c1,co,bn,epi", [
    (2, 32, 64, 8, 0, 32, False, "stats"),   # enc1.0: the 8-channel input, CK = 8 chunks
    (2, 30, 50, 8, 0, 32, False, "affine"),  # ragged tiles, BN affine epilogue (CK = 8, 32x32 MFMA epilogue)
    (1, 32, 64, 32, 0, 32, True, "store"),   # enc1.1 / dec1.1: 32 -> 32 with BN+ReLU, 16x32 tiles
    (1, 32, 64, 32, 32, 32, True, "stats"),  # dec1.0: cat([up, skip]) (two sources, four chunks)
    (1, 32, 64, 32, 32, 32, True, "affine"),
    (2, 15, 20, 64, 0, 64, True, "store"),   # N % 64 shapes: whole-image tiles, NT = 2, RT = 2 / 3
    (2, 15, 20, 64, 64, 128, True, "affine"),
    (1, 30, 40, 128, 0, 128, True, "affine"),
    (1, 32, 64, 64, 64, 64, True, "stats"),  # weights-in-registers instances (8x32 / 16x16 tiles) with hi/lo passes
    (1, 32, 48, 64, 0, 128, True, "store"),
])
def test_conv3x3_ex_split_weights_and_affine_epilogue(B, H, W, c0, c1, co, bn, epi):
    """sd_conv3x3_ex(SD_CONV_WSPLIT): the product of the bf16 operand with the fp32 weights (hi + lo), to within one bf16
    rounding of the output, where the plain bf16 conv carries the weights' bf16 rounding (~2^-9); BN statistics of the
    stored values as sd_conv_gemm. "affine": the eval BatchNorm in the epilogue, out = bf16(acc*scale + shift)."""
    lib = L()
    torch.manual_seed(3)
    ci = c0 + c1
    u = torch.randn(B, c0, H, W).to(torch.bfloat16).float() + (0.5 if not bn else 0.0)
    s = torch.randn(B, c1, H, W).to(torch.bfloat16).float() if c1 else None
    sc, sh = torch.rand(ci) + 0.5, torch.randn(ci) * 0.2
    w = torch.randn(co, ci, 3, 3) / (3 * ci ** 0.5)
    if c1:  # dec1.0 form: the up part raw, the skip part BN+ReLU
        xs = torch.relu(s * sc[None, c0:, None, None] + sh[None, c0:, None, None]).to(torch.bfloat16).float()
        x = torch.cat([u, xs], 1)
    elif bn:
        x = torch.relu(u * sc[None, :, None, None] + sh[None, :, None, None]).to(torch.bfloat16).float()
    else:
        x = u
    ref = F.conv2d(x.double(), w.double(), padding=1)
    wp, kpad, _ = _pack_split(w, ci)
    ud = _nhwc(u, "bf16")
    if c1:
        src = lib.make_src(ud, c0, H, W, taps=9, src1=_nhwc(s, "bf16"), c1=c1,
                           bn1=(sc[c0:].contiguous().to(DEV), sh[c0:].contiguous().to(DEV)))
    else:
        src = lib.make_src(ud, c0, H, W, taps=9, bn0=(sc.to(DEV), sh.to(DEV)) if bn else None)
    assert lib.call("sd_conv3x3_ex_ok", src, co) == 1
    out = torch.empty(B * H * W, co, dtype=torch.bfloat16, device=DEV)
    e = lib.SD_EPI_STATS if epi == "stats" else lib.SD_EPI_STORE
    rows = lib.call("sd_conv_gemm_stat_rows", lib.SD_BF16, B, H, W, co)
    stats = torch.zeros(rows, co, 2, device=DEV)
    osc, osh = torch.rand(co) + 0.5, torch.randn(co)
    osc[::5] *= -1
    aff = (osc.to(DEV), osh.to(DEV)) if epi == "affine" else (None, None)
    lib.call("sd_conv3x3_ex", src, B, H, W, wp.data_ptr(), co, kpad, e, lib.SD_CONV_WSPLIT, lib.ptr(aff[0]),
             lib.ptr(aff[1]), out.data_ptr(), stats.data_ptr() if e == lib.SD_EPI_STATS else None, lib.stream_handle())
    got = _from_nhwc(out, B, H, W, co).double()
    if epi == "affine":  # the stored value is the BN-applied z; compare z, and take y back out for the checks below
        ref = ref * osc.double()[None, :, None, None] + osh.double()[None, :, None, None]
        err = float((got - ref.float().to(torch.bfloat16).double()).abs().max())
        assert err <= 2.0 ** -7 * float(ref.abs().max()), err  # at most one bf16 ulp apart after rounding
        return
    # the output is stored bf16: compare the pre-rounding error through the rounding of the reference
    err = float((got - ref.float().to(torch.bfloat16).double()).abs().max())
    assert err <= 2.0 ** -7 * float(ref.abs().max()), err  # at most one bf16 ulp apart after rounding
    # the plain bf16 conv (weights rounded) vs the split one: mean error to the fp64 reference, before output rounding
    wq = w.to(torch.bfloat16).double()
    e_plain = float((F.conv2d(x.double(), wq, padding=1) - ref).abs().mean())
    e_split = float((got - ref).abs().mean())
    print(f"mean |err|: split (incl. bf16 output rounding) {e_split:.3g}, bf16 weights (before rounding) {e_plain:.3g}")
    if e == lib.SD_EPI_STATS:
        st = stats.double().sum(0).cpu()
        assert torch.allclose(st[:, 0], got.sum((0, 2, 3)), rtol=1e-4, atol=1e-2)
    # name of the launched instance (rocprofv3): the chunks run twice, so one-chunk layers keep their weights in LDS
    name = L().kernel_name("sd_conv3x3_ex_kernel_name", src, H, W, co, e, lib.SD_CONV_WSPLIT, 0)
    assert name.startswith("k_halo_conv<")


def test_convT_split_pack_doubled_k_matches_fp32_weights():
    """up1's hi/lo forward: the source twice along K (two sources of the 1x1 GEMM) against SD_PACK_CONVT_FWD_SPLIT
    rows [hi | lo]: ConvTranspose2d with the fp32 weights (bias, pixel shuffle) to one bf16 ulp of the output."""
    lib = L()
    torch.manual_seed(5)
    B, H, W, ci, co = 2, 12, 20, 64, 32
    y = torch.randn(B, ci, H, W).to(torch.bfloat16).float()
    sc, sh = torch.rand(ci) + 0.5, torch.randn(ci) * 0.2
    w = torch.randn(ci, co, 2, 2) / 8
    bias = torch.randn(co) * 0.1
    x = torch.relu(y * sc[None, :, None, None] + sh[None, :, None, None]).to(torch.bfloat16).float()
    ref = F.conv_transpose2d(x.double(), w.double(), bias.double(), stride=2)
    kpad = ((2 * ci + 63) // 64) * 64
    wp = torch.empty(4 * co * kpad, dtype=torch.bfloat16, device=DEV)
    wd = w.contiguous().to(DEV)
    job = (lib.SdPackJob * 1)(lib.SdPackJob(wd.data_ptr(), lib.SD_PACK_CONVT_FWD_SPLIT, co, ci, ci, kpad, 0))
    lib.call("sd_pack_weights", lib.SD_BF16, job, 1, wp.data_ptr(), lib.stream_handle())
    yd = _nhwc(y, "bf16")
    bn = (sc.to(DEV), sh.to(DEV))
    src = lib.make_src(yd, ci, H, W, taps=1, bn0=bn, src1=yd, c1=ci, bn1=bn)
    out = torch.empty(B * 4 * H * W, co, dtype=torch.bfloat16, device=DEV)
    bd = bias.to(DEV)
    lib.call("sd_conv_gemm", lib.SD_BF16, src, B, H, W, wp.data_ptr(), 4 * co, kpad, lib.SD_EPI_PIXSHUF,
             out.data_ptr(), None, 0, bd.data_ptr(), None, lib.stream_handle())
    got = _from_nhwc(out, B, 2 * H, 2 * W, co).double()
    err = float((got - ref.float().to(torch.bfloat16).double()).abs().max())
    assert err <= 2.0 ** -7 * float(ref.abs().max()), err


@pytest.mark.parametrize("prec", ["fp32", "bf16"])
@pytest.mark.parametrize("B,C,H,W", [(3, 6, 24, 32), (2, 7, 10, 14), (1, 6, 5, 7), (2, 8, 16, 20)])
def test_pack_input_nchw_to_padded_nhwc(prec, B, C, H, W):
    """sd_pack_input / sd_pack_input_amax: NCHW fp32 -> NHWC with the channels zero-padded to 8, in the path's dtype
    (the four-pixel form where H*W % 4 == 0, the per-pixel form otherwise); the amax form also takes max |x| into its
    slot and clears another."""
    lib = L()
    torch.manual_seed(17)
    x = (torch.randn(B, C, H, W) * 3).to(DEV)
    ref = torch.zeros(B, H, W, 8)
    ref[..., :C] = x.cpu().permute(0, 2, 3, 1)
    ref = ref.to(_adt(prec)).reshape(B * H * W, 8)
    s = lib.stream_handle()
    out = torch.full((B * H * W, 8), float("nan"), dtype=_adt(prec), device=DEV)
    lib.call("sd_pack_input", _sd(prec), x.data_ptr(), B, C, H, W, 8, out.data_ptr(), s)
    amax = torch.tensor([0, 12345], dtype=torch.int32, device=DEV)
    out2 = torch.full_like(out, float("nan"))
    lib.call("sd_pack_input_amax", _sd(prec), x.data_ptr(), B, C, H, W, 8, out2.data_ptr(), amax.data_ptr(), 0, 1, s)
    torch.cuda.synchronize()
    assert torch.equal(out.cpu(), ref) and torch.equal(out2.cpu(), ref)
    got_max = amax[:1].cpu().view(torch.float32).item()
    assert got_max == float(x.abs().max()) and int(amax[1]) == 0


@pytest.mark.parametrize("B,H,W,c0,c1,co", [
    (2, 24, 64, 64, 0, 64),      # 8x32 tiles, two chunks (weights resident: WCONST)
    (1, 36, 96, 72, 0, 128),     # ragged last tile row, a partial chunk, two N-blocks
    (2, 40, 48, 32, 32, 64),     # two raw sources (a ConvTranspose output + another raw tensor)
    (1, 30, 40, 160, 0, 256),    # 5 chunks: per-chunk weight DMA, four N-blocks
    (1, 15, 20, 96, 64, 512),    # whole-image tile (RT 3), 5 chunks over two sources
    (2, 32, 64, 32, 0, 32),      # N = 32, 16x32 tiles (RT 4, vertical reuse)
    (1, 48, 64, 96, 0, 32),      # N = 32, three chunks
])
def test_conv3x3_raw_source_dma_loaders_bit_identical(monkeypatch, B, H, W, c0, c1, co):
    """k_halo_conv RAW (every source raw: halo and weights by LDS-DMA, no register staging) stores bit for bit what the
    register-staged loaders store (SD_HALO_RAW=0): the same LDS images, the same MFMA order. STORE, STATS and the SPLIT
    dgrad epilogue; and the result matches F.conv2d."""
    lib = L()
    torch.manual_seed(23)
    ci = c0 + c1
    u = torch.randn(B, c0, H, W).to(torch.bfloat16).float()
    sk = torch.randn(B, c1, H, W).to(torch.bfloat16).float() if c1 else None
    w = (torch.randn(co, ci, 3, 3) / (3 * ci ** 0.5)).to(torch.bfloat16).float()
    x = torch.cat([u] + ([sk] if c1 else []), 1)
    ref = F.conv2d(x, w, padding=1)
    wp, kpad = _pack3(w, ci, False, "bf16")
    src = lib.make_src(_nhwc(u, "bf16"), c0, H, W, taps=9, src1=_nhwc(sk, "bf16") if c1 else None, c1=c1)
    res = {}
    for raw in ("1", "0"):
        monkeypatch.setenv("SD_HALO_RAW", raw)
        name = lib.kernel_name("sd_conv_gemm_kernel_name", lib.SD_BF16, src, B, H, W, co, lib.SD_EPI_STORE)
        assert name.endswith("true>" if raw == "1" else "false>"), name
        rows = lib.call("sd_conv_gemm_stat_rows", lib.SD_BF16, B, H, W, co)
        outs = {}
        for epi in (lib.SD_EPI_STORE, lib.SD_EPI_STATS):
            out = torch.full((B * H * W, co), float("nan"), dtype=torch.bfloat16, device=DEV)
            st = torch.full((rows, co, 2), float("nan"), device=DEV)
            lib.call("sd_conv_gemm", lib.SD_BF16, src, B, H, W, wp.data_ptr(), co, kpad, epi, out.data_ptr(), None, 0,
                     None, st.data_ptr() if epi == lib.SD_EPI_STATS else None, lib.stream_handle())
            outs[epi] = (out, st)
        ns = co // 2
        d0 = torch.full((B * H * W, ns), float("nan"), dtype=torch.bfloat16, device=DEV)
        d1 = torch.full((B * H * W, co - ns), float("nan"), dtype=torch.bfloat16, device=DEV)
        lib.call("sd_conv_gemm", lib.SD_BF16, src, B, H, W, wp.data_ptr(), co, kpad, lib.SD_EPI_SPLIT, d0.data_ptr(),
                 d1.data_ptr(), ns, None, None, lib.stream_handle())
        torch.cuda.synchronize()
        res[raw] = (outs, d0, d1)
    (o1, a0, a1), (o0, b0, b1) = res["1"], res["0"]
    for epi in (lib.SD_EPI_STORE, lib.SD_EPI_STATS):
        assert torch.equal(o1[epi][0], o0[epi][0]), epi
    assert torch.equal(o1[lib.SD_EPI_STATS][1], o0[lib.SD_EPI_STATS][1])
    assert torch.equal(a0, b0) and torch.equal(a1, b1)
    got = _from_nhwc(o1[lib.SD_EPI_STORE][0], B, H, W, co)
    assert float((got - ref).abs().max()) <= _tol(ref, "bf16")


@pytest.mark.parametrize("B,H,W", [(2, 16, 64), (1, 8, 32), (3, 24, 48)])
def test_conv3x3_bwd_fused_matches_reference(B, H, W):
    """sd_conv3x3_bwd_fused (enc1.1 / dec1.1 backward in one pass) against fp64 PyTorch on the same bf16 operands:
    dy = BatchNorm-backward(da, y) (the kernel stages it as bf16), dW = conv2d_weight(x, dy), x = relu(bn_prev(y_prev))
    (bf16), dx = conv2d_input(dy, W) (stored bf16), and the previous layer's BatchNorm-backward sums over (dx, y_prev).
    Bounds: dW 1e-3 of max (fp32 sums of bf16 products), dx one bf16 rounding (2^-7 relative + 1e-3 of max), sums 1e-2
    of their scale (they are taken over the bf16-rounded dx)."""
    lib = L()
    torch.manual_seed(31)
    C = 32
    bf = lambda t: t.to(torch.bfloat16).double()  # noqa: E731
    da, y, yp = bf(torch.randn(B, C, H, W)), bf(torch.randn(B, C, H, W)), bf(torch.randn(B, C, H, W))
    sc, sh = torch.rand(C).double() + 0.5, torch.randn(C).double() * 0.3
    sc[::5] *= -1
    mu, is_ = torch.randn(C).double() * 0.2, torch.rand(C).double() + 0.5
    coef = torch.randn(C, 3).double() * 0.1
    psc, psh = torch.rand(C).double() + 0.5, torch.randn(C).double() * 0.3
    pmu, pis = torch.randn(C).double() * 0.2, torch.rand(C).double() + 0.5
    w = (torch.randn(C, C, 3, 3) / 17.0).to(torch.bfloat16).double()
    v = lambda t: t[None, :, None, None]  # noqa: E731
    # reference
    z = y * v(sc) + v(sh)
    dz = torch.where(z > 0, da, torch.zeros_like(da))
    dy = v(sc) * (dz - v(coef[:, 1]) - v(coef[:, 2]) * (y - v(mu)) * v(is_))
    dy = bf(dy.float())
    x = bf(torch.relu(yp * v(psc) + v(psh)).float())
    dw_ref = torch.nn.grad.conv2d_weight(x, w.shape, dy, padding=1)
    dx_ref = torch.nn.grad.conv2d_input(x.shape, w, dy, padding=1)
    # kernel
    f32 = lambda t: t.float().contiguous().to(DEV)  # noqa: E731
    wp, kpad = _pack3(w.float(), C, True, "bf16")
    sp = lib.call("sd_conv3x3_bwd_fused_splits", B, H, W)
    assert lib.call("sd_conv3x3_bwd_fused_ok", C, C, H, W) == 1
    slab = torch.full((sp * C * 9 * C,), float("nan"), device=DEV)
    part = torch.full((sp, C, 2), float("nan"), device=DEV)
    dx = torch.full((B * H * W, C), float("nan"), dtype=torch.bfloat16, device=DEV)
    tens = [_nhwc(t.float(), "bf16") for t in (da, y, yp)]
    prm = [f32(t) for t in (sc, sh, mu, is_, coef, psc, psh, pmu, pis)]
    lib.call("sd_conv3x3_bwd_fused", tens[0].data_ptr(), tens[1].data_ptr(), *[t.data_ptr() for t in prm[:5]],
             tens[2].data_ptr(), *[t.data_ptr() for t in prm[5:]], wp.data_ptr(), kpad, B, H, W, dx.data_ptr(),
             slab.data_ptr(), part.data_ptr(), lib.stream_handle())
    dw = torch.empty(C, C, 3, 3, device=DEV)
    lib.call("sd_wgrad_reduce", slab.data_ptr(), sp, C, 9 * C, lib.SD_W_CONV3, C, dw.data_ptr(), lib.stream_handle())
    torch.cuda.synchronize()
    dw = dw.double().cpu()
    assert float((dw - dw_ref).abs().max()) <= 1e-3 * float(dw_ref.abs().max())
    got = _from_nhwc(dx, B, H, W, C).double()
    assert float(((got - dx_ref).abs() - 2.0 ** -7 * dx_ref.abs()).max()) <= 1e-3 * float(dx_ref.abs().max())
    # the previous layer's BatchNorm-backward sums over the stored (bf16) dx
    dzp = torch.where(yp * v(psc) + v(psh) > 0, got, torch.zeros_like(got))
    xh = (yp - v(pmu)) * v(pis)
    s_ref = torch.stack([dzp.sum((0, 2, 3)), (dzp * xh).sum((0, 2, 3))], 1)
    s_got = part.double().sum(0).cpu()
    assert float((s_got - s_ref).abs().max()) <= 1e-2 * (1 + float(s_ref.abs().max()))


@pytest.mark.parametrize("B,H,W", [(2, 16, 64), (1, 8, 16), (3, 24, 48)])
def test_conv3x3_bwd_fused_dec_matches_reference(B, H, W):
    """sd_conv3x3_bwd_fused_dec (dec1.0's backward in one pass) against fp64 PyTorch on the same bf16 operands:
    dy = BatchNorm-backward(da, y) (staged as bf16), x = cat(u, relu(bn_skip(y_skip))) (bf16),
    dW = conv2d_weight(x, dy), dx = conv2d_input(dy, W) stored bf16 as d(u) | d(skip), and the column sums of the
    stored d(u) (the ConvTranspose2d bias gradient). Bounds as test_conv3x3_bwd_fused_matches_reference."""
    lib = L()
    torch.manual_seed(37)
    C = 32
    bf = lambda t: t.to(torch.bfloat16).double()  # noqa: E731
    da, y = bf(torch.randn(B, C, H, W)), bf(torch.randn(B, C, H, W))
    u, ys = bf(torch.randn(B, C, H, W)), bf(torch.randn(B, C, H, W))
    sc, sh = torch.rand(C).double() + 0.5, torch.randn(C).double() * 0.3
    sc[::7] *= -1
    mu, is_ = torch.randn(C).double() * 0.2, torch.rand(C).double() + 0.5
    coef = torch.randn(C, 3).double() * 0.1
    ssc, ssh = torch.rand(C).double() + 0.5, torch.randn(C).double() * 0.3
    w = (torch.randn(C, 2 * C, 3, 3) / 24.0).to(torch.bfloat16).double()
    v = lambda t: t[None, :, None, None]  # noqa: E731
    z = y * v(sc) + v(sh)
    dz = torch.where(z > 0, da, torch.zeros_like(da))
    dy = bf((v(sc) * (dz - v(coef[:, 1]) - v(coef[:, 2]) * (y - v(mu)) * v(is_))).float())
    x = torch.cat([u, bf(torch.relu(ys * v(ssc) + v(ssh)).float())], 1)
    dw_ref = torch.nn.grad.conv2d_weight(x, w.shape, dy, padding=1)
    dx_ref = torch.nn.grad.conv2d_input(x.shape, w, dy, padding=1)
    f32 = lambda t: t.float().contiguous().to(DEV)  # noqa: E731
    wp, kpad = _pack3(w.float(), 2 * C, True, "bf16")
    sp = lib.call("sd_conv3x3_bwd_fused_splits", B, H, W)
    assert lib.call("sd_conv3x3_bwd_fused_dec_ok", C, C, C, H, W) == 1
    slab = torch.full((sp * C * 9 * 2 * C,), float("nan"), device=DEV)
    part = torch.full((sp, C, 2), float("nan"), device=DEV)
    du = torch.full((B * H * W, C), float("nan"), dtype=torch.bfloat16, device=DEV)
    dsk = torch.full((B * H * W, C), float("nan"), dtype=torch.bfloat16, device=DEV)
    tens = [_nhwc(t.float(), "bf16") for t in (da, y, u, ys)]
    prm = [f32(t) for t in (sc, sh, mu, is_, coef, ssc, ssh)]
    lib.call("sd_conv3x3_bwd_fused_dec", tens[0].data_ptr(), tens[1].data_ptr(), *[t.data_ptr() for t in prm[:5]],
             tens[2].data_ptr(), tens[3].data_ptr(), prm[5].data_ptr(), prm[6].data_ptr(), wp.data_ptr(), kpad, B, H,
             W, du.data_ptr(), dsk.data_ptr(), slab.data_ptr(), part.data_ptr(), lib.stream_handle())
    dw = torch.empty(C, 2 * C, 3, 3, device=DEV)
    lib.call("sd_wgrad_reduce", slab.data_ptr(), sp, C, 9 * 2 * C, lib.SD_W_CONV3, 2 * C, dw.data_ptr(),
             lib.stream_handle())
    bias = torch.empty(C, device=DEV)
    lib.call("sd_stat_rows_sum", part.data_ptr(), sp, C, C, bias.data_ptr(), lib.stream_handle())
    torch.cuda.synchronize()
    dw = dw.double().cpu()
    assert float((dw - dw_ref).abs().max()) <= 1e-3 * float(dw_ref.abs().max())
    got = torch.cat([_from_nhwc(du, B, H, W, C), _from_nhwc(dsk, B, H, W, C)], 1).double()
    assert float(((got - dx_ref).abs() - 2.0 ** -7 * dx_ref.abs()).max()) <= 1e-3 * float(dx_ref.abs().max())
    b_ref = got[:, :C].sum((0, 2, 3))
    assert float((bias.double().cpu() - b_ref).abs().max()) <= 1e-4 * (1 + float(b_ref.abs().max()))
