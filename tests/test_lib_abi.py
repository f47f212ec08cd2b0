"""C-ABI checks that need no GPU: the library loads, exports every symbol include/stereo_hip.h
declares, host-side argument validation rejects bad shapes before any launch."""

import ctypes
import re
from pathlib import Path

import pytest

from stereo_depth_estimation_amd import _lib as L

HEADER = Path(__file__).resolve().parents[1] / "include" / "stereo_hip.h"


def _declared():
    txt = HEADER.read_text()
    return sorted(set(re.findall(r"^(?:int|long long|const char\*)\s+(sd_\w+)\s*\(", txt, flags=re.M)))


def test_library_exports_every_declared_symbol():
    lib = L.load()
    declared = _declared()
    assert len(declared) >= 25
    for name in declared:
        assert hasattr(lib, name), name
    assert set(declared) == set(L.exported_symbols())
    assert lib.sd_version() >= 100


def test_sd_src_struct_layout_matches_header():
    # ptr[2], scale[2], shift[2] (6 pointers) + chans[2], xform[2], H, W, taps, pool (8 ints)
    assert ctypes.sizeof(L.SdSrc) == 6 * 8 + 8 * 4


def test_sd_pack_job_struct_layout_matches_header():
    # const float* w; int kind, co, ci, ci_pad, kpad; int64_t out_off
    assert ctypes.sizeof(L.SdPackJob) == 40
    assert L.SdPackJob.out_off.offset == 32


def test_pack_weights_validation_without_launch():
    bad = (L.SdPackJob * 1)(L.SdPackJob(16, L.SD_PACK_CONV3_FWD, 32, 32, 32, 100, 0))  # kpad not a multiple of 64
    with pytest.raises(L.StereoHipError, match="job 0"):
        L.call("sd_pack_weights", L.SD_BF16, bad, 1, 16, None)
    many = (L.SdPackJob * 65)()
    with pytest.raises(L.StereoHipError, match="max 64"):
        L.call("sd_pack_weights", L.SD_BF16, many, 65, 16, None)


def test_host_validation_rejects_bad_args_without_launch():
    src = L.make_src(None, 16, 8, 8)
    with pytest.raises(L.StereoHipError, match="null source 0"):
        L.call("sd_conv_gemm", L.SD_F32, src, 1, 8, 8, 1, 16, 192, L.SD_EPI_STORE, 1, None, 0, None, None, None)
    src = L.make_src(ctypes.c_void_p(16), 12, 8, 8)  # channels not a multiple of 8
    with pytest.raises(L.StereoHipError, match="multiple of 8"):
        L.call("sd_conv_gemm", L.SD_F32, src, 1, 8, 8, 1, 16, 192, L.SD_EPI_STORE, 1, None, 0, None, None, None)
    with pytest.raises(L.StereoHipError, match="dims must be even"):
        L.call("sd_pool_bwd_add", L.SD_F32, 1, 1, 1, None, 1, 1, 7, 8, 8, 1, None, None, None, None)
    with pytest.raises(L.StereoHipError, match="kpad"):
        L.call("sd_pack_conv3_w", L.SD_F32, 1, 32, 32, 32, 0, 100, 1, None)
    # row-sum jobs of the batched reduce (the ConvTranspose bias gradients): M = 1, C <= pitch, 8-B aligned rows
    for M, N, C, ptr in ((2, 64, 32, 16), (1, 16, 32, 16), (1, 64, 32, 20)):
        jobs = (L.SdWredJob * 1)(L.SdWredJob(ptr, 4, M, N, L.SD_W_ROWSUM, C, 16))
        with pytest.raises(L.StereoHipError, match="row-sum job 0"):
            L.call("sd_wgrad_reduce_batch", jobs, 1, None)


def test_planning_queries_are_host_only():
    assert L.call("sd_conv_gemm_stat_rows", L.SD_F32, 64, 240, 320, 32) == 64 * 240 * 320 // 128
    # bf16 3x3 convs: one stats row per persistent block (256 blocks split over the N-blocks)
    assert L.call("sd_conv_gemm_stat_rows", L.SD_BF16, 64, 240, 320, 32) == 256
    src = L.make_src(ctypes.c_void_p(16), 32, 240, 320, taps=9)
    assert L.kernel_name("sd_conv_gemm_kernel_name", L.SD_BF16, src, 64, 240, 320, 32, L.SD_EPI_STATS) == "k_halo_conv<1, 4, 32, true, true, 1, false, false, true>"  # 16x32 tiles, one chunk, raw source: all-DMA loaders
    assert L.kernel_name("sd_conv_gemm_kernel_name", L.SD_BF16, src, 64, 240, 320, 32, L.SD_EPI_STORE) == "k_halo_conv<1, 4, 32, false, true, 1, false, false, true>"  # 16x32
    # 3x3 convs with N % 64 == 0 take the halo kernel too; tile shape follows the image
    assert L.call("sd_conv_gemm_stat_rows", L.SD_BF16, 64, 60, 80, 128) == 128  # 2 N-blocks
    assert L.call("sd_conv_gemm_stat_rows", L.SD_BF16, 64, 15, 20, 512) == 32  # 8 N-blocks
    assert L.call("sd_conv_gemm_stat_rows", L.SD_BF16, 2, 15, 20, 512) == 2  # never more rows than tiles
    src15 = L.make_src(ctypes.c_void_p(16), 256, 15, 20, taps=9)
    assert L.kernel_name("sd_conv_gemm_kernel_name", L.SD_BF16, src15, 64, 15, 20, 512, L.SD_EPI_STATS) == "k_halo_conv<2, 3, 32, true, false, 1, false, false, true>"
    assert L.kernel_name("sd_conv_gemm_kernel_name", L.SD_BF16, src, 64, 240, 320, 96, L.SD_EPI_STORE).startswith("k_conv_fwd_bf16<")
    sp = L.call("sd_wgrad_splits", L.SD_BF16, 64, 240, 320, 32, 288)
    assert 1 <= sp <= 64 * 240 * 320 // 256
    assert L.call("sd_chan_reduce_rows", 1000, 32) >= 1
    # dgrads that also sum the BatchNorm backward of the layer they produce da for (not the 15x20 RT 3 tiles)
    assert L.call("sd_conv_gemm_bnsum_ok", L.SD_BF16, src, 32) == 1
    assert L.kernel_name("sd_conv_gemm_bnsum_kernel_name", src, 240, 320, 32) == "k_halo_conv<1, 4, 32, false, true, 1, true, false, false>"
    assert L.call("sd_conv_gemm_bnsum_rows", src, 64, 240, 320, 32) == 256
    assert L.call("sd_conv_gemm_bnsum_ok", L.SD_BF16, src15, 512) == 0
    # BatchNorm-backward apply fused into the warp-specialised weight gradients (every 3x3 wgrad but enc1.0's)
    dy = L.make_src(ctypes.c_void_p(16), 32, 240, 320, taps=1)
    assert L.call("sd_wgrad_bnbwd_ok", L.SD_BF16, dy, src, 32, 288) == 1
    assert L.kernel_name("sd_wgrad_bnbwd_kernel_name", dy, src, 32, 288) == "k_halo_wgrad_ws<32, 32, 22, 8, true, false>"
    x256 = L.make_src(ctypes.c_void_p(16), 256, 60, 80, taps=9)
    dy128 = L.make_src(ctypes.c_void_p(16), 128, 60, 80, taps=1)
    assert L.call("sd_wgrad_bnbwd_ok", L.SD_BF16, dy128, x256, 128, 2304) == 4  # four 64-channel x blocks
    x8 = L.make_src(ctypes.c_void_p(16), 8, 240, 320, taps=9)
    assert L.call("sd_wgrad_bnbwd_ok", L.SD_BF16, dy, x8, 32, 72) == 0  # enc1.0: only without a dy destination
    nody = L.make_src(None, 32, 240, 320, taps=1)
    assert L.call("sd_wgrad_bnbwd_ok", L.SD_BF16, nody, x8, 32, 72) == 1
    assert L.kernel_name("sd_wgrad_bnbwd_kernel_name", nody, x8, 32, 72) == "k_halo_wgrad<32, true, true>"  # the 8-channel x layout
    assert L.call("sd_wgrad_bnbwd_ok", L.SD_F32, dy, src, 32, 288) == 0
    # fp8 inference convs (live app, 960x720): one min/max row per persistent block
    assert L.call("sd_conv3x3_fp8_rows", 1, 720, 960, 32) == 256
    assert L.call("sd_conv3x3_fp8_rows", 1, 45, 60, 512) == 12  # 4x60 tiles, 8 N-blocks
    assert L.kernel_name("sd_conv3x3_fp8_kernel_name", 64) == "k_halo_conv_fp8<2>"
    assert L.call("sd_chan_minmax_rows", 691200, 32) == 256
    # fused full-resolution conv1 backward: 32 -> 32 channels on 8x16 tiles, one block per CU
    assert L.call("sd_conv3x3_bwd_fused_ok", 32, 32, 240, 320) == 1
    assert L.call("sd_conv3x3_bwd_fused_ok", 32, 32, 12, 96) == 0  # H % 8
    assert L.call("sd_conv3x3_bwd_fused_ok", 64, 32, 240, 320) == 0
    assert L.call("sd_conv3x3_bwd_fused_splits", 64, 240, 320) == 256
    assert L.call("sd_conv3x3_bwd_fused_splits", 1, 16, 32) == 8  # 2 tiles: a multiple of 8 blocks (the XCD map)
    assert L.call("sd_conv3x3_bwd_fused_dec_ok", 32, 32, 32, 240, 320) == 1  # dec1.0: cat(32 up, 32 skip) -> 32
    assert L.call("sd_conv3x3_bwd_fused_dec_ok", 32, 64, 32, 240, 320) == 0


def test_fused_bn_wgrad_host_validation():
    dy = L.make_src(ctypes.c_void_p(16), 32, 24, 32, taps=1)
    x8 = L.make_src(ctypes.c_void_p(16), 8, 24, 32, taps=9)
    with pytest.raises(L.StereoHipError, match="no fused kernel"):  # 8-channel x with a dy destination
        L.call("sd_wgrad_gemm_bnbwd", L.SD_BF16, dy, x8, 1, 24, 32, 32, 72, 1, 1, 1, 1, 1, 1, 1, 1, 1, None)
    x = L.make_src(ctypes.c_void_p(16), 32, 24, 32, taps=9)
    with pytest.raises(L.StereoHipError, match="bf16 only"):
        L.call("sd_wgrad_gemm_bnbwd", L.SD_F32, dy, x, 1, 24, 32, 32, 288, 1, 1, 1, 1, 1, 1, 1, 1, 1, None)
    with pytest.raises(L.StereoHipError, match="null pointer"):
        L.call("sd_wgrad_gemm_bnbwd", L.SD_BF16, dy, x, 1, 24, 32, 32, 288, None, 1, 1, 1, 1, 1, 1, 1, 1, None)


def test_fp8_host_validation():
    src = L.make_src(ctypes.c_void_p(16), 32, 8, 8, taps=9)  # identity transform: no quantisation affine
    with pytest.raises(L.StereoHipError, match="quantisation affine"):
        L.call("sd_conv3x3_fp8", src, 1, 8, 8, 1, 1, 1, 32, 320, 1, 1, None)
    with pytest.raises(L.StereoHipError, match="kpad"):
        L.call("sd_pack_conv3_w_fp8", 1, 32, 32, 32, 64, 1, 1, None)
    q = L.make_qsrc(None, 1, 8, 1, 1)
    with pytest.raises(L.StereoHipError, match="source 0"):
        L.call("sd_fp8_qparams", (L.SdQSrc * 1)(q), 1, 1, None)
    assert ctypes.sizeof(L.SdQSrc) == 56
