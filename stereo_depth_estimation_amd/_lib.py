"""ctypes binding of libstereo_hip.so (C ABI: include/stereo_hip.h).

The library is loaded after ``import torch`` so that it binds to the HIP runtime torch
already loaded (both carry SONAME libamdhip64.so.7): one runtime, one device context,
torch-allocated pointers valid in our kernels.  There is no fallback: if the library is
missing or fails to load, every entry point raises.
"""

from __future__ import annotations

import ctypes
import os
from pathlib import Path

import torch  # noqa: F401  (must precede the CDLL load, see module docstring)

# SD_HIP_LIB: an alternative build of the same C ABI (A/B timing of kernel variants); default in-tree
LIB_PATH = Path(os.environ.get("SD_HIP_LIB") or Path(__file__).resolve().parent / "libstereo_hip.so")

SD_F32, SD_BF16 = 0, 1
SD_IDENT, SD_BNRELU, SD_AFFINE = 0, 1, 2
SD_EPI_STORE, SD_EPI_STATS, SD_EPI_SPLIT, SD_EPI_PIXSHUF, SD_EPI_SPLIT_STATS = 0, 1, 2, 3, 4
SD_W_CONV3, SD_W_CONVT, SD_W_ROWSUM = 0, 1, 2
SD_HEADS_INFER, SD_HEADS_LOSS, SD_HEADS_GRADS = 0, 1, 2

_p = ctypes.c_void_p
_i = ctypes.c_int
_i64 = ctypes.c_int64
_f = ctypes.c_float
_d = ctypes.c_double


class SdSrc(ctypes.Structure):
    _fields_ = [
        ("ptr", _p * 2),
        ("scale", _p * 2),
        ("shift", _p * 2),
        ("chans", _i * 2),
        ("xform", _i * 2),
        ("H", _i),
        ("W", _i),
        ("taps", _i),
        ("pool", _i),
    ]


_SRC = ctypes.POINTER(SdSrc)


class SdQSrc(ctypes.Structure):
    """include/stereo_hip.h: sd_qsrc (one source of an fp8 conv input for sd_fp8_qparams)."""

    _fields_ = [
        ("rows", _p),
        ("nrows", _i),
        ("C", _i),
        ("scale", _p),
        ("shift", _p),
        ("relu", _i),
        ("ident", _i),
        ("qscale", _p),
        ("qshift", _p),
    ]


_QSRC = ctypes.POINTER(SdQSrc)


SD_PACK_CONV3_FWD, SD_PACK_CONV3_DGRAD, SD_PACK_CONVT_FWD, SD_PACK_CONVT_DGRAD = 0, 1, 2, 3
SD_PACK_CONV3_FWD_SPLIT, SD_PACK_CONVT_FWD_SPLIT = 4, 5
SD_CONV_WSPLIT = 1


class SdPackJob(ctypes.Structure):
    """include/stereo_hip.h: sd_pack_job (one weight tensor of sd_pack_weights)."""

    _fields_ = [
        ("w", _p),
        ("kind", _i),
        ("co", _i),
        ("ci", _i),
        ("ci_pad", _i),
        ("kpad", _i),
        ("out_off", _i64),
    ]


_PJOB = ctypes.POINTER(SdPackJob)


class SdWredJob(ctypes.Structure):
    """include/stereo_hip.h: sd_wred_job (one slab reduce of sd_wgrad_reduce_batch)."""

    _fields_ = [
        ("slab", _p),
        ("splits", _i),
        ("M", _i),
        ("N", _i),
        ("layout", _i),
        ("ci_real", _i),
        ("dw", _p),
    ]


_WJOB = ctypes.POINTER(SdWredJob)

# name -> (restype, argtypes); mirrors include/stereo_hip.h
PROTOTYPES: dict[str, tuple] = {
    "sd_version": (_i, []),
    "sd_debug_buffer": (_i, [_p]),
    "sd_clock_probe": (_i, [_i, _i, _p, _p, _p]),
    "sd_conv3x3_bwd_fused_ok": (_i, [_i, _i, _i, _i]),
    "sd_conv3x3_bwd_fused_splits": (_i, [_i, _i, _i]),
    "sd_conv3x3_bwd_fused": (_i, [_p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _i, _i, _i, _i, _p, _p, _p, _p]),
    "sd_conv3x3_bwd_fused_dec_ok": (_i, [_i, _i, _i, _i, _i]),
    "sd_conv3x3_bwd_fused_dec": (_i, [_p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _i, _i, _i, _i, _p, _p, _p, _p,
                                      _p]),
    "sd_last_error": (ctypes.c_char_p, []),
    "sd_device_init": (_i, [_i]),
    "sd_pack_input": (_i, [_i, _p, _i, _i, _i, _i, _i, _p, _p]),
    "sd_pack_input_amax": (_i, [_i, _p, _i, _i, _i, _i, _i, _p, _p, _i, _i, _p]),
    "sd_pack_conv3_w": (_i, [_i, _p, _i, _i, _i, _i, _i, _p, _p]),
    "sd_pack_convT_w": (_i, [_i, _p, _i, _i, _i, _i, _p, _p]),
    "sd_pack_weights": (_i, [_i, _PJOB, _i, _p, _p]),
    "sd_conv_gemm": (_i, [_i, _SRC, _i, _i, _i, _p, _i, _i, _i, _p, _p, _i, _p, _p, _p]),
    "sd_conv_gemm_stat_rows": (_i, [_i, _i, _i, _i, _i]),
    "sd_conv_gemm_bnsum": (_i, [_i, _SRC, _i, _i, _i, _p, _i, _i, _p, _p, _p, _p, _p, _p, _p, _p]),
    "sd_conv_gemm_bnsum_ok": (_i, [_i, _SRC, _i]),
    "sd_conv_gemm_bnsum_rows": (_i, [_SRC, _i, _i, _i, _i]),
    "sd_conv_gemm_bnsum_kernel_name": (ctypes.c_char_p, [_SRC, _i, _i, _i]),
    "sd_conv_gemm_kernel_name": (ctypes.c_char_p, [_i, _SRC, _i, _i, _i, _i, _i]),
    "sd_conv3x3_ex": (_i, [_SRC, _i, _i, _i, _p, _i, _i, _i, _i, _p, _p, _p, _p, _p]),
    "sd_conv3x3_ex_ws": (_i, [_SRC, _i, _i, _i, _p, _i, _i, _i, _i, _p, _p, _p, _p, _p, ctypes.c_longlong, _p]),
    "sd_conv3x3_ex_ws_bytes": (ctypes.c_longlong, [_SRC, _i, _i, _i, _i, _i, _i]),
    "sd_conv3x3_ex_ok": (_i, [_SRC, _i]),
    "sd_conv3x3_ex_kernel_name": (ctypes.c_char_p, [_SRC, _i, _i, _i, _i, _i, _i]),
    "sd_wgrad_kernel_name": (ctypes.c_char_p, [_i, _SRC, _SRC, _i, _i]),
    "sd_wgrad_splits": (_i, [_i, _i, _i, _i, _i, _i]),
    "sd_wgrad_gemm": (_i, [_i, _SRC, _SRC, _i, _i, _i, _i, _i, _p, _i, _p]),
    "sd_wgrad_bnbwd_ok": (_i, [_i, _SRC, _SRC, _i, _i]),
    "sd_wgrad_gemm_bnbwd": (_i, [_i, _SRC, _SRC, _i, _i, _i, _i, _i, _p, _p, _p, _p, _p, _p, _p, _p, _i, _p]),
    "sd_wgrad_bnbwd_kernel_name": (ctypes.c_char_p, [_SRC, _SRC, _i, _i]),
    "sd_wgrad_reduce": (_i, [_p, _i, _i, _i, _i, _i, _p, _p]),
    "sd_wgrad_reduce_batch": (_i, [_WJOB, _i, _p]),
    "sd_bn_fwd_finalize": (_i, [_p, _i, _i, _d, _p, _p, _p, _p, _p, _f, _f, _p, _p, _p, _p, _p]),
    "sd_bn_eval_coeffs": (_i, [_p, _p, _p, _p, _i, _f, _p, _p, _p, _p, _p]),
    "sd_chan_reduce_rows": (_i, [_i64, _i]),
    "sd_bn_bwd_reduce": (_i, [_i, _p, _p, _p, _p, _p, _p, _i64, _i, _p, _p]),
    "sd_bn_bwd_finalize": (_i, [_p, _i, _i, _d, _p, _p, _i, _p, _p, _p, _p]),
    "sd_read_cache_batch": (_i, [_p, _i, _i, _i, _p, _p, _p, _i, ctypes.c_char_p, _i]),
    "sd_png_size": (_i, [ctypes.c_char_p, _p, _p]),
    "sd_read_png_batch": (_i, [_p, _i, _i, _i, _p, _i, ctypes.c_char_p, _i]),
    "sd_bn_rows_sum64": (_i, [_p, _i, _i, _d, _p, _p]),
    "sd_bn_fwd_finalize64": (_i, [_p, _i, _p, _p, _p, _p, _p, _f, _f, _p, _p, _p, _p, _p]),
    "sd_bn_bwd_finalize64": (_i, [_p, _p, _i, _p, _p, _i, _p, _p, _p, _p]),
    "sd_bn_bwd_apply": (_i, [_i, _p, _p, _p, _p, _p, _p, _p, _i64, _i, _p, _p]),
    "sd_pool_bwd_add": (_i, [_i, _p, _p, _p, _p, _p, _i, _i, _i, _i, _p, _p, _p, _p, _p]),
    "sd_pool_bwd_rows": (_i, [_i, _i, _i, _i]),
    "sd_bnrelu_pool": (_i, [_i, _p, _p, _p, _i, _i, _i, _i, _p, _p]),
    "sd_chan_sum": (_i, [_i, _p, _i64, _i, _p, _p, _p]),
    "sd_stat_rows_sum": (_i, [_p, _i, _i, _i, _p, _p]),
    "sd_count_valid": (_i, [_p, _p, _i64, _p, _i, _p, _p]),
    "sd_step_prologue": (_i, [_i, _PJOB, _i, _p, _p, _i, _i, _i, _i, _i, _p, _p, _p, _i64, _p, _i, _p, _p]),
    "sd_heads_rows": (_i, [_i64]),
    "sd_heads": (_i, [_i, _i, _p, _p, _p, _i64, _i, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p]),
    "sd_heads_bnsum": (_i, [_i, _i, _p, _p, _p, _i64, _i, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p,
                            _p, _p]),
    "sd_heads_finalize": (_i, [_p, _i, _i, _p, _p, _p, _p, _p, _p, _p]),
    "sd_pack_conv3_w_fp8": (_i, [_p, _i, _i, _i, _i, _p, _p, _p]),
    "sd_conv3x3_fp8": (_i, [_SRC, _i, _i, _i, _p, _p, _p, _i, _i, _p, _p, _p]),
    "sd_conv3x3_q8": (_i, [_SRC, _i, _i, _i, _p, _p, _p, _i, _i, _p, _p]),
    "sd_conv3x3_q8_kernel_name": (ctypes.c_char_p, [_i, _i, _i, _i, _i, _i]),
    "sd_conv3x3_fp8_rows": (_i, [_i, _i, _i, _i]),
    "sd_conv3x3_fp8_kernel_name": (ctypes.c_char_p, [_i]),
    "sd_chan_minmax_rows": (_i, [_i64, _i]),
    "sd_chan_minmax": (_i, [_p, _i64, _i, _p, _p]),
    "sd_fp8_qparams": (_i, [_QSRC, _i, _p, _p]),
    "sd_adamw": (_i, [_p, _p, _p, _p, _i64, _d, _d, _d, _d, _d, _p, _p, _p, _p]),
    "sd_resize_bilinear": (_i, [_p, _i, _i, _i, _p, _i, _i, _f, _p]),
    "sd_stereo_preprocess": (_i, [_p, _p, _p, _i, _i, _i, _i, _i, _p, _p, _p, _p]),
    "sd_stereo_from_cache": (_i, [_p, _p, _p, _i, _i, _i, _p, _p, _p, _p]),
    "sd_augment_rgb": (_i, [_p, _i, _i, _i, _p, _i, ctypes.c_uint64, _p, _p]),
}

_lib = None


class StereoHipError(RuntimeError):
    pass


def load() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not LIB_PATH.exists():
            raise StereoHipError(
                f"{LIB_PATH} not found: build the HIP library first (`make` or __graft_entry__.build()). "
                "There is no CPU fallback."
            )
        lib = ctypes.CDLL(str(LIB_PATH), mode=os.RTLD_NOW | getattr(os, "RTLD_GLOBAL", 0))
        for name, (res, args) in PROTOTYPES.items():
            if os.environ.get("SD_HIP_LIB") and not hasattr(lib, name):
                continue  # an A/B build may predate an entry point
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
    return _lib


_hook = None


def set_call_hook(fn) -> None:
    """fn(name, args, phase) with phase 'pre'/'post' around every launch (profiling; None disables)."""
    global _hook
    _hook = fn


def kernel_name(name: str, *args) -> str:
    return getattr(load(), name)(*args).decode()


def call(name: str, *args) -> int:
    """Call an int-returning entry point; raise StereoHipError with sd_last_error() on failure."""
    lib = load()
    if name.endswith(("_rows", "_splits", "_ok", "_bytes")) or name == "sd_version":
        return getattr(lib, name)(*args)
    if _hook is not None:
        _hook(name, args, "pre")
    rc = getattr(lib, name)(*args)
    if _hook is not None:
        _hook(name, args, "post")
    if rc != 0:
        raise StereoHipError(f"{name} failed ({rc}): {lib.sd_last_error().decode(errors='replace')}")
    return rc


def ptr(t) -> int | None:
    """Raw device pointer of a tensor (None for None; raw ints / c_void_p pass through)."""
    if t is None or isinstance(t, int):
        return t
    if isinstance(t, ctypes.c_void_p):
        return t.value
    return t.data_ptr()


def stream_handle(device=None) -> int:
    return torch.cuda.current_stream(device).cuda_stream


def make_src(
    src0,
    c0: int,
    H: int,
    W: int,
    taps: int = 9,
    pool: bool = False,
    bn0=None,
    src1=None,
    c1: int = 0,
    bn1=None,
    xform0: int | None = None,
    xform1: int | None = None,
) -> SdSrc:
    """sd_src for one or two NHWC tensors; bnX = (scale, shift) float32 tensors or None (identity).
    A given affine is SD_BNRELU unless xformX overrides it (SD_AFFINE: the fp8 gather's signed form)."""
    s = SdSrc()
    s.ptr[0] = ptr(src0)
    s.ptr[1] = ptr(src1) if src1 is not None else None
    s.chans[0], s.chans[1] = c0, c1
    for i, bn in ((0, bn0), (1, bn1)):
        if bn is None:
            s.xform[i] = SD_IDENT
            s.scale[i] = s.shift[i] = None
        else:
            xf = (xform0, xform1)[i]
            s.xform[i] = SD_BNRELU if xf is None else xf
            s.scale[i], s.shift[i] = ptr(bn[0]), ptr(bn[1])
    s.H, s.W, s.taps, s.pool = H, W, taps, int(bool(pool))
    # the struct holds raw pointers: keep the tensors alive as long as it is (temporaries such as
    # `bn0=(sc.to(dev), sh.to(dev))` would otherwise return to the caching allocator before the launch)
    s._keep = (src0, src1, bn0, bn1)
    return s


def make_qsrc(rows, nrows: int, C: int, qscale, qshift, bn=None, relu: bool = False, ident: bool = False) -> SdQSrc:
    """sd_qsrc for sd_fp8_qparams; bn = (scale, shift) of the source's transform or None (identity)."""
    q = SdQSrc()
    q.rows, q.nrows, q.C = ptr(rows), nrows, C
    q.scale, q.shift = (None, None) if bn is None else (ptr(bn[0]), ptr(bn[1]))
    q.relu, q.ident = int(bool(relu)), int(bool(ident))
    q.qscale, q.qshift = ptr(qscale), ptr(qshift)
    return q


def exported_symbols() -> list[str]:
    return list(PROTOTYPES)
