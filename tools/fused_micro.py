"""Micro-benchmark of the fused full-resolution conv1 backward (sd_conv3x3_bwd_fused) at the bench shape.

    SD_HIP_LIB=build_ab/libstereo_hip_<variant>.so python tools/fused_micro.py [--n=20] [--dec]

B = 64, 240x320, 32 -> 32 channels (--dec: sd_conv3x3_bwd_fused_dec, 32 + 32 -> 32), random operands; prints us per
launch (HIP events, median of 3 rounds of n launches). Variants built with tools/build_variant.sh (e.g. "-DFB_EXP=1") isolate the kernel's phases.
"""

from __future__ import annotations

import json
import os
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import torch  # noqa: E402

from stereo_depth_estimation_amd import _lib as L  # noqa: E402


def main():
    n = next((int(a.split("=")[1]) for a in sys.argv[1:] if a.startswith("--n=")), 20)
    dev = "cuda"
    B, H, W, C = 64, 240, 320, 32
    torch.manual_seed(0)
    bf = lambda *s: torch.randn(*s, device=dev).to(torch.bfloat16)  # noqa: E731
    da, y, yp = bf(B * H * W, C), bf(B * H * W, C), bf(B * H * W, C)
    f = lambda lo=0.5: torch.rand(C, device=dev) + lo  # noqa: E731
    sc, sh, mu, iv, psc, psh, pmu, piv = f(), f(-0.5), f(-0.5), f(), f(), f(-0.5), f(-0.5), f()
    coef = torch.rand(3 * C, device=dev)
    kpad = 320
    wd = bf(C * kpad) * 0.05
    dx = torch.empty(B * H * W, C, device=dev, dtype=torch.bfloat16)
    sp = L.call("sd_conv3x3_bwd_fused_splits", B, H, W)
    slab = torch.empty(sp * C * 288, device=dev)
    part = torch.empty(sp * C * 2, device=dev)
    s = torch.cuda.current_stream().cuda_stream
    fn = "sd_conv3x3_bwd_fused"
    args = [t.data_ptr() for t in (da, y, sc, sh, mu, iv, coef, yp, psc, psh, pmu, piv, wd)] + [kpad, B, H, W] + \
        [dx.data_ptr(), slab.data_ptr(), part.data_ptr(), s]
    if "--dec" in sys.argv:
        fn = "sd_conv3x3_bwd_fused_dec"
        xs, wd2 = bf(B * H * W, C), bf(2 * C * kpad) * 0.05
        dsk = torch.empty_like(dx)
        slab = torch.empty(sp * C * 576, device=dev)
        args = [t.data_ptr() for t in (da, y, sc, sh, mu, iv, coef, yp, xs, psc, psh, wd2)] + [kpad, B, H, W] + \
            [dx.data_ptr(), dsk.data_ptr(), slab.data_ptr(), part.data_ptr(), s]
    for _ in range(3):
        L.call(fn, *args)
    torch.cuda.synchronize()
    res = []
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(n):
            L.call(fn, *args)
        e1.record()
        torch.cuda.synchronize()
        res.append(e0.elapsed_time(e1) * 1e3 / n)
    res.sort()
    out = {"lib": os.path.basename(str(L.LIB_PATH)), "kernel": fn, "us": round(res[1], 1), "rounds": [round(r, 1) for r in res]}
    if "--diag" in sys.argv:  # a -DFB_EXP=32 build: per-wave phase cycles (s_memtime ticks), mean per tile
        dbg = torch.zeros(sp * 8 * 8, dtype=torch.int64, device=dev)
        L.call("sd_debug_buffer", dbg.data_ptr())
        L.call(fn, *args)
        torch.cuda.synchronize()
        d = dbg.view(sp, 8, 8).double().cpu()
        nt = d[:, 0, 7].sum()
        mf = d[:, :4, :7].sum(dim=(0, 1)) / (4 * nt)
        ld = d[:, 4:, :5].sum(dim=(0, 1)) / (4 * nt)
        out["mfma_per_tile"] = dict(zip(["barrier", "wgrad_issue", "dgrad", "epilogue_prev", "unused4", "unused5", "total"], mf.round().tolist()))
        out["loader_per_tile"] = dict(zip(["transform_store", "load_issue", "barrier", "load_wait", "total"], ld.round().tolist()))
    print(json.dumps(out))


if __name__ == "__main__":
    main()
