"""Micro-benchmark of the bf16 3x3 conv (sd_conv_gemm) at the model's layer shapes.

    python tools/conv_micro.py [--modes=default,ck16] [--compare] [--rounds=R]

Times forward convs (BN+ReLU gather, STATS epilogue) and dgrad-style convs (plain gather, STORE
epilogue) at B=64 for each U-Net level with HIP events and prints us/launch and TFLOP/s.
--modes runs each layer once per mode (ck16 / ck32 = SD_HALO_CK, n32x8 = SD_HALO_N32=8, raw0 = SD_HALO_RAW=0); --compare checks that every mode
stores the same outputs as the first (max |diff| relative to max |out|).
"""

from __future__ import annotations

import os
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import torch  # noqa: E402

from stereo_depth_estimation_amd import _lib as L  # noqa: E402

LAYERS = [  # (H, W, cin, cout, stats)
    (240, 320, 8, 32, True),     # enc1.0 (the 8-channel packed network input, CK=8 chunks)
    (240, 320, 32, 32, True),
    (240, 320, 32, 32, False),   # enc1.1 / dec1.1 dgrad
    (240, 320, 32, 64, False),   # dec1.0 dgrad
    (120, 160, 32, 64, True),    # enc2.0
    (120, 160, 64, 64, True),
    (120, 160, 64, 128, False),  # dec2.0 dgrad
    (60, 80, 64, 128, True),
    (60, 80, 128, 128, True),
    (60, 80, 128, 256, False),
    (30, 40, 256, 256, True),
    (30, 40, 512, 256, True),    # dec4.0
    (15, 20, 256, 512, True),
    (15, 20, 512, 512, True),
    (240, 320, 32, 32, "bns"),   # enc1.1 / dec1.1 dgrad with the fused BatchNorm-backward sums (sd_conv_gemm_bnsum)
    (120, 160, 64, 64, "bns"),
]


def run(B, H, W, ci, co, stats, s, dev, n=20):
    torch.manual_seed(0)
    y = torch.randn(B * H * W, ci, device=dev).to(torch.bfloat16)
    sc = torch.rand(ci, device=dev) + 0.5
    sh = torch.randn(ci, device=dev) * 0.1
    kpad = ((9 * ci + 63) // 64) * 64
    w = (torch.randn(co * kpad, device=dev) * 0.05).to(torch.bfloat16)
    o = torch.empty(B * H * W, co, device=dev, dtype=torch.bfloat16)
    bns = stats == "bns"
    stats = stats is True
    epi = L.SD_EPI_STATS if stats else L.SD_EPI_STORE
    src = L.make_src(y, ci, H, W, taps=9, bn0=(sc, sh) if stats else None)
    rows = L.call("sd_conv_gemm_bnsum_rows", src, B, H, W, co) if bns else L.call("sd_conv_gemm_stat_rows",
                                                                                  L.SD_BF16, B, H, W, co)
    st = torch.zeros(rows * co * 2, device=dev)
    if bns:  # the BatchNorm layer whose upstream gradient this dgrad stores: its raw output and constants
        yb = torch.randn(B * H * W, co, device=dev).to(torch.bfloat16)
        bsc, bsh = torch.rand(co, device=dev) + 0.5, torch.randn(co, device=dev) * 0.1
        bmu, bis = torch.randn(co, device=dev) * 0.1, torch.rand(co, device=dev) + 0.5

    def once():
        if bns:
            L.call("sd_conv_gemm_bnsum", L.SD_BF16, src, B, H, W, w.data_ptr(), co, kpad, o.data_ptr(), yb.data_ptr(),
                   bsc.data_ptr(), bsh.data_ptr(), bmu.data_ptr(), bis.data_ptr(), st.data_ptr(), s)
            return
        L.call("sd_conv_gemm", L.SD_BF16, src, B, H, W, w.data_ptr(), co, kpad, epi, o.data_ptr(),
               None, 0, None, st.data_ptr() if stats else None, s)

    for _ in range(3):
        once()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        once()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1000 / n
    name = L.kernel_name("sd_conv_gemm_kernel_name", L.SD_BF16, src, B, H, W, co, epi) + (" bns" if bns else "")
    if os.environ.get("SD_WG_DIAG"):  # per-wave cycle counters of a -DWG_EXP=1024 build
        dbg = torch.zeros(4096 * 8 * 4, dtype=torch.int64, device=dev)
        L.call("sd_debug_buffer", dbg.data_ptr())
        once()
        torch.cuda.synchronize()
        L.call("sd_debug_buffer", None)
        d = dbg.view(-1, 8, 4).double().cpu()
        used = d[:, 0, 3] > 0
        m, ld = d[used, :4].mean((0, 1)), d[used, 4:].mean((0, 1))
        print(f"  diag {H}x{W} {ci}->{co}: mfma compute {m[0]:.0f} epilogue {m[1]:.0f} barrier {m[2]:.0f} total {m[3]:.0f}"
              f" | loader store {ld[0]:.0f} load {ld[1]:.0f} barrier {ld[2]:.0f} total {ld[3]:.0f}", flush=True)
    tot = st.view(rows, co, 2).double().sum(0) if stats else None
    return us, name, o.float(), tot


WGRAD_LAYERS = [  # (H, W, dy channels M, x channels ci)
    (240, 320, 32, 32), (240, 320, 32, 64), (120, 160, 64, 32), (120, 160, 64, 64), (60, 80, 128, 128),
    (30, 40, 256, 256)]
# the ten launches of the 64 x 64-block weight gradient in one training step (enc3.1 .. dec2.0), plus dec2.1
WGRAD_STEP = [(60, 80, 128, 128), (30, 40, 256, 128), (30, 40, 256, 256), (15, 20, 512, 256), (15, 20, 512, 512),
              (30, 40, 256, 512), (30, 40, 256, 256), (60, 80, 128, 256), (60, 80, 128, 128), (120, 160, 64, 128),
              (120, 160, 64, 64)]
WGRAD_MODES = {"mf1": {"SD_WS_MF32": "1", "SD_WS_CO128": "0"}, "mf0": {"SD_WS_MF32": "0", "SD_WS_CO128": "0"},
               "co1": {"SD_WS_CO128": "1"}, "co0": {"SD_WS_CO128": "0"}}


def wgrad(B, s, dev, layers=WGRAD_LAYERS, modes=("default",), rounds=1):
    """sd_wgrad_gemm + sd_wgrad_reduce at the model's 3x3 weight-gradient shapes (bf16); modes (WGRAD_MODES keys)
    alternate per round, the minimum time per mode is printed with each mode's max |dW - dW(first mode)|."""
    for H, W, M, ci in layers:
        P = B * H * W
        dy = torch.randn(P, M, device=dev).to(torch.bfloat16)
        x = torch.randn(P, ci, device=dev).to(torch.bfloat16)
        sc, sh = torch.rand(ci, device=dev) + 0.5, torch.randn(ci, device=dev) * 0.1
        a = L.make_src(dy, M, H, W, taps=1)
        b = L.make_src(x, ci, H, W, taps=9, bn0=(sc, sh))
        N = 9 * ci
        sp = L.call("sd_wgrad_splits", L.SD_BF16, B, H, W, M, N)
        slab = torch.empty(sp * M * N, device=dev)
        dw = torch.empty(M, ci, 3, 3, device=dev)

        def gemm():
            L.call("sd_wgrad_gemm", L.SD_BF16, a, b, B, H, W, M, N, slab.data_ptr(), sp, s)

        def red():
            L.call("sd_wgrad_reduce", slab.data_ptr(), sp, M, N, L.SD_W_CONV3, ci, dw.data_ptr(), s)

        if modes != ("default",):
            flops = 2.0 * P * M * N
            best, ref, line = {}, None, f"wgrad {H}x{W} M={M} ci={ci}:"
            for _ in range(rounds):
                for mode in modes:
                    for k in ("SD_WS_MF32", "SD_WS_CO128"):
                        os.environ.pop(k, None)
                    os.environ.update(WGRAD_MODES.get(mode, {}))
                    t = _time(gemm)
                    best[mode] = min(best.get(mode, 1e30), t)
                    red()
                    torch.cuda.synchronize()
                    if ref is None:
                        ref = dw.clone()
                    best["d" + mode] = float((dw - ref).abs().max() / ref.abs().max())
                    best["n" + mode] = L.kernel_name("sd_wgrad_kernel_name", L.SD_BF16, a, b, M, N)
            for mode in modes:
                line += (f" | {mode}: {best['n' + mode].replace('k_halo_wgrad_ws', '')} {best[mode]:7.1f} us "
                         f"{flops / best[mode] / 1e6:6.1f} TF d={best['d' + mode]:.1e}")
            print(line, flush=True)
            continue
        tg, tr = _time(gemm), _time(red)
        if os.environ.get("SD_WG_DIAG"):  # per-wave cycle counters of a -DWG_EXP=1024 build
            dbg = torch.zeros(4096 * 8 * 4, dtype=torch.int64, device=dev)
            L.call("sd_debug_buffer", dbg.data_ptr())
            gemm()
            torch.cuda.synchronize()
            L.call("sd_debug_buffer", None)
            d = dbg.view(-1, 8, 4).double().cpu()
            used = d[:, 0, 3] > 0
            if bool(used.any()):
                raw = dbg.view(-1, 8, 4).cpu()
                vm = (raw[used, 4:, 1] >> 32).double().mean()
                d[:, 4:, 1] = (raw[:, 4:, 1] & 0xFFFFFFFF).double()
                m, ld = d[used, :4].mean((0, 1)), d[used, 4:].mean((0, 1))
                print(f"  diag cycles/wave: mfma compute {m[0]:.0f} barrier {m[2]:.0f} total {m[3]:.0f} | "
                      f"loader store {ld[0]:.0f} (of it vmcnt wait {vm:.0f}) load {ld[1]:.0f} barrier {ld[2]:.0f} "
                      f"total {ld[3]:.0f}", flush=True)
        flops = 2.0 * P * M * N
        name = L.kernel_name("sd_wgrad_kernel_name", L.SD_BF16, a, b, M, N)
        print(f"wgrad {H}x{W} M={M} ci={ci}: {name} {tg:7.1f} us {flops / tg / 1e6:6.1f} TF | reduce {tr:6.1f} us "
              f"(splits {sp})", flush=True)


def _time(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1000 / n


def main():
    """--modes a,b,...: each mode = env settings joined by '+', e.g. ck16 (SD_HALO_CK=16)."""
    L.load()
    dev = torch.device("cuda:0")
    B = 64
    s = L.stream_handle()
    modes = ["default"]
    for a in sys.argv[1:]:
        if a.startswith("--modes="):
            modes = a.split("=", 1)[1].split(",")
    compare = "--compare" in sys.argv
    rounds = 1
    for a in sys.argv[1:]:
        if a.startswith("--rounds="):  # modes alternate per round; the minimum time per mode is printed
            rounds = int(a.split("=", 1)[1])
    if "--wgrad" in sys.argv or "--wgrad-step" in sys.argv:
        wgrad(B, s, dev, WGRAD_STEP if "--wgrad-step" in sys.argv else WGRAD_LAYERS, tuple(modes), rounds)
        return
    for H, W, ci, co, stats in LAYERS:
        flops = 2.0 * B * H * W * co * 9 * ci
        line = f"{H}x{W} {ci}->{co} {'bns ' if stats == 'bns' else 'fwd ' if stats else 'dgrd'}"
        ref = None
        best = {}
        for _ in range(rounds):
            for mode in modes:
                os.environ.pop("SD_HALO_CK", None)
                os.environ.pop("SD_HALO_N32", None)
                os.environ.pop("SD_HALO_RAW", None)
                for part in mode.split("+"):
                    if part.startswith("ck"):
                        os.environ["SD_HALO_CK"] = part[2:]
                    elif part.startswith("n32x"):  # N=32 full-res tile rows (SD_HALO_N32)
                        os.environ["SD_HALO_N32"] = part[4:]
                    elif part == "raw0":  # register-staged halos for raw sources (SD_HALO_RAW=0)
                        os.environ["SD_HALO_RAW"] = "0"
                us, name, out, tot = run(B, H, W, ci, co, stats, s, dev)
                if mode not in best or us < best[mode][0]:
                    best[mode] = (us, name)
                if compare and ref is None:
                    ref = (out, tot)
                elif compare and mode != modes[0] and "d" + mode not in best:
                    best["d" + mode] = float((out - ref[0]).abs().max()) / max(float(ref[0].abs().max()), 1e-30)
        for mode in modes:
            us, name = best[mode]
            line += f" | {mode}: {name.replace('k_halo_conv', '')} {us:7.1f} us {flops / us / 1e6:6.1f} TF"
            if "d" + mode in best:
                line += f" d={best['d' + mode]:.1e}"
        print(line, flush=True)


if __name__ == "__main__":
    main()
