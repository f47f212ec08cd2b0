#!/usr/bin/env python3
"""bench.py — stereo pairs/s of the HIP training step @320x240 bf16 on 1..8 MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 \
        --master-port P bench.py --gpus N --steps K --warmup W

A "step" = one full training step of StereoUNet(base 32) on one batch of 64 synthetic
320x240 stereo pairs per GPU (BASELINE.json configs[1]; configs[2] at N=8): pack weights,
forward with BN-stat epilogues, heads + masked heteroscedastic NLL + its gradient, full
backward, (N>1: bucketed RCCL all-reduce overlapped with backward), fused AdamW.
Inputs are pre-generated and resident in HBM (ring of 4 batches).  Timing: W untimed
warmup steps, barrier + synchronize, K steps, barrier + synchronize, max over ranks.
`value` = pairs processed by all ranks / that time (weak scaling: 64 pairs per GPU).

`roofline`: the dominant GEMM kernel instance (largest summed time), timed live with HIP
events around each of its launches inside the timed region; achieved = algorithmic FLOPs
(2*M*N*K with real, unpadded channels) per launch / mean launch duration; peak = 2500
TFLOP/s dense bf16 (MI355X_MICROARCH.md). A kernel below the ridge (FLOP per byte < 2500/8) is priced in
bytes instead: algorithmic bytes per launch / mean launch duration against 8000 GB/s. `traffic` = that kernel's HBM bytes per launch from
the committed rocprofv3 PMC summary of this same command (profiles/pmc_traffic.json, made by
tools/pmc_traffic.py: 1024*(2*FETCH_SIZE + WRITE_SIZE), the guide's gfx950 corrections).
`cpu_baseline`: the oracle's PyTorch-CPU fp32 restatement of the reference train step (B=2,
320x240), timed on this host (rank 0, N=1). `epe` (N=1): after --epe-steps synthetic training
steps, the validation EPE (the reference's `mae`) of the bf16 path, the fp32 path (pinned to the
reference within 1e-3 per pixel by the tests) and their difference.
`comm` (N>1): process-group backend and world size, bucket sizes, and the all-reduce time per
step that backward did not hide.
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time
from collections import defaultdict

METRIC = "stereo pairs/s training @320x240 bf16, 1/2/4/8 MI355X; EPE vs ref"
PEAK_BF16_TFLOPS = 2500.0
PEAK_F32_TFLOPS = 157.3
TRAIN_GFLOP_PER_PAIR = 85.025  # SURVEY §8d (fwd 28.430 + dgrad 28.165 + wgrad 28.430 at 320x240)


def log(msg):
    print(f"[bench] {msg}", file=sys.stderr, flush=True)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=64, help="pairs per GPU")
    ap.add_argument("--height", type=int, default=240)
    ap.add_argument("--width", type=int, default=320)
    ap.add_argument("--precision", default="bf16", choices=("bf16", "fp32"))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-roofline", action="store_true")
    ap.add_argument("--no-infer", action="store_true", help="skip the 960x720 fp8/bf16/fp32 inference lines")
    ap.add_argument("--sync-bn", action="store_true", help="N > 1: global-batch BatchNorm statistics (SyncBatchNorm)")
    ap.add_argument("--epe-steps", type=int, default=2000,
                    help="N=1: synthetic training steps before the EPE comparison (0 skips it)")
    return ap.parse_args()


class GemmTimer:
    """L.call hook: HIP events around every conv-GEMM / wgrad-GEMM launch, grouped by kernel instance."""

    def __init__(self, torch, L, engine):
        self.torch, self.L, self.eng = torch, L, engine
        self.pending = []
        self.cur = None
        self.encoder = []
        self._last_phase = ""
        self._fwd_conv = 0
        self._streams = {}

    def _stream(self, handle):
        cur = self.torch.cuda.current_stream()
        if not handle or handle == cur.cuda_stream:
            return cur
        if handle not in self._streams:
            self._streams[handle] = self.torch.cuda.ExternalStream(handle)
        return self._streams[handle]

    def _flops_and_name(self, name, args):
        L, eng = self.L, self.eng
        if name == "sd_conv3x3_bwd_fused":  # weight gradient + dgrad of a 32 -> 32 full-resolution conv, one pass
            B, H, W = args[14:17]
            return 2.0 * 2.0 * B * H * W * 32 * 9 * 32, "k_bwd_fused32"
        if name == "sd_conv3x3_bwd_fused_dec":  # the same for dec1.0 (64 -> 32 channels)
            B, H, W = args[13:16]
            return 2.0 * 2.0 * B * H * W * 32 * 9 * 64, "k_bwd_fused_dec"
        xin = eng.ws.t["xin"].data_ptr()
        if name in ("sd_conv_gemm", "sd_conv_gemm_bnsum"):
            dt, src, B, H, W, _, N = args[:7]
            s = src._obj if hasattr(src, "_obj") else src
            ctot = s.chans[0] + s.chans[1]
            if s.ptr[0] == xin:
                ctot = eng.in_channels  # enc1.0: 6 real channels padded to 8
            flops = 2.0 * B * H * W * N * s.taps * ctot
            if name == "sd_conv_gemm_bnsum":  # a dgrad (STORE) that also sums the BatchNorm backward
                return flops, L.kernel_name("sd_conv_gemm_bnsum_kernel_name", s, H, W, N)
            return flops, L.kernel_name("sd_conv_gemm_kernel_name", dt, s, B, H, W, N, args[8])
        dt, a, b, B, H, W, M, N = args[:8]
        sb = b._obj if hasattr(b, "_obj") else b
        n_real = N
        if sb.ptr[0] == xin:
            n_real = sb.taps * eng.in_channels
        if name == "sd_wgrad_gemm_bnbwd":
            return 2.0 * B * H * W * M * n_real, L.kernel_name("sd_wgrad_bnbwd_kernel_name", a, sb, M, N)
        return 2.0 * B * H * W * M * n_real, L.kernel_name("sd_wgrad_kernel_name", dt, a, sb, M, N)

    def __call__(self, name, args, phase):
        if name not in ("sd_conv_gemm", "sd_conv_gemm_bnsum", "sd_wgrad_gemm", "sd_wgrad_gemm_bnbwd",
                        "sd_conv3x3_bwd_fused", "sd_conv3x3_bwd_fused_dec"):
            return
        ev = self.torch.cuda.Event(enable_timing=True)
        ev.record(self._stream(args[-1]))  # the launch stream (SD_SIDE_REDUCE=2 puts some GEMMs on a second one)
        if phase == "pre":
            self.cur = (ev, *self._flops_and_name(name, args))
            if getattr(self.eng, "phase", "") != self._last_phase:
                self._last_phase = self.eng.phase
                self._fwd_conv = 0
        else:
            start, flops, kname = self.cur
            nbytes = self._min_bytes(args) if name in ("sd_conv_gemm", "sd_conv_gemm_bnsum") else 0.0
            if name == "sd_conv3x3_bwd_fused":  # da, y, y_prev read, dx written once (bf16, 32 channels)
                nbytes = 4.0 * args[14] * args[15] * args[16] * 32 * 2
            if name == "sd_conv3x3_bwd_fused_dec":  # da, y, u, y_skip read, d(u), d(skip) written once
                nbytes = 6.0 * args[13] * args[14] * args[15] * 32 * 2
            self.pending.append((kname, flops, start, ev, name, self._shape(name, args), nbytes))
            if name == "sd_conv_gemm" and self._last_phase == "fwd":
                # forward order (model.py:79-104): the first 10 3x3 convs are enc1..enc4, bottleneck
                if self._fwd_conv < 10 and args[1].taps == 9:
                    self.encoder.append((self._fwd_conv, flops, self._min_bytes(args), start, ev))
                    self._fwd_conv += 1

    def _min_bytes(self, args):
        """Minimal HBM bytes of one conv-GEMM launch: read the input once, write the output once (bf16),
        read the weights. The input has B*H*W pixels of the GEMM grid for 1x1 and 3x3 (halo) sources and 4x that for
        the 2x2 sub-pixel source of a ConvTranspose2d dgrad (taps = 4: the 2x-resolution gradient); the weights are
        taps x cin x N."""
        s, B, H, W, N = args[1], args[2], args[3], args[4], args[6]
        cin = s.chans[0] + s.chans[1]
        if s.ptr[0] == self.eng.ws.t["xin"].data_ptr():
            cin = self.eng.in_channels
        in_px = B * H * W * (4 if s.taps == 4 else 1)
        return 2.0 * (in_px * cin + B * H * W * N + s.taps * cin * N)

    def encoder_roofline(self, steps, peak_tflops, hbm_gbs=8000.0):
        """Encoder conv forward (enc1..bottleneck) against the per-layer roofline
        min(P_mfma, AI x BW): frac = sum of attainable times / sum of measured times."""
        self.torch.cuda.synchronize()
        per = defaultdict(lambda: [0.0, 0.0, 0.0, 0])  # flops, bytes, ms, n
        for i, flops, nbytes, a, b in self.encoder:
            r = per[i]
            r[0] += flops
            r[1] += nbytes
            r[2] += a.elapsed_time(b)
            r[3] += 1
        layers, t_meas, t_att, fl_tot = [], 0.0, 0.0, 0.0
        names = ["enc1.0", "enc1.1", "enc2.0", "enc2.1", "enc3.0", "enc3.1", "enc4.0", "enc4.1", "bottleneck.0",
                 "bottleneck.1"]
        for i in sorted(per):
            fl, by, ms, n = per[i]
            att_ms = max(fl / (peak_tflops * 1e12), by / (hbm_gbs * 1e9)) * 1e3
            layers.append({"layer": names[i], "ms": round(ms / n, 4), "tflops": round(fl / (ms * 1e-3) / 1e12, 1),
                           "attainable_ms": round(att_ms / n, 4), "bound": "mfma" if fl / (peak_tflops * 1e12)
                           >= by / (hbm_gbs * 1e9) else "hbm", "frac": round(att_ms / ms, 3)})
            t_meas += ms
            t_att += att_ms
            fl_tot += fl
        if not layers:
            return None
        # mfma_frac: SURVEY §8d's encoder-MFMA fraction (encoder fwd FLOPs / their kernel time / the bf16 peak), beside
        # the per-layer roofline fraction (HBM-bound layers priced at their byte time)
        return {"frac_of_roofline": round(t_att / t_meas, 4), "mfma_frac": round(fl_tot / (t_meas * 1e-3) / 1e12 / peak_tflops, 4),
                "achieved_tflops": round(fl_tot / (t_meas * 1e-3) / 1e12, 1),
                "ms_per_step": round(t_meas / steps, 4), "peak_tflops": peak_tflops, "hbm_gbs": hbm_gbs,
                "layers": layers}

    @staticmethod
    def _shape(name, args):
        if name == "sd_conv3x3_bwd_fused":
            return f"bwd_fused P={args[14] * args[15] * args[16]} C=32"
        if name == "sd_conv3x3_bwd_fused_dec":
            return f"bwd_fused_dec P={args[13] * args[14] * args[15]} C=64->32"
        if name in ("sd_conv_gemm", "sd_conv_gemm_bnsum"):
            s = args[1]
            return f"fwd M={args[2] * args[3] * args[4]} N={args[6]} K={s.taps}x{s.chans[0] + s.chans[1]}"
        b = args[2]
        return f"wgrad P={args[3] * args[4] * args[5]} M={args[6]} N={args[7]} taps={b.taps}"

    def per_layer(self, steps):
        self.torch.cuda.synchronize()
        agg = defaultdict(lambda: [0, 0.0, 0.0, ""])
        for kname, flops, a, b, name, shape, _ in self.pending:
            r = agg[shape]
            r[0] += 1
            r[1] += flops
            r[2] += a.elapsed_time(b)
            r[3] = kname
        rows = sorted(((v[2] / steps, k, v[3], v[1] / (v[2] * 1e-3) / 1e12) for k, v in agg.items()), reverse=True)
        return [{"layer": k, "kernel": kn, "ms_per_step": round(ms, 3), "tflops": round(tf, 1)} for ms, k, kn, tf in rows]

    def summary(self, steps):
        self.torch.cuda.synchronize()
        agg = defaultdict(lambda: [0, 0.0, 0.0, 0.0])  # launches, flops, ms, algorithmic bytes
        for kname, flops, a, b, _, _, nbytes in self.pending:
            r = agg[kname]
            r[0] += 1
            r[1] += flops
            r[2] += a.elapsed_time(b)
            r[3] += nbytes
        rows = sorted(((v[2], k, v[0], v[1], v[3]) for k, v in agg.items()), reverse=True)
        if os.environ.get("SD_BENCH_LAYERS"):
            for r in self.per_layer(steps):
                log(json.dumps(r))
        return [{"kernel": k, "launches_per_step": n / steps, "avg_us": 1e3 * ms / n, "flops_per_launch": fl / n,
                 "alg_bytes_per_launch": by / n if by else None, "tflops": fl / (ms * 1e-3) / 1e12,
                 "ms_per_step": ms / steps} for ms, k, n, fl, by in rows]


def conv_layers(H: int = 240, W: int = 320, base: int = 32, cin: int = 6):
    """The U-Net's GEMM-shaped layers (model.py:61-77): (name, kind, cin, cout, out_h, out_w, in_h, in_w); kind conv3
    (3x3, pad 1), convT (2x2 stride 2: in_h x in_w -> out), head (the two 1x1 heads as one 32 -> 2 GEMM)."""
    ch = [base, 2 * base, 4 * base, 8 * base, 16 * base]
    L = []
    c = cin
    for i, blk in enumerate(("enc1", "enc2", "enc3", "enc4", "bottleneck")):
        h, w = H >> i, W >> i
        L += [(blk + ".0", "conv3", c, ch[i], h, w, h, w), (blk + ".1", "conv3", ch[i], ch[i], h, w, h, w)]
        c = ch[i]
    for i, (up, dec) in zip((3, 2, 1, 0), (("up4", "dec4"), ("up3", "dec3"), ("up2", "dec2"), ("up1", "dec1"))):
        h, w = H >> i, W >> i
        L += [(up, "convT", ch[i + 1], ch[i], h, w, h // 2, w // 2),
              (dec + ".0", "conv3", 2 * ch[i], ch[i], h, w, h, w), (dec + ".1", "conv3", ch[i], ch[i], h, w, h, w)]
    L.append(("heads", "head", base, 2, H, W, H, W))
    return L


def step_roofline(ms_per_step: float | None, B: int = 64, H: int = 240, W: int = 320, peak_tflops: float = 2500.0,
                  hbm_gbs: float = 8000.0):
    """SURVEY §8d's whole-step conv roofline: for every conv3x3 / ConvTranspose2d / head GEMM of the training step and
    each of its forward, dgrad (not enc1.0's: the input needs no gradient) and weight gradient, the attainable time
    max(FLOPs / peak, algorithmic bytes / HBM); frac = that sum / the measured ms per step. Algorithmic bytes (bf16
    activations, minimal): fwd reads the input once, writes the output once, reads the weights; dgrad reads dy and the
    weights, writes dx; wgrad reads x and dy, writes the fp32 dW. FLOPs = 2 MACs with real channel counts (85.025
    GFLOP per pair at 320x240)."""
    rows, t_att, fl_tot = {}, 0.0, 0.0
    for name, kind, ci, co, h, w, hi, wi in conv_layers(H, W):
        px_o, px_i = B * h * w, B * hi * wi
        k = 9 if kind == "conv3" else 1
        wts = k * ci * co * (4 if kind == "convT" else 1)
        macs = px_o * co * ci * k if kind != "convT" else px_i * ci * 4 * co
        x_b, y_b = 2.0 * px_i * ci, 2.0 * px_o * co
        ops = {"fwd": (2.0 * macs, x_b + y_b + 2.0 * wts), "wgrad": (2.0 * macs, x_b + y_b + 4.0 * wts)}
        if name != "enc1.0":
            ops["dgrad"] = (2.0 * macs, y_b + x_b + 2.0 * wts)
        r = {}
        for op, (fl, by) in ops.items():
            t_f, t_b = fl / (peak_tflops * 1e12), by / (hbm_gbs * 1e9)
            r[op] = [round(max(t_f, t_b) * 1e6, 2), "mfma" if t_f >= t_b else "hbm"]
            t_att += max(t_f, t_b)
            fl_tot += fl
        rows[name] = r
    res = {"attainable_ms_per_step": round(t_att * 1e3, 4), "gflop_per_pair": round(fl_tot / B / 1e9, 3),
           "ceiling_pairs_s": round(B / t_att, 1), "peak_tflops": peak_tflops, "hbm_gbs": hbm_gbs,
           "definition": "sum over conv3x3/ConvTranspose2d/head GEMMs x {fwd, dgrad, wgrad} of max(FLOPs/peak, "
                         "algorithmic bytes/HBM) at this batch, divided by the measured ms per step (SURVEY §8d)",
           "layers_us": rows}
    if ms_per_step:
        res["measured_ms_per_step"] = round(ms_per_step, 4)
        res["frac"] = round(t_att * 1e3 / ms_per_step, 4)
    return res


def lib_sha256() -> str:
    import hashlib

    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "stereo_depth_estimation_amd", "libstereo_hip.so")
    with open(path, "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()


def pmc_traffic(kernel: str):
    """(HBM bytes per launch of `kernel`, source note) from the committed PMC summary. The bytes are None unless the
    summary was collected from this very library build (its lib_sha256 equals the loaded .so's)."""
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return None, "no PMC summary"
    sha = lib_sha256()
    if d.get("lib_sha256") != sha:
        return None, f"profiles/pmc_traffic.json is from another build ({str(d.get('lib_sha256'))[:12]} != {sha[:12]})"
    ks = d.get("kernels", {})
    # rocprofv3 names every template argument; the library's names leave out trailing defaults (k_halo_conv's OAFF)
    k = ks.get(kernel) or ks.get(kernel[:-1] + ", false>") or ks.get(kernel[:-1] + ", false, false>")
    if k is None:
        return None, "kernel not in profiles/pmc_traffic.json"
    return k.get("hbm_bytes_per_launch"), f"profiles/pmc_traffic.json (same build, {sha[:12]})"


def epe_block(torch, model, opt, dev, steps: int):
    """North star "disparity EPE within 1e-3 of reference" (EPE = the reference's `mae`, the mean |pred - target| over
    valid pixels, train.py:350,406). The bench model is first trained on synthetic pairs (bf16, lr 1e-3, the
    reference's AdamW) until its disparity tracks the targets; then the validation epoch (eval BN, train.py:301)
    runs on held-out synthetic pairs with the same weights in bf16 and in fp32 (the fp32 path is held to the
    reference's CPU path within 1e-3 per pixel; tests/test_gpu_configs.py also checks both EPEs against the CPU
    oracle on a trained checkpoint)."""
    from stereo_depth_estimation_amd.data import synthetic_batch
    from stereo_depth_estimation_amd.model import StereoUNet
    from stereo_depth_estimation_amd.train import run_epoch, train_step

    train = [synthetic_batch(64, 240, 320, seed=50_000 + i, device=dev) for i in range(16)]
    t0 = time.perf_counter()
    model.train()
    for i in range(steps):
        b = train[i % len(train)]
        train_step(model, opt, b["input"], b["target"], b["valid_mask"])
    torch.cuda.synchronize()
    t_train = time.perf_counter() - t0
    val = [synthetic_batch(64, 240, 320, seed=90_000 + i, device=dev) for i in range(2)]
    m16, _ = run_epoch(model, val, dev, optimizer=None)
    ref = StereoUNet(precision="fp32").to(dev)
    ref.load_state_dict(model.state_dict())
    m32, _ = run_epoch(ref, val, dev, optimizer=None)
    ref.eval()
    model.eval()
    with torch.no_grad():
        d16, d32 = model(val[0]["input"]), ref(val[0]["input"])
    vmask = val[0]["valid_mask"]
    # for cpu_autocast_bound (the cpu_baseline leg): the same pairs and weights on the host
    epe_block.held = {"x": val[0]["input"].cpu(), "state": {k: v.detach().cpu().numpy() for k, v in model.state_dict().items()},
                      "d16": d16.float().cpu(), "d32": d32.float().cpu()}
    res = {"train_steps": steps, "train_s": round(t_train, 2), "eval_pairs": 128,
           "epe_bf16": round(m16["mae"], 6), "epe_fp32": round(m32["mae"], 6),
           "delta": round(abs(m16["mae"] - m32["mae"]), 6), "target": 1e-3,
           "met": abs(m16["mae"] - m32["mae"]) < 1e-3,
           "mean_disparity": round(float(d32[vmask].mean()), 3), "mean_target": round(float(val[0]["target"][vmask].mean()), 3),
           "per_pixel_bf16_vs_fp32": {"mean": round(float((d16 - d32).abs().mean()), 6),
                                      "max": round(float((d16 - d32).abs().max()), 6)}}
    model.train()
    return res


def infer_fp8(torch, model, dev, H=720, W=960, iters=20):
    """BASELINE config 5: the live app's forward (depth_live_dl.py:516-529, B=1, eval, both heads) at
    960x720 with e4m3 3x3 convs, next to the bf16 and fp32 forwards of the same trained weights.
    Latency = mean over `iters` back-to-back forwards (HIP events); EPE = mean |disparity - fp32|."""
    from stereo_depth_estimation_amd.data import synthetic_batch
    from stereo_depth_estimation_amd.model import StereoUNet

    sd = model.state_dict()
    x = synthetic_batch(1, H, W, seed=5, device=dev)["input"]
    out, ms = {}, {}
    for prec in ("fp8", "bf16", "bf16_fast", "fp32"):
        m = StereoUNet(precision=prec.split("_")[0])
        m.load_state_dict({k: v.detach().cpu() for k, v in sd.items()})
        m = m.to(dev).eval()
        if prec == "bf16_fast":  # plain bf16 weights in the eval forward (sd_conv3x3_ex's hi/lo pairs off)
            m.engine().wsplit_eval = False
        with torch.inference_mode():
            for _ in range(3):
                m(x, return_uncertainty=True)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(iters):
                d, lv = m(x, return_uncertainty=True)
            e1.record()
            torch.cuda.synchronize()
        ms[prec] = e0.elapsed_time(e1) / iters
        out[prec] = (d.float(), lv.float())
        del m
    d32 = out["fp32"][0]
    res = {"workload": f"StereoUNet(base=32) eval forward, B=1, {W}x{H}, disparity+logvar (live app)",
           "ms_fp8": round(ms["fp8"], 4), "ms_bf16": round(ms["bf16"], 4), "ms_bf16_fast": round(ms["bf16_fast"], 4),
           "ms_fp32": round(ms["fp32"], 4),
           "bf16_eval": "bf16: every weight as a hi/lo bf16 pair and BN-applied stores (the EPE-accurate eval forward, "
                        "sd_conv3x3_ex); bf16_fast: BN-applied stores, plain bf16 weights",
           "pairs_per_s_fp8": round(1e3 / ms["fp8"], 2), "fwd_gflop": 255.87,
           "tflops_fp8": round(255.87e9 / (ms["fp8"] * 1e-3) / 1e12, 1),
           "mean_disparity_fp32": round(float(d32.mean()), 4),
           "fp8_path": "e4m3 3x3 convs at 480x360 and below (80 % of the forward's FLOPs) with static activation scales "
                       "from the first (calibration) forward of the model state; full-res 32-channel convs, ConvTranspose "
                       "and heads bf16",
           "timing": f"mean of {iters} forwards after 3 (calibration, capture, replay): each precision's eval forward "
                     "replays a captured HIP graph"}
    for prec in ("fp8", "bf16", "bf16_fast"):
        res[f"epe_{prec}_vs_fp32"] = round(float((out[prec][0] - d32).abs().mean()), 5)
    return res


def clock_probe(torch, L, dev, iters: int = 20000):
    """Effective shader clock under MFMA load (sd_clock_probe: one block of 4 MFMA waves per CU, ~1 ms): MHz =
    d(s_memtime) / d(s_memrealtime) x 100 per block, and the chip's back-to-back bf16 MFMA rate. Run right before and
    right after the timed region, so box-to-box differences of the same binary can be told apart: a lower clock
    (power/thermal state) moves both the probe and the kernels, contention or a slow memory system only the kernels."""
    n = 256
    if not hasattr(L.load(), "sd_clock_probe"):  # an older build of the C ABI (A/B runs)
        return None
    out = torch.zeros(4 * n, dtype=torch.int64, device=dev)
    sink = torch.zeros(256, dtype=torch.float32, device=dev)
    L.call("sd_clock_probe", n, iters, out.data_ptr(), sink.data_ptr(), L.stream_handle(dev))
    torch.cuda.synchronize(dev)
    o = out.view(n, 4).cpu().double()
    mhz = ((o[:, 1] - o[:, 0]) / (o[:, 3] - o[:, 2]) * 100.0).sort().values
    span_s = float(o[:, 3].max() - o[:, 2].min()) / 100e6
    tflops = n * 4 * iters * 4 * 2 * 32 * 32 * 16 / span_s / 1e12
    return {"mhz_median": round(float(mhz[n // 2]), 1), "mhz_min": round(float(mhz[0]), 1),
            "mfma_tflops": round(tflops, 1), "probe_ms": round(span_s * 1e3, 3)}


def cpu_baseline(seconds: float, height: int, width: int):
    """The oracle's fp32 PyTorch-CPU restatement of the reference train step (train.py:320-343)."""
    import torch

    from oracle import unet_ref as U
    from stereo_depth_estimation_amd.data import synthetic_batch

    cores = max(1, min(16, len(os.sched_getaffinity(0))))
    torch.set_num_threads(cores)
    net = U.Net(U.make_state(32, seed=0))
    opt = U.AdamWState(net.trainable(), lr=1e-3, weight_decay=1e-4)
    bsz = 2
    b = {k: v.numpy() for k, v in synthetic_batch(bsz, height, width, seed=7).items()}
    U.run_epoch(net, [b], opt)  # warm-up
    n, t0 = 0, time.perf_counter()
    while True:
        U.run_epoch(net, [b], opt)
        n += 1
        if time.perf_counter() - t0 >= seconds:
            break
    dt = time.perf_counter() - t0
    return {"value": n * bsz / dt, "unit": "pairs/s", "cores": cores, "kind": "port",
            "sample": f"{n} train steps x {bsz} pairs @{width}x{height} fp32 (oracle restatement of train.py:320-343)"}


def cpu_autocast_bound(held: dict, chunk: int = 8):
    """The checker of epe.per_pixel_bf16_vs_fp32, run on the host in the cpu_baseline leg: the
    reference's own bf16 behaviour on the bench model's weights and validation pairs — the oracle's eval forward under
    torch.autocast("cpu", bfloat16) against its fp32 forward (model.py:79-104; the yardstick of tests/test_gpu_configs.py)
    — beside the HIP bf16 path's deviation from the HIP fp32 path on the same pairs (and the HIP fp32 path's from the
    oracle's fp32, which the tests hold within 1e-3)."""
    import torch

    from oracle import unet_ref as U

    t0 = time.perf_counter()
    net = U.Net(held["state"])
    x = held["x"]
    d32s, dacs = [], []
    with torch.no_grad():
        for i in range(0, x.shape[0], chunk):
            xb = x[i:i + chunk]
            d32s.append(net.forward(xb, train=False)[0])
            with torch.autocast("cpu", dtype=torch.bfloat16):
                dacs.append(net.forward(xb, train=False)[0].float())
    o32, oac = torch.cat(d32s), torch.cat(dacs)
    dev_ac = (oac - o32).abs()
    dev16 = (held["d16"] - held["d32"]).abs()
    flat = int(dev16.flatten().argmax())

    def tail(d):  # the worst pixel of 4.9 M is one draw: the tail's counts and high quantiles beside it
        f = d.flatten().double()
        q = torch.quantile(f[torch.randperm(f.numel(), generator=torch.Generator().manual_seed(0))[:1 << 24]],
                           torch.tensor([0.999, 0.99999], dtype=torch.float64))
        return {"px_over_0.5": int((f > 0.5).sum()), "px_over_1": int((f > 1.0).sum()), "px_over_2": int((f > 2.0).sum()),
                "q999": round(float(q[0]), 5), "q99999": round(float(q[1]), 5)}

    return {"pairs": int(x.shape[0]), "pixels": int(dev16.numel()), "hip_bf16_tail": tail(dev16),
            "reference_autocast_tail": tail(dev_ac), "hip_bf16_max": round(float(dev16.max()), 5),
            "reference_autocast_max": round(float(dev_ac.max()), 5),
            "hip_bf16_mean": round(float(dev16.mean()), 6), "reference_autocast_mean": round(float(dev_ac.mean()), 6),
            "reference_autocast_at_hip_worst_pixel": round(float(dev_ac.flatten()[flat]), 5),
            "hip_fp32_vs_oracle_fp32_max": round(float((held["d32"] - o32).abs().max()), 6),
            "within": float(dev16.max()) <= float(dev_ac.max()), "seconds": round(time.perf_counter() - t0, 1)}


def _free_port() -> int:
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_plan(gpus: int, env: dict, argv: list[str]) -> list[str] | None:
    """How this invocation runs (decided before anything touches a GPU).

    None: run in this process (N=1, or a rank already started by torch.distributed.run). Otherwise the command of a
    CHILD launcher that starts N rank processes of this script (`python bench.py --gpus N` without WORLD_SIZE: the
    driver's own BENCH command form); the parent only waits for it and exits with its code, it never execs.
    A --gpus / WORLD_SIZE mismatch is an error, never a silent one-GPU measurement."""
    if gpus < 1:
        raise SystemExit(f"bench.py: --gpus {gpus} must be >= 1")
    world = env.get("WORLD_SIZE")
    if world is not None:
        if int(world) != gpus:
            raise SystemExit(f"bench.py: --gpus {gpus} but WORLD_SIZE={world}: refusing to measure a different "
                             "number of GPUs than asked for")
        return None
    if gpus == 1:
        return None
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
            "--master-addr", "127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__), *argv]


def _probe_rank(args):
    """SD_BENCH_PROBE=1 (the launcher test, tests/test_bench_launch_cpu.py): each rank joins a gloo group, sums the
    ranks and rank 0 prints one JSON line; no GPU is touched."""
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    t = torch.tensor([rank + 1.0])
    if world > 1:
        dist.init_process_group("gloo")
        dist.all_reduce(t)
    if rank == 0:
        print(json.dumps({"probe": True, "n_gpus": world, "gpus_arg": args.gpus, "rank_sum": float(t.item()),
                          "local_ranks": os.environ.get("LOCAL_WORLD_SIZE")}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main():
    args = parse()
    cmd = launch_plan(args.gpus, dict(os.environ), sys.argv[1:])
    if cmd is not None:
        import subprocess

        log(f"--gpus {args.gpus}: starting {args.gpus} rank processes: {' '.join(cmd)}")
        env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
        raise SystemExit(subprocess.call(cmd, env=env))
    if os.environ.get("SD_BENCH_PROBE") == "1":
        return _probe_rank(args)
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and os.environ.get("SD_BENCH_SHARE_DEVICE", "0") != "1" and torch.cuda.device_count() < world:
        raise SystemExit(f"bench.py: {world} ranks but {torch.cuda.device_count()} visible GPUs")
    # SD_BENCH_SHARE_DEVICE=1: every rank on cuda:0 over gloo, a rehearsal of the N > 1 path (buckets, count
    # all-reduce, barriers, max-over-ranks timing) on a one-GPU box; its rate is not a scaling number
    share = world > 1 and os.environ.get("SD_BENCH_SHARE_DEVICE", "0") == "1"
    if share:
        local_rank = 0
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    if world > 1:
        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        if share:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)

    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from stereo_depth_estimation_amd import _lib as L
    from stereo_depth_estimation_amd.data import synthetic_batch
    from stereo_depth_estimation_amd.model import StereoUNet
    from stereo_depth_estimation_amd.optim import FusedAdamW
    from stereo_depth_estimation_amd.train import train_step

    torch.manual_seed(42)
    model = StereoUNet(precision=args.precision).to(dev).train()
    opt = FusedAdamW(model.parameters(), lr=1e-3, weight_decay=1e-4)
    ddp = None
    if world > 1:
        from stereo_depth_estimation_amd.ddp import DataParallel

        ddp = DataParallel(model, sync_bn=args.sync_bn)
    B, H, W = args.batch, args.height, args.width
    ring = [synthetic_batch(B, H, W, seed=1000 * rank + i, device=dev) for i in range(4)]
    log(f"rank {rank}/{world}: model + {len(ring)} resident batches of {B}x6x{H}x{W} ready")

    def step(i):
        b = ring[i % len(ring)]
        if ddp is not None:
            ddp.step(model, opt, b["input"], b["target"], b["valid_mask"])
        else:
            train_step(model, opt, b["input"], b["target"], b["valid_mask"])

    t_w = time.perf_counter()
    for i in range(args.warmup):
        step(i)
    torch.cuda.synchronize()
    log(f"warmup {args.warmup} steps: {time.perf_counter() - t_w:.1f}s")

    clk_before = clock_probe(torch, L, dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(i)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    clk_after = clock_probe(torch, L, dev)

    # Per-kernel HIP-event timing runs over a second K-step region right after the timed one: an
    # event record between two launches is a barrier packet on the stream (it serialises the queue
    # and added ~0.5 ms per step, 4 %), so the headline region carries none.
    timer = None
    if not args.no_roofline:
        timer = GemmTimer(torch, L, model._engine)
        L.set_call_hook(timer)
        if ddp is not None:
            ddp._reducer().wait_events = []
        for i in range(args.steps):
            step(i)
        torch.cuda.synchronize()
        L.set_call_hook(None)
    if world > 1:
        t = torch.tensor([dt], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    ms_per_step = 1e3 * dt / args.steps
    value = world * B * args.steps / dt
    log(f"timed {args.steps} steps: {dt:.3f}s, {ms_per_step:.2f} ms/step, {value:.1f} pairs/s")

    result = {
        "metric": METRIC,
        "value": round(value, 3),
        "unit": "pairs/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": args.precision,
        "data": "synthetic (pre-generated, HBM-resident rectified stereo pairs; SURVEY §8d recipe)",
        "config": {
            "workload": f"StereoUNet(base=32) full train step (fwd+bwd+AdamW), {W}x{H}, {B} pairs/GPU",
            "global_batch": world * B,
            "per_gpu_batch": B,
            "height": H,
            "width": W,
            "parallelism": f"dp{world}",
            "batchnorm": "sync" if (args.sync_bn and world > 1) else "per-rank",
        },
    }
    result["clock"] = {"before": clk_before, "after": clk_after,
                       "probe": "sd_clock_probe: 256 blocks x 4 waves of back-to-back bf16 MFMAs, ~1 ms, outside the "
                                "timed region; MHz = d(s_memtime)/d(s_memrealtime) x 100"}
    if share:
        result["rehearsal"] = f"gloo, {world} ranks sharing cuda:0 (SD_BENCH_SHARE_DEVICE=1): not a scaling number"
    if world > 1:
        ar = ddp._reducer()
        comm = {"backend": dist.get_backend(), "world_size": dist.get_world_size(), "buckets": len(ar.buckets),
                "bucket_mb": [round((b - a) * 4 / 2**20, 2) for _, a, b in ar.buckets]}
        if ar.wait_events:
            torch.cuda.synchronize()
            exposed = sum(a.elapsed_time(b) for a, b in ar.wait_events) / args.steps
            t = torch.tensor([exposed], device=dev, dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            comm["allreduce_exposed_ms_per_step"] = round(float(t.item()), 4)
            comm["exposed_region"] = "HIP events around the bucket waits before AdamW, max over ranks (second region)"
        result["comm"] = comm
    peak = PEAK_BF16_TFLOPS if args.precision == "bf16" else PEAK_F32_TFLOPS
    step_tflops = TRAIN_GFLOP_PER_PAIR * 1e9 * B * (H * W) / (240 * 320) / (dt / args.steps) / 1e12
    result["step_conv_tflops"] = round(step_tflops, 2)
    if args.precision == "bf16":
        result["step_roofline"] = step_roofline(ms_per_step, B, H, W, peak)
    if timer is not None:
        kern = timer.summary(args.steps)
        top = kern[0]
        traffic, tsrc = pmc_traffic(top["kernel"])
        # arithmetic intensity against the ridge (peak FLOP/s / 8 TB/s): from the PMC bytes of this build when present,
        # else from the algorithmic bytes (inputs and output once, bf16, + weights: SURVEY §8d)
        ai = top["flops_per_launch"] / traffic if traffic else None
        alg = top.get("alg_bytes_per_launch")
        ai_alg = top["flops_per_launch"] / alg if alg else None
        ai_b = ai if ai is not None else ai_alg
        bound = ("mfma" if ai_b >= peak * 1e12 / 8e12 else "hbm") if ai_b is not None else None
        if bound == "hbm":  # priced in bytes: algorithmic bytes per launch / launch time against 8 TB/s
            ach, pk, unit = alg / (top["avg_us"] * 1e-6) / 1e9, 8000.0, "GB/s"
        else:
            ach, pk, unit = top["tflops"], peak, "TFLOP/s"
        result["roofline"] = {
            "bound": bound,
            "alg_bytes_per_launch": alg,
            "flop_per_alg_byte": round(ai_alg, 1) if ai_alg else None,
            "kernel": top["kernel"],
            "achieved": round(ach, 2),
            "peak": pk,
            "unit": unit,
            "frac": round(ach / pk, 4),
            "tflops": round(top["tflops"], 2),
            "traffic": traffic,
            "traffic_source": tsrc,
            "flop_per_byte": round(ai, 1) if ai else None,
            "avg_launch_us": round(top["avg_us"], 2),
            "flops_per_launch": top["flops_per_launch"],
            "launches_per_step": top["launches_per_step"],
            "region": f"HIP events around every conv/wgrad launch of {args.steps} steps after the timed region",
        }
        result["clock"]["dominant_kernel"] = {"kernel": top["kernel"], "avg_launch_us": round(top["avg_us"], 2)}
        result["gemm_kernels"] = [{k: (round(v, 3) if isinstance(v, float) else v) for k, v in r.items()} for r in kern]
        result["encoder_conv_roofline"] = timer.encoder_roofline(args.steps, peak)
    if world == 1 and args.epe_steps > 0:
        log(f"EPE: {args.epe_steps} synthetic training steps, then bf16 / fp32 / oracle validation ...")
        result["epe"] = epe_block(torch, model, opt, dev, args.epe_steps)
    if rank == 0 and world == 1 and not args.no_infer:
        log("fp8 inference (config 5) ...")
        result["infer_960x720"] = infer_fp8(torch, model, dev)
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        log("cpu baseline ...")
        result["cpu_baseline"] = cpu_baseline(args.cpu_seconds, H, W)
        held = getattr(epe_block, "held", None)
        if held is not None and "epe" in result:
            log("reference autocast bound of the bf16 per-pixel deviation (oracle, host) ...")
            result["epe"]["per_pixel_bf16_vs_fp32"]["bound"] = cpu_autocast_bound(held)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
