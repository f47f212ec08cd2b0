"""Where does the bf16 eval forward lose EPE? ("localise")

CPU emulation of the HIP bf16 eval forward (engine.py `_forward_body`, eval BN) in fp32 torch ops, with every
rounding point of the kernels made explicit and switchable per layer:
  in   : the packed network input (sd_pack_input: fp32 -> bf16)
  w    : a layer's packed weights (sd_pack_weights: fp32 -> bf16, RNE)
  a    : a layer's gathered operand (relu(bn(y)) in fp32 -> bf16 MFMA operand; pooled tensors are stored bf16)
  y    : a layer's raw output stored in HBM (fp32 accumulator -> bf16)
MFMA accumulates in fp32, which the fp32 conv here restates up to summation order; the heads run in fp32 on
relu(bn(y_dec1.1)) (k_heads). With every switch on, this is the product bf16 path; with every switch off, the
reference's fp32 forward. Prints EPE (the reference's `mae`, train.py:350,406) deltas against fp32 for
single-layer ablations (one layer exact, the rest bf16) and for candidate fixes.

    python tools/precision_study.py [tests/golden/trained_state.npz]
"""

from __future__ import annotations

import sys
from pathlib import Path

import numpy as np
import torch
import torch.nn.functional as F

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

from oracle import unet_ref as U  # noqa: E402
from stereo_depth_estimation_amd.data import synthetic_batch  # noqa: E402

CONVS = [f"{b}.{i}" for b in U.BLOCKS for i in (0, 1)]
LAYERS = CONVS + list(U.UPS)


def rb(x):
    return x.to(torch.bfloat16).float()


def e4m3(x, scale):
    """Round x/scale to e4m3 (saturating at 448) and back (the q8 kernels' v_cvt_pk_fp8_f32, RNE)."""
    return (x / scale).clamp(-448, 448).to(torch.float8_e4m3fn).float() * scale


class Emu:
    """cfg[layer] = set of rounding points kept for that layer ({"w","a","y"}); cfg["in"] = bool; hi/lo options:
    cfg["wsplit"] = layers whose weights are hi+lo bf16 (exact to ~2^-17), cfg["asplit"] = layers whose operand is
    hi+lo, cfg["y32"] = layers whose output is stored fp32. fp8 = set of conv layers run as e4m3 (static scales)."""

    def __init__(self, state, cfg, fp8=()):
        self.s = {k: torch.as_tensor(np.asarray(v)).float() for k, v in state.items()}
        self.cfg = cfg
        self.fp8 = set(fp8)

    def _has(self, layer, what):
        return what in self.cfg.get(layer, {"w", "a", "y"})

    def coeff(self, name):
        blk, idx = name.split(".")
        pre = f"{blk}.block.{1 if idx == '0' else 4}"
        rm, rv = self.s[pre + ".running_mean"], self.s[pre + ".running_var"]
        g, b = self.s[pre + ".weight"], self.s[pre + ".bias"]
        invstd = 1.0 / torch.sqrt(rv + U.BN_EPS)
        sc = g * invstd
        return sc.view(1, -1, 1, 1), (b - rm * sc).view(1, -1, 1, 1)

    def act(self, name, y):
        sc, sh = self.coeff(name)
        return torch.relu(y * sc + sh)

    def operand(self, layer, z):
        if layer in self.cfg.get("asplit", ()):
            return rb(z) + rb(z - rb(z))
        return rb(z) if self._has(layer, "a") else z

    def weight(self, layer, w):
        if layer in self.cfg.get("wsplit", ()):
            return rb(w) + rb(w - rb(w))
        return rb(w) if self._has(layer, "w") else w

    def store(self, layer, y):
        if layer in self.cfg.get("y32", ()):
            return y
        if layer in self.cfg.get("zstore", ()) and layer in CONVS:  # store the BN-applied z = scale*y + shift in bf16
            sc, sh = self.coeff(layer)
            return (rb(y * sc + sh) - sh) / sc
        if layer in self.cfg.get("yoff", ()) and layer in CONVS:  # store y - running_mean (BN's centre) in bf16
            blk, idx = layer.split(".")
            c = self.s[f"{blk}.block.{1 if idx == '0' else 4}.running_mean"].view(1, -1, 1, 1)
            return rb(y - c) + c
        return rb(y) if self._has(layer, "y") else y

    def conv(self, name, a):
        blk, idx = name.split(".")
        w = self.s[f"{blk}.block.{0 if idx == '0' else 3}.weight"]
        if name in self.fp8:
            amax = a.abs().max()
            sa = amax / 448.0
            sw = w.abs().amax(dim=(1, 2, 3), keepdim=True) / 448.0
            aq = a if self.cfg.get("f8w_only") else e4m3(a, sa)
            wq = w if self.cfg.get("f8a_only") else e4m3(w, sw)
            y = F.conv2d(aq, wq, padding=1)
            if self.cfg.get("f8emp"):  # empirical per-channel bias correction on this input: + mean(exact - fp8)
                y = y + (F.conv2d(a, w, padding=1) - y).mean(dim=(0, 2, 3), keepdim=True)
            if self.cfg.get("f8bc"):  # bias correction: minus sum_k (wq - w)_ok * mean(a_k) (per output channel)
                am = a.mean(dim=(0, 2, 3))
                y = y - ((wq - w).sum(dim=(2, 3)) * am[None, :]).sum(1).view(1, -1, 1, 1)
        else:
            y = F.conv2d(self.operand(name, a), self.weight(name, w), padding=1)
        return self.store(name, y)

    def up(self, name, z):
        w, b = self.s[name + ".weight"], self.s[name + ".bias"]
        return self.store(name, F.conv_transpose2d(self.operand(name, z), self.weight(name, w), b, stride=2))

    def block(self, blk, a0):
        y0 = self.conv(blk + ".0", a0)
        y1 = self.conv(blk + ".1", self.act(blk + ".0", y0))
        return self.act(blk + ".1", y1)

    def pool(self, z, layer):
        # bf16: sd_bnrelu_pool materialises max(relu(bn(y))) in bf16 (the next layer's operand, rounding = monotone)
        return F.max_pool2d(z, 2)

    @torch.no_grad()
    def forward(self, x):
        x = rb(x) if self.cfg.get("in", True) else x
        s1 = self.block("enc1", x)
        s2 = self.block("enc2", self.pool(s1, "enc2.0"))
        s3 = self.block("enc3", self.pool(s2, "enc3.0"))
        s4 = self.block("enc4", self.pool(s3, "enc4.0"))
        b = self.block("bottleneck", self.pool(s4, "bottleneck.0"))
        d4 = self.block("dec4", torch.cat([self.up("up4", b), s4], 1))
        d3 = self.block("dec3", torch.cat([self.up("up3", d4), s3], 1))
        d2 = self.block("dec2", torch.cat([self.up("up2", d3), s2], 1))
        d1 = self.block("dec1", torch.cat([self.up("up1", d2), s1], 1))
        disp = F.softplus(F.conv2d(d1, self.s["disparity_head.weight"], self.s["disparity_head.bias"]))
        lv = F.conv2d(d1, self.s["logvar_head.weight"], self.s["logvar_head.bias"]).clamp(-6.0, 3.0)
        return disp, lv


def epe(disp, target, valid):
    m = valid & torch.isfinite(target)
    return float((disp[m].double() - target[m].double()).abs().mean())


def main():
    path = sys.argv[1] if len(sys.argv) > 1 else "tests/golden/trained_state.npz"
    st = dict(np.load(path))
    torch.set_num_threads(8)
    H, W, B = (int(v) for v in (sys.argv[2:5] if len(sys.argv) > 4 else (240, 320, 4)))
    b = synthetic_batch(B, H, W, seed=90_001)
    x, t, v = b["input"], b["target"], b["valid_mask"]
    ref = Emu(st, {l: set() for l in LAYERS} | {"in": False})
    d32, _ = ref.forward(x)
    e32 = epe(d32, t, v)
    full = Emu(st, {})
    d16, _ = full.forward(x)
    print(f"fp32 EPE {e32:.6f}  bf16 EPE {epe(d16, t, v):.6f}  delta {epe(d16, t, v) - e32:+.2e}  "
          f"per-pixel mean |d| {float((d16 - d32).abs().mean()):.2e}  max {float((d16 - d32).abs().max()):.2e}")

    def run(tag, cfg, fp8=()):
        d, _ = Emu(st, cfg, fp8).forward(x)
        print(f"{tag:40s} delta {epe(d, t, v) - e32:+.2e}  mean|d| {float((d - d32).abs().mean()):.2e}", flush=True)

    full_res = ["enc1.0", "enc1.1", "dec1.0", "dec1.1", "up1"]
    if "--fp8" in sys.argv:  # the fp8 live path: e4m3 convs below full resolution (static per-tensor activation scales)
        inner = [c for c in CONVS if not c.endswith(("1.0", "1.1")) or c.startswith(("enc2", "dec2", "enc3", "dec3",
                                                                                         "enc4", "dec4", "bott"))]
        lvl = {c: (0 if c.split(".")[0] in ("enc1", "dec1") else 1 if c.split(".")[0] in ("enc2", "dec2") else 2)
               for c in CONVS}
        for tag, cfg, f8 in (
            ("bf16 + wsplit full-res", {"wsplit": full_res}, ()),
            ("fp8 levels>=1, full-res bf16", {}, [c for c in CONVS if lvl[c] >= 1]),
            ("fp8 levels>=1, full-res wsplit", {"wsplit": full_res}, [c for c in CONVS if lvl[c] >= 1]),
            ("fp8 levels>=2, wsplit full-res", {"wsplit": full_res}, [c for c in CONVS if lvl[c] >= 2]),
            ("fp8 encoder>=1 only, wsplit", {"wsplit": full_res}, [c for c in CONVS if lvl[c] >= 1 and c[0] in "eb"]),
            ("fp8 decoder>=1 only, wsplit", {"wsplit": full_res}, [c for c in CONVS if lvl[c] >= 1 and c[0] == "d"]),
            ("fp8>=1 weights only (exact acts)", {"wsplit": full_res, "f8w_only": 1}, [c for c in CONVS if lvl[c] >= 1]),
            ("fp8>=1 acts only (exact weights)", {"wsplit": full_res, "f8a_only": 1}, [c for c in CONVS if lvl[c] >= 1]),
            ("fp8>=1 + bias correction", {"wsplit": full_res, "f8bc": 1}, [c for c in CONVS if lvl[c] >= 1]),
            ("fp8>=1 + empirical bias corr", {"wsplit": LAYERS, "zstore": CONVS, "f8emp": 1},
             [c for c in CONVS if lvl[c] >= 1]),
            ("fp8 enc>=1 + empirical bias corr", {"wsplit": LAYERS, "zstore": CONVS, "f8emp": 1},
             [c for c in CONVS if lvl[c] >= 1 and c[0] in "eb"]),
            ("fp8>=1, zstore+wsplit bf16 rest", {"wsplit": LAYERS, "zstore": CONVS}, [c for c in CONVS if lvl[c] >= 1]),
            ("fp8>=1 + bias corr + wsplit all", {"wsplit": LAYERS, "f8bc": 1}, [c for c in CONVS if lvl[c] >= 1]),
        ):
            run(tag, cfg, f8)
        del inner
        return
    if "--many" in sys.argv:  # EPE deltas over more validation pairs (8 batches): does the remainder average out?
        cfgs = {"bf16": {}, "wsplit enc1.0": {"wsplit": ["enc1.0"]},
                "wsplit full-res": {"wsplit": ["enc1.0", "enc1.1", "dec1.0", "dec1.1", "up1"]},
                "wsplit all": {"wsplit": LAYERS}}
        if "--product" in sys.argv:  # the engine's eval forward options
            cfgs = {"wsplit all + zstore": {"wsplit": LAYERS, "zstore": CONVS},
                    "wsplit convs + zstore": {"wsplit": CONVS, "zstore": CONVS},
                    "zstore only": {"zstore": CONVS}}
        if "--actgroups" in sys.argv:  # with every weight split: which activation roundings carry the noise
            dec = [l for l in LAYERS if l.startswith(("dec", "up"))]
            enc = [l for l in LAYERS if l.startswith(("enc", "bott"))]
            cfgs = {"wsplit all": {"wsplit": LAYERS},
                    "+ zstore all": {"wsplit": LAYERS, "zstore": LAYERS},
                    "+ zstore + asplit all": {"wsplit": LAYERS, "zstore": LAYERS, "asplit": LAYERS},
                    "+ y32 all": {"wsplit": LAYERS, "y32": LAYERS},
                    "+ asplit all": {"wsplit": LAYERS, "asplit": LAYERS},
                    "+ dec acts exact": {"wsplit": LAYERS, "asplit": dec, "y32": dec},
                    "+ enc acts exact": {"wsplit": LAYERS, "asplit": enc, "y32": enc},
                    "+ full-res acts exact": {"wsplit": LAYERS, "asplit": full_res, "y32": full_res}}
        if "--subsets" in sys.argv:
            cfgs = {"+".join(s): {"wsplit": list(s)} for s in (
                ("enc1.0", "enc1.1"), ("enc1.0", "dec1.1"), ("enc1.0", "dec1.0"), ("enc1.0", "up1"),
                ("enc1.0", "dec1.0", "dec1.1"), ("enc1.0", "enc1.1", "dec1.1"), ("enc1.0", "enc1.1", "dec1.0", "dec1.1"))}
        acc = {k: [0.0, 0.0, 0] for k in cfgs}  # sum |p-t| (cfg), sum |p-t| (fp32), n
        per = {k: [] for k in cfgs}
        for i in range(8):
            bb = synthetic_batch(B, H, W, seed=91_000 + i)
            m = bb["valid_mask"] & torch.isfinite(bb["target"])
            p32, _ = ref.forward(bb["input"])
            e32 = float((p32[m].double() - bb["target"][m].double()).abs().sum())
            line = []
            for k, cfg in cfgs.items():
                p, _ = Emu(st, cfg).forward(bb["input"])
                e = float((p[m].double() - bb["target"][m].double()).abs().sum())
                n = int(m.sum())
                acc[k][0] += e
                acc[k][1] += e32
                acc[k][2] += n
                per[k].append((e - e32) / n)
                line.append(f"{k}: {(e - e32) / n:+.2e}")
            print(f"batch {i}: " + "  ".join(line), flush=True)
        for k, (e, e32, n) in acc.items():
            d = np.array(per[k])
            print(f"{k:22s} delta over {8 * B} pairs: {(e - e32) / n:+.2e}   per-batch std {d.std():.2e} "
                  f"max |.| {np.abs(d).max():.2e}")
        return
    if "--off" in sys.argv:  # centred bf16 storage of the conv outputs (y - running_mean)
        for pre in CONVS:
            blk, idx = pre.split(".")
            k = f"{blk}.block.{1 if idx == '0' else 4}"
            rm, rv = st[k + ".running_mean"], st[k + ".running_var"]
            r = np.abs(rm) / np.sqrt(rv + 1e-5)
            print(f"{pre:14s} |mean|/std: median {np.median(r):7.2f}  max {r.max():7.2f}")
        run("wsplit enc1.0", {"wsplit": ["enc1.0"]})
        run("wsplit enc1.0 + yoff all", {"wsplit": ["enc1.0"], "yoff": CONVS})
        run("wsplit enc1.0 + yoff enc1.0", {"wsplit": ["enc1.0"], "yoff": ["enc1.0"]})
        run("wsplit full-res + yoff all", {"wsplit": ["enc1.0", "enc1.1", "dec1.0", "dec1.1", "up1"], "yoff": CONVS})
        run("wsplit all + yoff all", {"wsplit": LAYERS, "yoff": CONVS})
        run("yoff all", {"yoff": CONVS})
        return
    if "--act" in sys.argv:  # with every weight split: which layers' activation roundings remain
        base = {"wsplit": LAYERS}
        run("wsplit all", base)
        for l in LAYERS:
            run(f"+ {l} activations exact", base | {"asplit": [l], "y32": [l]})
        for grp, ls in (("dec1", ["dec1.0", "dec1.1"]), ("dec1+up1", ["dec1.0", "dec1.1", "up1"]),
                        ("decoder", [l for l in LAYERS if l.startswith(("dec", "up"))]),
                        ("encoder", [l for l in LAYERS if l.startswith(("enc", "bottleneck"))]),
                        ("full-res", ["enc1.0", "enc1.1", "dec1.0", "dec1.1", "up1"])):
            run(f"+ {grp} activations exact", base | {"asplit": ls, "y32": ls})
            run(f"+ {grp} y32 only", base | {"y32": ls})
        return
    if "--fixes" in sys.argv:
        full_res = ["enc1.0", "enc1.1", "dec1.0", "dec1.1", "up1"]
        for tag, cfg in (
            ("wsplit enc1.0", {"wsplit": ["enc1.0"]}),
            ("wsplit enc1.0 + input exact", {"wsplit": ["enc1.0"], "in": False}),
            ("wsplit enc1", {"wsplit": ["enc1.0", "enc1.1"]}),
            ("wsplit full-res", {"wsplit": full_res}),
            ("wsplit full-res + input exact", {"wsplit": full_res, "in": False}),
            ("wsplit all", {"wsplit": LAYERS}),
            ("wsplit all + input exact", {"wsplit": LAYERS, "in": False}),
            ("wsplit all + asplit enc1.0", {"wsplit": LAYERS, "in": False, "asplit": ["enc1.0"]}),
            ("wsplit all + y32 full-res", {"wsplit": LAYERS, "in": False, "y32": full_res}),
        ):
            run(tag, cfg)
        for l in LAYERS:
            run(f"wsplit {l} only", {"wsplit": [l]})
        return
    run("input exact", {"in": False})
    for what in ("w", "a", "y"):
        run(f"all layers: no '{what}' rounding", {l: {"w", "a", "y"} - {what} for l in LAYERS})
    for l in LAYERS:
        run(f"{l} exact", {l: set()})
    for grp, ls in (("dec1", ["dec1.0", "dec1.1", "up1"]), ("dec1+dec2", ["dec1.0", "dec1.1", "up1", "dec2.0", "dec2.1", "up2"]),
                    ("enc1", ["enc1.0", "enc1.1"]), ("full-res (enc1, dec1, up1)", ["enc1.0", "enc1.1", "dec1.0", "dec1.1", "up1"])):
        run(f"{grp} exact", {l: set() for l in ls})
        run(f"{grp} exact + input", {l: set() for l in ls} | {"in": False})


if __name__ == "__main__":
    main()
