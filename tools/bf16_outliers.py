"""Where the bf16 eval forward's largest per-pixel disparity deviations from fp32 come from.

    python tools/bf16_outliers.py [--bench-model] > gpurun_out/outliers.json

On the reference-trained checkpoint (tests/golden/trained_state.npz) and its held-out sets (val240: 4 pairs at
240x320, val720: 1 pair at 960x720, regenerated from their seeds), runs the fp32 and the bf16 eval forward of the HIP
path and reports, per set:
  * max / mean / p99.99 of |disp_bf16 - disp_fp32|, beside the reference's own torch.autocast(bf16) drift on the same
    pairs (trained_eval.npz: max / mean of |disp_autocast - disp_fp32|);
  * the top outlier pixels: position, distance to the image border, fp32 disparity and logvar;
  * for the worst pixel, each conv layer's deviation at the pixel's position on that layer's grid (relative to the
    channel RMS of the fp32 activation there), and whether a 2x2 MaxPool window on its path picked another argmax
    channel-wise in bf16 than in fp32 (the pool-argmax-flip hypothesis).
--bench-model: also the model bench.py's EPE block trains (2000 bf16 steps over 16 batches of 64 synthetic pairs, seed
42) on its 64 validation pairs.
"""

from __future__ import annotations

import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import numpy as np  # noqa: E402
import torch  # noqa: E402

DEV = "cuda"
LAYERS = ["enc1.0", "enc1.1", "enc2.0", "enc2.1", "enc3.0", "enc3.1", "enc4.0", "enc4.1", "bottleneck.0",
          "bottleneck.1", "dec4.0", "dec4.1", "dec3.0", "dec3.1", "dec2.0", "dec2.1", "dec1.0", "dec1.1"]
LEVEL = {"enc1": 0, "enc2": 1, "enc3": 2, "enc4": 3, "bottleneck": 4, "dec4": 3, "dec3": 2, "dec2": 1, "dec1": 0}


def _z(eng, name):
    """The layer's eval-mode BN output z = scale*y + shift (NHWC fp32), whether the forward stored y or z."""
    t = eng.ws.t
    y = t["y:" + name].float()
    if name in eng._zs:
        return y
    return y * t["scale:" + name][None, :] + t["shift:" + name][None, :]


def _forward(model, x):
    with torch.no_grad():
        d, lv = model(x, return_uncertainty=True)
    eng = model._engine
    acts = {n: _z(eng, n).cpu() for n in LAYERS}
    return d.cpu(), lv.cpu(), acts


def _layer_trace(acts32, acts16, B, H, W, b, h, w):
    rows = []
    for n in LAYERS:
        lv = LEVEL[n.split(".")[0]]
        Hl, Wl = H >> lv, W >> lv
        a32 = acts32[n].view(B, Hl, Wl, -1)
        a16 = acts16[n].view(B, Hl, Wl, -1)
        hl, wl = h >> lv, w >> lv
        v32, v16 = a32[b, hl, wl], a16[b, hl, wl]
        rms = float(v32.pow(2).mean().sqrt()) + 1e-12
        r32, r16 = torch.relu(v32), torch.relu(v16)
        row = {"layer": n, "pos": [hl, wl], "rel_dev": round(float((v16 - v32).abs().max()) / rms, 5),
               "relu_sign_flips": int(((v32 > 0) != (v16 > 0)).sum()),
               "near_zero_frac": round(float((v32.abs() < 1e-2 * rms).float().mean()), 4)}
        if n.endswith(".1") and n.split(".")[0] in ("enc1", "enc2", "enc3", "enc4"):
            # the MaxPool2d(2) window of this pixel's path: per channel, which of the 4 positions wins
            h0, w0 = (hl // 2) * 2, (wl // 2) * 2
            win32 = torch.relu(a32[b, h0:h0 + 2, w0:w0 + 2]).reshape(4, -1)
            win16 = torch.relu(a16[b, h0:h0 + 2, w0:w0 + 2]).reshape(4, -1)
            row["pool_argmax_flips"] = int((win32.argmax(0) != win16.argmax(0)).sum())
            row["pool_value_dev"] = round(float((win16.max(0).values - win32.max(0).values).abs().max()) / rms, 5)
        rows.append(row)
    return rows


def analyse(m32, m16, x, ref_ac=None, topk=8):
    B, _, H, W = x.shape
    d32, lv32, a32 = _forward(m32, x)
    d16, lv16, a16 = _forward(m16, x)
    dev = (d16 - d32).abs()[:, 0]
    flat = dev.flatten()
    vals, idx = flat.topk(topk)
    top = []
    for v, i in zip(vals.tolist(), idx.tolist()):
        b, r = divmod(i, H * W)
        h, w = divmod(r, W)
        top.append({"b": b, "h": h, "w": w, "dev": round(v, 4), "border_dist": min(h, w, H - 1 - h, W - 1 - w),
                    "disp_fp32": round(float(d32[b, 0, h, w]), 3), "logvar_fp32": round(float(lv32[b, 0, h, w]), 3)})
    out = {"max": round(float(dev.max()), 4), "mean": round(float(dev.mean()), 5),
           "p99_99": round(float(torch.quantile(flat, 0.9999)), 4),
           "frac_over_0.5px": float((dev > 0.5).float().mean()), "top": top}
    if ref_ac is not None:
        d_ref, d_ac = ref_ac
        acd = (d_ac - d_ref).abs()
        out["reference_autocast"] = {"max": round(float(acd.max()), 4), "mean": round(float(acd.mean()), 5),
                                     "p99_99": round(float(torch.quantile(acd.flatten(), 0.9999)), 4)}
        out["fp32_vs_reference_max"] = float((d32 - d_ref).abs().max())
    t0 = top[0]
    out["worst_pixel_trace"] = _layer_trace(a32, a16, B, H, W, t0["b"], t0["h"], t0["w"])
    return out


def main():
    from stereo_depth_estimation_amd.data import synthetic_batch
    from stereo_depth_estimation_amd.model import StereoUNet

    st = dict(np.load(ROOT / "tests/golden/trained_state.npz"))
    ev = np.load(ROOT / "tests/golden/trained_eval.npz")

    def model(prec, state):
        m = StereoUNet(precision=prec)
        m.load_state_dict({k: torch.as_tensor(np.asarray(v)) for k, v in state.items()})
        return m.to(DEV).eval()

    res = {}
    m32, m16 = model("fp32", st), model("bf16", st)
    for name in ("val240", "val720"):
        nb, bsz, h, w = (int(v) for v in ev[f"{name}/shape"])
        b0 = synthetic_batch(bsz, h, w, seed=int(ev[f"{name}/seed"]))
        ref = (torch.as_tensor(ev[f"{name}/fp32/disp0"]), torch.as_tensor(ev[f"{name}/bf16/disp0"]))
        res[name] = analyse(m32, m16, b0["input"].to(DEV), ref)
    if "--bench-model" in sys.argv:
        from stereo_depth_estimation_amd.optim import FusedAdamW
        from stereo_depth_estimation_amd.train import train_step

        torch.manual_seed(42)
        mb = StereoUNet(precision="bf16").to(DEV).train()
        opt = FusedAdamW(mb.parameters(), lr=1e-3, weight_decay=1e-4)
        data = [synthetic_batch(64, 240, 320, seed=50_000 + i, device=DEV) for i in range(16)]  # bench.epe_block's
        for i in range(2000):
            b = data[i % 16]
            train_step(mb, opt, b["input"], b["target"], b["valid_mask"])
        state = {k: v.detach().cpu() for k, v in mb.state_dict().items()}
        val = synthetic_batch(64, 240, 320, seed=90_000)
        res["bench_model"] = analyse(model("fp32", state), model("bf16", state), val["input"].to(DEV))
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
