"""Calibration probe (GPU box): how far the HIP bf16 / fp8 paths drift from the fp32 reference, next to how
far the reference itself drifts under torch.autocast(bf16) on the same inputs. Prints one JSON object; the
bounds in tests/test_gpu_model.py / test_gpu_configs.py are set from these numbers.

    python tools/bf16_drift.py [parts...]     parts: full c4 c5 c2 (default: all)
"""

from __future__ import annotations

import json
import sys
import time
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

from oracle import unet_ref as U  # noqa: E402

DEV = "cuda"
G = ROOT / "tests" / "golden"


def hip_model(state, precision, base=32):
    from stereo_depth_estimation_amd.model import StereoUNet

    m = StereoUNet(base_channels=base, precision=precision)
    m.load_state_dict({k: torch.as_tensor(np.asarray(v)) for k, v in state.items()}, strict=True)
    return m.to(DEV)


def stats(got, ref):
    got, ref = np.asarray(got, np.float64), np.asarray(ref, np.float64)
    d = np.abs(got - ref)
    return {"max": float(d.max()), "mean": float(d.mean()), "rel_max": float((d / (1 + np.abs(ref))).max())}


def hip_step(state, precision, batch):
    """One fused train step: (metrics, grads before AdamW)."""
    from stereo_depth_estimation_amd.optim import FusedAdamW
    from stereo_depth_estimation_amd.train import run_epoch

    m = hip_model(state, precision)
    opt = FusedAdamW(m.parameters(), lr=1e-3, weight_decay=1e-4)
    grads = {}
    orig = opt.fused_step

    def rec(**kw):
        if not grads:
            torch.cuda.synchronize()
            grads.update({k: v.detach().double().norm().item() for k, v in m._grad_views.items()})
        orig(**kw)

    opt.fused_step = rec
    bd = {k: torch.as_tensor(np.asarray(v)).to(DEV) for k, v in batch.items()}
    metrics, _ = run_epoch(m, [bd], torch.device(DEV), optimizer=opt)
    return metrics, grads


def oracle_step(state, batch, autocast=False):
    net = U.Net(state)
    opt = U.AdamWState(net.trainable())
    grads = {}
    orig = opt.step

    def rec(params):
        params = list(params)
        grads.update({k: p.grad.double().norm().item() for k, p in params})
        orig(params)

    opt.step = rec
    with torch.autocast("cpu", dtype=torch.bfloat16, enabled=autocast):
        metrics, _ = U.run_epoch(net, [batch], opt)
    return metrics, grads


def rel(a: dict, b: dict):
    return {k: abs(a[k] - b[k]) / (abs(b[k]) + 1e-12) for k in b}


def part_full(out):
    ac = np.load(G / "full_bf16.npz")
    ev, tr = np.load(G / "full_eval.npz"), np.load(G / "full_train.npz")
    st = U.make_state(32, seed=3)
    m = hip_model(st, "bf16").eval()
    x = torch.as_tensor(U.make_batch(1, 240, 320, seed=4)["input"]).to(DEV)
    with torch.no_grad():
        d, lv = m(x, return_uncertainty=True)
    out["full_eval"] = {"hip_disp": stats(d.cpu(), ev["disp"]), "ac_disp": stats(ac["eval_disp"], ev["disp"]),
                        "hip_logvar": stats(lv.cpu(), ev["logvar"]), "ac_logvar": stats(ac["eval_logvar"], ev["logvar"])}
    b = U.make_batch(2, 240, 320, seed=6)
    m = hip_model(st, "bf16").train()
    with torch.no_grad():
        d, lv = m(torch.as_tensor(b["input"]).to(DEV), return_uncertainty=True)
    out["full_train_fwd"] = {"hip_disp": stats(d.cpu(), tr["train_fwd_disp"]),
                             "ac_disp": stats(ac["train_fwd_disp"], tr["train_fwd_disp"]),
                             "hip_logvar": stats(lv.cpu(), tr["train_fwd_logvar"]),
                             "ac_logvar": stats(ac["train_fwd_logvar"], tr["train_fwd_logvar"])}
    met, gn = hip_step(st, "bf16", b)
    ref_m = {k[8:]: float(tr[k]) for k in tr.files if k.startswith("metrics/")}
    ac_m = {k[8:]: float(ac[k]) for k in ac.files if k.startswith("metrics/")}
    ref_g = {k[6:]: float(tr[k]) for k in tr.files if k.startswith("gnorm/")}
    ac_g = {k[6:]: float(ac[k]) for k in ac.files if k.startswith("gnorm/")}
    out["full_step"] = {"hip_metrics_rel": rel(met, ref_m), "ac_metrics_rel": rel(ac_m, ref_m),
                        "hip_gnorm_rel": rel(gn, ref_g), "ac_gnorm_rel": rel(ac_g, ref_g)}


def part_c4(out):
    st = U.make_state(32, seed=3)
    b = U.make_batch(2, 480, 640, seed=12)
    t0 = time.time()
    ref_m, ref_g = oracle_step(st, b)
    t1 = time.time()
    ac_m, ac_g = oracle_step(st, b, autocast=True)
    t2 = time.time()
    met, gn = hip_step(st, "bf16", b)
    out["c4_step"] = {"hip_metrics_rel": rel(met, ref_m), "ac_metrics_rel": rel(ac_m, ref_m),
                      "hip_gnorm_rel": rel(gn, ref_g), "ac_gnorm_rel": rel(ac_g, ref_g),
                      "oracle_s": t1 - t0, "oracle_ac_s": t2 - t1}


def part_c5(out):
    st = U.make_state(32, seed=3)
    x = U.make_batch(1, 720, 960, seed=13)["input"]
    net = U.Net(st)
    t0 = time.time()
    with torch.no_grad():
        d_ref, lv_ref = net.forward(torch.as_tensor(x), train=False)
        with torch.autocast("cpu", dtype=torch.bfloat16):
            d_ac, lv_ac = net.forward(torch.as_tensor(x), train=False)
    res = {"oracle_s": time.time() - t0, "ac_disp": stats(d_ac.float(), d_ref), "ac_logvar": stats(lv_ac.float(), lv_ref)}
    for prec in ("fp32", "bf16", "fp8"):
        m = hip_model(st, prec).eval()
        with torch.inference_mode():
            d, lv = m(torch.as_tensor(x).to(DEV), return_uncertainty=True)
        res[prec + "_disp"] = stats(d.cpu(), d_ref)
        res[prec + "_logvar"] = stats(lv.cpu(), lv_ref)
    out["c5_eval"] = res


def part_c2(out):
    from stereo_depth_estimation_amd.data import synthetic_batch

    st = U.make_state(32, seed=3)
    b = {k: v.numpy() for k, v in synthetic_batch(64, 240, 320, seed=21).items()}
    met16, g16 = hip_step(st, "bf16", b)
    met32, g32 = hip_step(st, "fp32", b)
    net = U.Net(st)
    t0 = time.time()
    with torch.no_grad():
        d, lv = net.forward(torch.as_tensor(b["input"]), train=True)
        _, sums = U.masked_nll(d, lv, torch.as_tensor(b["target"]), torch.as_tensor(b["valid_mask"]))
    n = sums["n"]
    ref_m = {"nll": sums["nll"] / n, "mae": sums["abs"] / n, "rmse": (sums["sq"] / n) ** 0.5, "sigma": sums["sigma"] / n}
    out["c2_step"] = {"oracle_s": time.time() - t0,
                      "bf16_metrics_rel": rel({k: met16[k] for k in ref_m}, ref_m),
                      "fp32_metrics_rel": rel({k: met32[k] for k in ref_m}, ref_m),
                      "bf16_vs_fp32_gnorm_rel": rel(g16, g32)}


def main():
    torch.set_num_threads(16)
    parts = sys.argv[1:] or ["full", "c4", "c5", "c2"]
    out = {}
    for p in parts:
        t0 = time.time()
        globals()["part_" + p](out)
        print(f"[drift] {p}: {time.time() - t0:.1f}s", file=sys.stderr, flush=True)
    for v in out.values():  # summarise per-tensor dicts: worst 5 + median
        for k in list(v):
            if isinstance(v[k], dict) and len(v[k]) > 10:
                items = sorted(v[k].items(), key=lambda kv: -kv[1])
                v[k] = {"median": float(np.median([x for _, x in items])), "worst": items[:6]}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
