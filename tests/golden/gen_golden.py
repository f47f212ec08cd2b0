"""Generate the committed golden fixtures by running the REFERENCE itself (build container only).

Usage (from the repo root, in the container that has /root/reference):
    PYTHONDONTWRITEBYTECODE=1 python tests/golden/gen_golden.py

The reference (read-only, ``/root/reference/src``) is imported with inert stubs for
the two absent third-party modules: ``torchvision`` (only the
augmentation path uses it; goldens use ``augment=False``) and ``mlflow``
(``log_metrics`` no-op).  Weights and inputs come from the build's documented
numpy PCG64 recipes (``oracle.unet_ref.make_state`` / ``make_batch``) so the GPU
box can regenerate the inputs without the reference.  Only data (inputs and
expected outputs) is written; no reference source is copied.
"""

from __future__ import annotations

import copy
import sys
import tempfile
import types
from pathlib import Path

import numpy as np
import torch

REPO = Path(__file__).resolve().parents[2]
sys.path.insert(0, str(REPO))
sys.dont_write_bytecode = True
sys.path.insert(0, "/root/reference/src")

_tv = types.ModuleType("torchvision")
_tvt = types.ModuleType("torchvision.transforms")
_tvf = types.ModuleType("torchvision.transforms.functional")
_tv.transforms = _tvt
_tvt.functional = _tvf
_ml = types.ModuleType("mlflow")
_ml.log_metrics = lambda *a, **k: None
sys.modules.update({"torchvision": _tv, "torchvision.transforms": _tvt, "torchvision.transforms.functional": _tvf, "mlflow": _ml})

from foundation_stereo_depth import dataset as ref_dataset  # noqa: E402
from foundation_stereo_depth import eval_utils as ref_eval  # noqa: E402
from foundation_stereo_depth import model as ref_model  # noqa: E402
from foundation_stereo_depth import train as ref_train  # noqa: E402

from oracle.data_ref import encode_disparity_to_rgb  # noqa: E402
from oracle.unet_ref import TRAINABLE_KINDS, make_batch, make_state, param_spec  # noqa: E402

OUT = Path(__file__).resolve().parent


def build_ref(base, state):
    torch.manual_seed(0)
    m = ref_model.StereoUNet(in_channels=6, out_channels=1, base_channels=base)
    m.load_state_dict({k: torch.as_tensor(v) for k, v in state.items()}, strict=True)
    return m


def batch_to_torch(b):
    return {k: torch.as_tensor(v) for k, v in b.items()}


class RecordingAdamW(torch.optim.AdamW):
    """The reference's optimizer (train.py:578) that snapshots grads before each step."""

    def __init__(self, params, names, **kw):
        super().__init__(params, **kw)
        self.names = names
        self.grads = []

    def step(self, closure=None):
        self.grads.append({n: p.grad.detach().clone() for n, p in self.names})
        return super().step(closure)


def trainable_named(m):
    named = dict(m.named_parameters())
    return [(k, named[k]) for k, _, kind in param_spec(base_channels=m.enc1.block[0].out_channels) if kind in TRAINABLE_KINDS]


def gen_tiny():
    base, B, H, W = 8, 2, 32, 48
    state = make_state(base, seed=0, signed_gamma=True)
    b1 = make_batch(B, H, W, seed=1)
    b2 = make_batch(B, H, W, seed=2)
    out = {}
    # train-mode forward (BN batch stats) on a copy, and eval-mode forward
    m = build_ref(base, state)
    mc = copy.deepcopy(m).train()
    with torch.no_grad():
        d, lv = mc(torch.as_tensor(b1["input"]), return_uncertainty=True)
    out["train_fwd_disp"], out["train_fwd_logvar"] = d.numpy(), lv.numpy()
    me = copy.deepcopy(m).eval()
    with torch.no_grad():
        d, lv = me(torch.as_tensor(b1["input"]), return_uncertainty=True)
        d_only = me(torch.as_tensor(b1["input"]))
    out["eval_disp"], out["eval_logvar"] = d.numpy(), lv.numpy()
    assert torch.equal(d, d_only)
    # two reference train steps through the reference run_epoch (train.py:292-418)
    names = trainable_named(m)
    opt = RecordingAdamW([p for _, p in names], names, lr=1e-3, weight_decay=1e-4)
    metrics, gstep = ref_train.run_epoch(m, [batch_to_torch(b1), batch_to_torch(b2)], torch.device("cpu"), optimizer=opt, global_step=0, log_every_batches=10)
    assert gstep == 2 and len(opt.grads) == 2
    for k, g in opt.grads[0].items():
        out["grad1/" + k] = g.numpy()
    sd = m.state_dict()
    for k, _, kind in param_spec(base_channels=base):
        if kind in TRAINABLE_KINDS:
            out["delta2/" + k] = (sd[k].numpy() - state[k]).astype(np.float32)
        else:
            out["buf2/" + k] = sd[k].numpy()
    for k, v in metrics.items():
        out["metrics/" + k] = np.float64(v)
    # val epoch after training (eval-mode BN, no optimizer) on batch 1
    vmetrics, _ = ref_train.run_epoch(m, [batch_to_torch(b1)], torch.device("cpu"), optimizer=None)
    for k, v in vmetrics.items():
        out["val_metrics/" + k] = np.float64(v)
    np.savez_compressed(OUT / "tiny_train.npz", **out)

    # zero-valid batch is skipped after zero_grad (train.py:325-332)
    m = build_ref(base, state)
    names = trainable_named(m)
    opt = RecordingAdamW([p for _, p in names], names, lr=1e-3, weight_decay=1e-4)
    bz = make_batch(B, H, W, seed=5)
    bz["target"][:] = 0.0
    bz["valid_mask"][:] = False
    metrics, gstep = ref_train.run_epoch(m, [batch_to_torch(bz), batch_to_torch(b1)], torch.device("cpu"), optimizer=opt, global_step=0)
    skip = {"metrics/" + k: np.float64(v) for k, v in metrics.items()}
    skip["global_step"] = np.int64(gstep)
    skip["n_steps"] = np.int64(len(opt.grads))
    sd = m.state_dict()
    for k in ("enc1.block.0.weight", "up1.bias", "logvar_head.bias", "enc1.block.1.running_mean"):
        skip["after/" + k] = sd[k].numpy()
    np.savez_compressed(OUT / "tiny_skip.npz", **skip)


def gen_full():
    base = 32
    state = make_state(base, seed=3)
    m = build_ref(base, state).eval()
    b = make_batch(1, 240, 320, seed=4)
    with torch.no_grad():
        d, lv = m(torch.as_tensor(b["input"]), return_uncertainty=True)
    np.savez_compressed(OUT / "full_eval.npz", disp=d.numpy(), logvar=lv.numpy())

    # full-size train step: outputs, metrics and per-tensor gradient checksums
    m = build_ref(base, state)
    b = make_batch(2, 240, 320, seed=6)
    mc = copy.deepcopy(m).train()
    with torch.no_grad():
        d, lv = mc(torch.as_tensor(b["input"]), return_uncertainty=True)
    names = trainable_named(m)
    opt = RecordingAdamW([p for _, p in names], names, lr=1e-3, weight_decay=1e-4)
    metrics, _ = ref_train.run_epoch(m, [batch_to_torch(b)], torch.device("cpu"), optimizer=opt, global_step=0)
    out = {"train_fwd_disp": d.numpy(), "train_fwd_logvar": lv.numpy()}
    for k, v in metrics.items():
        out["metrics/" + k] = np.float64(v)
    for k, g in opt.grads[0].items():
        g64 = g.double()
        out["gsum/" + k] = np.float64(g64.sum().item())
        out["gnorm/" + k] = np.float64(g64.norm().item())
    np.savez_compressed(OUT / "full_train.npz", **out)


def gen_data():
    from PIL import Image

    out = {}
    # reference test vector (tests/test_dataset.py:31-35)
    disp = np.array([[0.0, 0.125, 1.25], [2.0, 3.5, 10.0]], dtype=np.float32)
    enc = encode_disparity_to_rgb(disp)
    out["codec_rgb"] = enc
    out["codec_decoded"] = ref_dataset.depth_uint8_decoding(enc)
    rng = np.random.Generator(np.random.PCG64(11))
    with tempfile.TemporaryDirectory() as td:
        root = Path(td) / "fs"
        for scene in ("sceneA", "sceneB"):
            for sub in ("left/rgb", "right/rgb", "left/disparity"):
                (root / scene / "dataset" / "data" / sub).mkdir(parents=True)
        k = 0
        for scene in ("sceneA", "sceneB"):
            for stem in ("000000", "000001"):
                left = rng.integers(0, 256, size=(45, 61, 3), dtype=np.uint8)
                right = rng.integers(0, 256, size=(45, 61, 3), dtype=np.uint8)
                dd = rng.uniform(0.0, 40.0, size=(45, 61)).astype(np.float32)
                dd[rng.random(dd.shape) < 0.1] = 0.0
                drgb = encode_disparity_to_rgb(dd)
                base = root / scene / "dataset" / "data"
                Image.fromarray(left, "RGB").save(base / "left/rgb" / f"{stem}.png")
                Image.fromarray(right, "RGB").save(base / "right/rgb" / f"{stem}.png")
                Image.fromarray(drgb, "RGB").save(base / "left/disparity" / f"{stem}.png")
                out[f"src{k}_left"], out[f"src{k}_right"], out[f"src{k}_disp_rgb"] = left, right, drgb
                k += 1
        samples = ref_dataset.discover_samples(root)
        assert len(samples) == 4
        ds = ref_dataset.FoundationStereoDataset(samples, image_size=(24, 32), augment=False)
        for i in range(len(ds)):
            item = ds[i]
            out[f"item{i}_input"] = item["input"].numpy()
            out[f"item{i}_target"] = item["target"].numpy()
            out[f"item{i}_valid"] = item["valid_mask"].numpy()
    for n in (10, 64):
        tr, va = ref_eval.split_samples(list(range(n)), 0.1, 42)
        out[f"split{n}_train"], out[f"split{n}_val"] = np.array(tr), np.array(va)
    np.savez_compressed(OUT / "data_path.npz", **out)


def gen_bf16():
    """The reference's own bf16 behaviour: the same full-size forwards and train step as
    gen_full, run under torch.autocast("cpu", dtype=torch.bfloat16). The drift of these outputs from the fp32
    ones is the yardstick the HIP bf16 path's bounds are calibrated to (tests/test_gpu_model.py)."""
    base = 32
    state = make_state(base, seed=3)
    out = {}
    m = build_ref(base, state).eval()
    b = make_batch(1, 240, 320, seed=4)
    with torch.no_grad(), torch.autocast("cpu", dtype=torch.bfloat16):
        d, lv = m(torch.as_tensor(b["input"]), return_uncertainty=True)
    out["eval_disp"], out["eval_logvar"] = d.float().numpy(), lv.float().numpy()
    m = build_ref(base, state)
    b = make_batch(2, 240, 320, seed=6)
    mc = copy.deepcopy(m).train()
    with torch.no_grad(), torch.autocast("cpu", dtype=torch.bfloat16):
        d, lv = mc(torch.as_tensor(b["input"]), return_uncertainty=True)
    out["train_fwd_disp"], out["train_fwd_logvar"] = d.float().numpy(), lv.float().numpy()
    names = trainable_named(m)
    opt = RecordingAdamW([p for _, p in names], names, lr=1e-3, weight_decay=1e-4)
    with torch.autocast("cpu", dtype=torch.bfloat16):
        metrics, _ = ref_train.run_epoch(m, [batch_to_torch(b)], torch.device("cpu"), optimizer=opt, global_step=0)
    for k, v in metrics.items():
        out["metrics/" + k] = np.float64(v)
    for k, g in opt.grads[0].items():
        out["gnorm/" + k] = np.float64(g.double().norm().item())
    np.savez_compressed(OUT / "full_bf16.npz", **out)


if __name__ == "__main__":
    torch.set_num_threads(8)
    parts = sys.argv[1:] or ["data", "tiny", "full", "bf16"]
    for part in parts:
        {"data": gen_data, "tiny": gen_tiny, "full": gen_full, "bf16": gen_bf16}[part]()
    for p in sorted(OUT.glob("*.npz")):
        print(p.name, p.stat().st_size)
