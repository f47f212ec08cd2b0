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


TRAINED_STEPS, TRAINED_B, TRAINED_LR = 600, 4, 5e-3
# held-out evaluation sets of the trained checkpoint: (name, batches, batch size, H, W, first seed of synthetic_batch on
# the CPU, batches whose output maps are stored); EPE over all batches (the validation epoch's mean)
TRAINED_EVAL = (("val240", 4, 4, 240, 320, 90_001, 1), ("val720", 2, 1, 720, 960, 90_101, 1))


def _synthetic(batch, h, w, seed):
    from stereo_depth_estimation_amd.data import synthetic_batch

    return {k: v.numpy() for k, v in synthetic_batch(batch, h, w, seed=seed).items()}


def _input_digest(b):
    """sha256 of a synthetic batch's bytes: the GPU box regenerates the batch from its seed and checks this before
    trusting the stored outputs (same torch CPU generator and kernels, same image)."""
    import hashlib

    h = hashlib.sha256()
    for k in ("input", "target", "valid_mask"):
        h.update(np.ascontiguousarray(b[k]).tobytes())
    return np.array(h.hexdigest())


def gen_trained():
    """A reference-TRAINED base-32 checkpoint: the reference's own run_epoch (train.py:292-418)
    with its AdamW (train.py:578, --lr 5e-3) trains StereoUNet from the make_state(seed=3) weights for TRAINED_STEPS
    steps on fresh synthetic rectified pairs (stereo_depth_estimation_amd.data.synthetic_batch, the bench's SURVEY
    §8d recipe) at 240x320, batch TRAINED_B. Written: the state_dict (trained_state.npz) and, per held-out set of
    TRAINED_EVAL, the reference's eval-mode validation (train.py:301: eval BN, no optimizer) in fp32 and under
    torch.autocast("cpu", bfloat16): metrics (EPE = `mae`, train.py:350,406), disparity and logvar maps, and the
    input checksums (trained_eval.npz). ~4 min on 8 cores."""
    import time

    base = 32
    m = build_ref(base, make_state(base, seed=3)).train()
    names = trainable_named(m)
    opt = torch.optim.AdamW([p for _, p in names], lr=TRAINED_LR, weight_decay=1e-4)
    t0 = time.time()
    for i in range(TRAINED_STEPS):
        b = batch_to_torch(_synthetic(TRAINED_B, 240, 320, seed=60_000 + i))
        metrics, _ = ref_train.run_epoch(m, [b], torch.device("cpu"), optimizer=opt, global_step=i)
        if i % 50 == 0 or i == TRAINED_STEPS - 1:
            print(f"step {i}: mae {metrics['mae']:.3f} nll {metrics['nll']:.3f} ({time.time() - t0:.0f}s)", flush=True)
    sd = m.state_dict()
    np.savez_compressed(OUT / "trained_state.npz", **{k: v.numpy() for k, v in sd.items()})
    out = {"train/steps": np.int64(TRAINED_STEPS), "train/batch": np.int64(TRAINED_B), "train/lr": np.float64(TRAINED_LR)}
    for name, nb, bsz, h, w, seed, nmaps in TRAINED_EVAL:
        bs = [_synthetic(bsz, h, w, seed + i) for i in range(nb)]
        out[f"{name}/seed"], out[f"{name}/shape"] = np.int64(seed), np.array([nb, bsz, h, w])
        out[f"{name}/digest"] = np.array([_input_digest(b) for b in bs])
        for tag, ac in (("fp32", False), ("bf16", True)):
            me = copy.deepcopy(m).eval()
            with torch.no_grad(), torch.autocast("cpu", dtype=torch.bfloat16, enabled=ac):
                for i in range(nmaps):
                    d, lv = me(torch.as_tensor(bs[i]["input"]), return_uncertainty=True)
                    out[f"{name}/{tag}/disp{i}"], out[f"{name}/{tag}/logvar{i}"] = d.float().numpy(), lv.float().numpy()
                vm, _ = ref_train.run_epoch(me, [batch_to_torch(b) for b in bs], torch.device("cpu"), optimizer=None)
            for k, v in vm.items():
                out[f"{name}/{tag}/metrics/{k}"] = np.float64(v)
            print(f"{name} {tag}: {vm}", flush=True)
    np.savez_compressed(OUT / "trained_eval.npz", **out)


# BASELINE configs' per-GPU train steps: (name, batch, H, W, synthetic_batch seed)
CONFIG_STEPS = (("c2", 64, 240, 320, 21), ("c4", 16, 480, 640, 22))


def gen_configs():
    """One reference train step (run_epoch, train.py:292-418, AdamW lr 1e-3) at BASELINE config 2's per-GPU batch
    (64 x 320x240) and config 4's (16 x 640x480), from make_state(32, seed=3), in fp32 and under
    torch.autocast("cpu", bfloat16): metrics and per-tensor gradient norms / sums, plus the input digest
    (configs_steps.npz). ~15 GB of host memory per step."""
    import time

    out = {}
    state = make_state(32, seed=3)
    for name, bsz, h, w, seed in CONFIG_STEPS:
        b = _synthetic(bsz, h, w, seed)
        out[f"{name}/seed"], out[f"{name}/shape"] = np.int64(seed), np.array([bsz, h, w])
        out[f"{name}/digest"] = _input_digest(b)
        for tag, ac in (("fp32", False), ("bf16", True)):
            t0 = time.time()
            m = build_ref(32, state)
            names = trainable_named(m)
            opt = RecordingAdamW([p for _, p in names], names, lr=1e-3, weight_decay=1e-4)
            with torch.autocast("cpu", dtype=torch.bfloat16, enabled=ac):
                metrics, _ = ref_train.run_epoch(m, [batch_to_torch(b)], torch.device("cpu"), optimizer=opt)
            for k, v in metrics.items():
                out[f"{name}/{tag}/metrics/{k}"] = np.float64(v)
            for k, g in opt.grads[0].items():
                out[f"{name}/{tag}/gnorm/{k}"] = np.float64(g.double().norm().item())
                out[f"{name}/{tag}/gsum/{k}"] = np.float64(g.double().sum().item())
            print(f"{name} {tag}: {metrics} ({time.time() - t0:.0f}s)", flush=True)
            del m, opt
    np.savez_compressed(OUT / "configs_steps.npz", **out)


if __name__ == "__main__":
    torch.set_num_threads(8)
    parts = sys.argv[1:] or ["data", "tiny", "full", "bf16"]
    for part in parts:
        {"data": gen_data, "tiny": gen_tiny, "full": gen_full, "bf16": gen_bf16, "trained": gen_trained,
         "configs": gen_configs}[part]()
    for p in sorted(OUT.glob("*.npz")):
        print(p.name, p.stat().st_size)
