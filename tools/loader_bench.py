"""On-device data path throughput (SURVEY §8f row 1 / BASELINE C4's "async host aug + pinned H2D"): a synthetic
FoundationStereo-layout tree of PNG pairs and its reference-format `.npz` cache, read through
`FoundationStereoDataset` + `DeviceLoader` (worker processes -> pinned uint8 -> side-stream H2D -> HIP decode /
resize / augment), alone and feeding `run_epoch` training. Compare with bench.py's HBM-resident `value`.
    python tools/loader_bench.py [pairs] [H] [W] [batch]
    python tools/loader_bench.py c4 [pairs] [H] [W] [batch]     (BASELINE config 4 per GPU: 640x480, 16 pairs)
Prints one JSON line. Data: random smooth images (no dataset on the box)."""

import json
import os
import sys
import tempfile
import time
from pathlib import Path

import numpy as np
import torch
from PIL import Image

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
from stereo_depth_estimation_amd import dataset as D  # noqa: E402
from stereo_depth_estimation_amd.model import StereoUNet  # noqa: E402
from stereo_depth_estimation_amd.optim import FusedAdamW  # noqa: E402
from stereo_depth_estimation_amd.train import run_epoch  # noqa: E402


def write_tree(root: Path, pairs: int, H: int, W: int, per_scene: int = 64):
    rng = np.random.default_rng(0)
    yy, xx = np.mgrid[0:H, 0:W]
    for i in range(pairs):
        data = root / f"scene{i // per_scene:03d}" / "dataset" / "data"
        for d in ("left/rgb", "right/rgb", "left/disparity"):
            (data / d).mkdir(parents=True, exist_ok=True)
        ph = rng.uniform(0, 6.28, 3)
        base = (127 + 100 * np.sin(xx[..., None] / 17.0 + yy[..., None] / 23.0 + ph)).astype(np.int16)
        left = np.clip(base + rng.integers(-20, 20, (H, W, 3)), 0, 255).astype(np.uint8)
        right = np.roll(left, -8, axis=1)
        drgb = np.stack([np.zeros((H, W)), (xx % 256), (yy % 256)], -1).astype(np.uint8)  # any RGB24 code decodes
        stem = f"{i % per_scene:06d}"
        Image.fromarray(left).save(data / "left/rgb" / f"{stem}.png")
        Image.fromarray(right).save(data / "right/rgb" / f"{stem}.png")
        Image.fromarray(drgb).save(data / "left/disparity" / f"{stem}.png")


def loader_rate(ds, batch, workers, epochs=2, native=False):
    loader = D.DeviceLoader(ds, batch, shuffle=True, num_workers=workers, device="cuda", persistent_workers=True,
                            native=native)
    for b in loader:  # epoch 0: worker start-up, first touch
        pass
    torch.cuda.synchronize()
    t0, n = time.perf_counter(), 0
    for _ in range(epochs):
        for b in loader:
            n += b["input"].shape[0]
    torch.cuda.synchronize()
    return n / (time.perf_counter() - t0)


def train_rate(ds, batch, workers, epochs=2, native=False, read_threads=16):
    torch.manual_seed(42)
    model = StereoUNet(precision="bf16").cuda()
    opt = FusedAdamW(model.parameters(), lr=1e-3, weight_decay=1e-4)
    loader = D.DeviceLoader(ds, batch, shuffle=True, num_workers=workers, device="cuda", persistent_workers=True,
                            drop_last=True, native=native, read_threads=read_threads)
    run_epoch(model, loader, torch.device("cuda"), optimizer=opt)  # warm-up epoch
    torch.cuda.synchronize()
    t0, n = time.perf_counter(), 0
    for _ in range(epochs):
        run_epoch(model, loader, torch.device("cuda"), optimizer=opt)
        n += len(loader) * batch
    torch.cuda.synchronize()
    return n / (time.perf_counter() - t0)


def host_enqueue_ms(batch, H, W, steps=10):
    """Host time to enqueue one HBM-resident train step (the GPU runs behind): the main thread's share of a step."""
    from stereo_depth_estimation_amd.data import synthetic_batch
    from stereo_depth_estimation_amd.train import train_step

    torch.manual_seed(42)
    model = StereoUNet(precision="bf16").cuda()
    opt = FusedAdamW(model.parameters(), lr=1e-3, weight_decay=1e-4)
    b = synthetic_batch(batch, H, W, seed=1, device="cuda")
    for _ in range(3):
        train_step(model, opt, b["input"], b["target"], b["valid_mask"])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        train_step(model, opt, b["input"], b["target"], b["valid_mask"])
    t_host = time.perf_counter() - t0
    torch.cuda.synchronize()
    t_all = time.perf_counter() - t0
    return 1e3 * t_host / steps, 1e3 * t_all / steps


def host_loader_rate(ds, batch, workers, epochs=2):
    """The torch DataLoader alone (workers -> collate -> pinned host batches), no H2D or HIP work."""
    from torch.utils.data import DataLoader

    dl = DataLoader(ds, batch_size=batch, shuffle=True, num_workers=workers, collate_fn=D.collate_uint8,
                    pin_memory=True, persistent_workers=True)
    for _ in dl:
        pass
    t0, n = time.perf_counter(), 0
    for _ in range(epochs):
        for groups in dl:
            n += sum(len(g["index"]) for g in groups)
    return n / (time.perf_counter() - t0)


def resident_rate(batch, H, W, steps=30):
    """bench.py's HBM-resident rate for the same config (a ring of 4 pre-generated device batches)."""
    from stereo_depth_estimation_amd.data import synthetic_batch
    from stereo_depth_estimation_amd.train import train_step

    torch.manual_seed(42)
    model = StereoUNet(precision="bf16").cuda()
    opt = FusedAdamW(model.parameters(), lr=1e-3, weight_decay=1e-4)
    ring = [synthetic_batch(batch, H, W, seed=i, device="cuda") for i in range(4)]
    for i in range(5):
        b = ring[i % 4]
        train_step(model, opt, b["input"], b["target"], b["valid_mask"])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        b = ring[i % 4]
        train_step(model, opt, b["input"], b["target"], b["valid_mask"])
    torch.cuda.synchronize()
    return steps * batch / (time.perf_counter() - t0)


def c4(pairs=256, H=480, W=640, batch=16, epoch_pairs=2048):
    """BASELINE config 4 per GPU (640x480, 16 pairs, async augmentation with pinned H2D overlap): loader-fed training as a
    fraction of the HBM-resident rate, for the reference-format cache (+ augmentation) and PNG (+ augmentation) sources."""
    out = {"config": "C4 per GPU: 640x480, batch 16, bf16", "pairs": pairs, "hw": [H, W], "batch": batch}
    out["resident_pairs_s"] = round(resident_rate(batch, H, W), 1)
    print(f"resident: {out}", file=sys.stderr, flush=True)
    aug = dict(augment=True, brightness_jitter=0.2, contrast_jitter=0.2, saturation_jitter=0.2, hue_jitter=0.05,
               gamma_jitter=0.1, noise_std_max=0.02, blur_prob=0.3, blur_sigma_max=1.0)
    with tempfile.TemporaryDirectory(dir="/tmp") as tmp:
        root, cache = Path(tmp) / "data", Path(tmp) / "cache"
        t0 = time.perf_counter()
        write_tree(root, pairs, H, W)
        samples = D.discover_samples(root)
        png = D.FoundationStereoDataset(samples, image_size=(H, W), cache_root=cache)
        for _ in D.DeviceLoader(png, batch, num_workers=8, device="cuda"):
            pass
        torch.cuda.synchronize()
        out["tree_and_cache_write_s"] = round(time.perf_counter() - t0, 1)
        # epochs of `epoch_pairs` (the files repeated): a training epoch runs thousands of steps, so the per-epoch start
        # (first batch read and copied with nothing to overlap, the end-of-epoch metric read) must not weigh more than it
        # does there
        samples = samples * max(1, epoch_pairs // len(samples))
        out["epoch_pairs"] = len(samples)
        print(f"tree + cache: {out}", file=sys.stderr, flush=True)
        arms = {"cache_aug_native": (D.FoundationStereoDataset(samples, image_size=(H, W), cache_root=cache,
                                                               require_cache=True, **aug), 0, True),
                "cache_native": (D.FoundationStereoDataset(samples, image_size=(H, W), cache_root=cache,
                                                           require_cache=True), 0, True),
                "png_aug_native": (D.FoundationStereoDataset(samples, image_size=(H, W), **aug), 0, True),
                "png_aug_w16": (D.FoundationStereoDataset(samples, image_size=(H, W), **aug), 16, False)}
        if os.environ.get("SD_C4_TRACE"):  # one arm only, for a kernel / memory-copy trace of loader-fed training
            arm = os.environ["SD_C4_TRACE"]
            ds, workers, native = arms[arm]
            out[f"train_{arm}_pairs_s"] = round(train_rate(ds, batch, workers, native=native, epochs=2), 1)
            print(json.dumps(out), flush=True)
            return
        if os.environ.get("SD_C4_SIDE_AB"):  # prep kernels before the step (default) vs beside it, alternating
            ds = arms["cache_aug_native"][0]
            for rnd in range(2):
                for side in ("0", "1"):
                    os.environ["SD_LOADER_PREP_SIDE"] = side
                    out[f"ab_side{side}_r{rnd}_pairs_s"] = round(train_rate(ds, batch, 0, native=True, epochs=2), 1)
            os.environ["SD_LOADER_PREP_SIDE"] = "0"
            print(json.dumps(out), flush=True)
            return
        if os.environ.get("SD_C4_EXPERIMENTS"):  # where the cache+aug arm loses time (A/B arms, one process)
            ds = arms["cache_aug_native"][0]
            out["loader_only_cache_aug_native_pairs_s"] = round(loader_rate(ds, batch, 0, native=True), 1)
            for rt in (4, 8):
                out[f"train_cache_aug_native_t{rt}_pairs_s"] = round(train_rate(ds, batch, 0, native=True, epochs=3,
                                                                                 read_threads=rt), 1)
            hi = torch.cuda.Stream(priority=-1)
            with torch.cuda.stream(hi):
                out["train_cache_aug_native_hiprio_pairs_s"] = round(train_rate(ds, batch, 0, native=True, epochs=3), 1)
            print(f"experiments: {out}", file=sys.stderr, flush=True)
        for name, (ds, workers, native) in arms.items():
            r = train_rate(ds, batch, workers, native=native, epochs=2)
            out[f"train_{name}_pairs_s"] = round(r, 1)
            out[f"train_{name}_frac_of_resident"] = round(r / out["resident_pairs_s"], 3)
            print(f"{name}: {out}", file=sys.stderr, flush=True)
    print(json.dumps(out), flush=True)


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "c4":
        c4(*(int(a) for a in sys.argv[2:]))
        return
    pairs = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    H = int(sys.argv[2]) if len(sys.argv) > 2 else 240
    W = int(sys.argv[3]) if len(sys.argv) > 3 else 320
    batch = int(sys.argv[4]) if len(sys.argv) > 4 else 64
    out = {"pairs": pairs, "hw": [H, W], "batch": batch}
    quick = len(sys.argv) > 5 and sys.argv[5] == "quick"  # native training arm only (A/B runs)
    with tempfile.TemporaryDirectory(dir="/tmp") as tmp:
        root, cache = Path(tmp) / "data", Path(tmp) / "cache"
        t0 = time.perf_counter()
        write_tree(root, pairs, H, W)
        samples = D.discover_samples(root)
        out["tree_write_s"] = round(time.perf_counter() - t0, 1)
        # the first pass writes the reference-format cache (uint8 RGB, f16 disparity)
        png = D.FoundationStereoDataset(samples, image_size=(H, W), cache_root=cache)
        for _ in D.DeviceLoader(png, batch, num_workers=8, device="cuda"):
            pass
        torch.cuda.synchronize()
        cached = D.FoundationStereoDataset(samples, image_size=(H, W), cache_root=cache, require_cache=True)
        png_aug = D.FoundationStereoDataset(samples, image_size=(H, W), augment=True, brightness_jitter=0.2,
                                            contrast_jitter=0.2, saturation_jitter=0.2, hue_jitter=0.05,
                                            gamma_jitter=0.1, noise_std_max=0.02, blur_prob=0.3, blur_sigma_max=1.0)
        print(f"tree + cache written: {time.perf_counter() - t0:.1f}s", file=sys.stderr, flush=True)
        if quick:
            out["train_cache_native_t16_pairs_s"] = round(train_rate(cached, batch, 0, native=True, epochs=4), 1)
            print(json.dumps(out), flush=True)
            return
        out["host_enqueue_ms_per_step"], out["gpu_ms_per_step"] = (round(v, 2) for v in host_enqueue_ms(batch, H, W))
        out["host_dataloader_cache_w16_pairs_s"] = round(host_loader_rate(cached, batch, 16), 1)
        print(f"host: {out}", file=sys.stderr, flush=True)
        for w in (8, 16):
            out[f"loader_cache_w{w}_pairs_s"] = round(loader_rate(cached, batch, w), 1)
            out[f"loader_png_aug_w{w}_pairs_s"] = round(loader_rate(png_aug, batch, w), 1)
            print(f"loaders w={w}: {out}", file=sys.stderr, flush=True)
        cached_aug = D.FoundationStereoDataset(samples, image_size=(H, W), cache_root=cache, require_cache=True,
                                               augment=True, brightness_jitter=0.2, contrast_jitter=0.2,
                                               saturation_jitter=0.2, hue_jitter=0.05, gamma_jitter=0.1,
                                               noise_std_max=0.02, blur_prob=0.3, blur_sigma_max=1.0)
        out["loader_cache_aug_native_t16_pairs_s"] = round(loader_rate(cached_aug, batch, 0, native=True), 1)
        out["train_cache_aug_native_t16_pairs_s"] = round(train_rate(cached_aug, batch, 0, native=True), 1)
        out["loader_png_aug_native_t16_pairs_s"] = round(loader_rate(png_aug, batch, 0, native=True), 1)
        out["train_png_aug_native_t16_pairs_s"] = round(train_rate(png_aug, batch, 0, native=True), 1)
        out["loader_cache_native_t16_pairs_s"] = round(loader_rate(cached, batch, 0, native=True), 1)
        out["train_cache_native_t16_pairs_s"] = round(train_rate(cached, batch, 0, native=True), 1)
        print(f"native: {out}", file=sys.stderr, flush=True)
        out["train_cache_w16_pairs_s"] = round(train_rate(cached, batch, 16), 1)
        print(f"train cache: {out}", file=sys.stderr, flush=True)
        out["train_png_aug_w16_pairs_s"] = round(train_rate(png_aug, batch, 16), 1)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
