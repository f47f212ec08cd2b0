"""Data path of the HIP trainer: the reference's dataset API with the tensor work on the GPU.

Mirror of reference ``dataset.py`` (``StereoSample``, ``discover_samples``,
``sample_cache_relpath``, ``FoundationStereoDataset`` with the same constructor, validation
errors and cache layout) and ``eval_utils.split_samples``. What moves:

* DataLoader workers only decode image files to **uint8** (PIL, as the reference) and, when
  augmenting, sample the per-image jitter factors with torch's CPU generator in the
  reference's order (``dataset.py:214-270``);
* :class:`DeviceLoader` collates uint8, copies pinned batches host->HBM asynchronously on a side
  stream and runs ``sd_stereo_preprocess`` / ``sd_stereo_from_cache`` (decode, /255, bilinear
  resize, disparity width scaling, valid mask: ``dataset.py:184-212,305-311``) and
  ``sd_augment_rgb`` (``dataset.py:248-270``) there, yielding the reference's batch dict
  ``{"input" [B,6,H,W] f32, "target" [B,1,H,W] f32, "valid_mask" [B,1,H,W] bool}`` on the device.

Differences a user sees: items of :class:`FoundationStereoDataset` are uint8 arrays, not float
tensors (iterate them through :class:`DeviceLoader`); the
additive noise field is drawn on the GPU (same distribution, not the same numbers as torch's CPU
generator), and the factors sampled after a noisy image therefore continue from a different
generator state than the reference's.
"""

from __future__ import annotations

import ctypes
import hashlib
import os
import random
from concurrent.futures import ThreadPoolExecutor
from dataclasses import dataclass
from pathlib import Path
from typing import Iterable

import numpy as np
import torch
from PIL import Image
from torch.utils.data import DataLoader, Dataset

from . import _lib as L

AUG_PARAMS = 7  # brightness, contrast, saturation, hue shift, gamma, blur sigma (0 = off), noise std


@dataclass(frozen=True)
class StereoSample:
    left_rgb_path: Path
    right_rgb_path: Path
    disparity_path: Path


def _resolve_frame_path(frame_dir: Path, stem: str) -> Path | None:
    for ext in (".jpg", ".jpeg", ".png"):
        candidate = frame_dir / f"{stem}{ext}"
        if candidate.exists():
            return candidate
    return None


def discover_samples(dataset_root: str | Path) -> list[StereoSample]:
    """FoundationStereo layout ``<scene>/dataset/data/{left,right}/rgb`` + ``left/disparity/*.png``
    (reference ``dataset.py:41-65``): scenes sorted, disparity PNGs sorted, frames without both
    RGB images skipped."""
    root = Path(dataset_root).expanduser().resolve()
    if not root.exists():
        raise FileNotFoundError(f"Dataset root does not exist: {root}")
    samples: list[StereoSample] = []
    for scene_dir in sorted(p for p in root.iterdir() if p.is_dir()):
        data = scene_dir / "dataset" / "data"
        left_dir, right_dir, disp_dir = data / "left" / "rgb", data / "right" / "rgb", data / "left" / "disparity"
        if not (left_dir.exists() and right_dir.exists() and disp_dir.exists()):
            continue
        for disparity_path in sorted(disp_dir.glob("*.png")):
            left = _resolve_frame_path(left_dir, disparity_path.stem)
            right = _resolve_frame_path(right_dir, disparity_path.stem)
            if left is None or right is None:
                continue
            samples.append(StereoSample(left, right, disparity_path))
    return samples


def sample_cache_relpath(sample: StereoSample) -> Path:
    """Cache file of a sample relative to the cache root (reference ``dataset.py:68-83``)."""
    parts = sample.left_rgb_path.parts
    if "dataset" in parts:
        i = parts.index("dataset")
        if i > 0:
            return Path(parts[i - 1]) / f"{sample.disparity_path.stem}.npz"
    key = f"{sample.left_rgb_path.as_posix()}|{sample.right_rgb_path.as_posix()}|{sample.disparity_path.as_posix()}"
    digest = hashlib.blake2s(key.encode("utf-8"), digest_size=8).hexdigest()
    return Path("misc") / f"{sample.disparity_path.stem}_{digest}.npz"


def split_samples(samples, val_fraction: float, seed: int, require_non_empty_train: bool = True):
    """Seeded shuffle, tail as validation (reference ``eval_utils.py:14-39``)."""
    if not 0.0 <= val_fraction < 1.0:
        raise ValueError(f"--val-fraction must be in [0, 1), got: {val_fraction}")
    shuffled = list(samples)
    random.Random(seed).shuffle(shuffled)
    if val_fraction == 0.0:
        return shuffled, []
    val_count = max(int(len(shuffled) * val_fraction), 1)
    if require_non_empty_train and val_count >= len(shuffled):
        raise ValueError("Validation set consumes all data. Reduce --val-fraction or provide more samples.")
    val_count = min(val_count, len(shuffled))
    return shuffled[:-val_count], shuffled[-val_count:]


def read_rgb_uint8(path: Path) -> np.ndarray:
    """HWC uint8, as ``np.array(Image.open(path).convert("RGB"))`` in the reference."""
    with Image.open(path) as im:
        return np.array(im.convert("RGB"), dtype=np.uint8)


def _load_cached_uint8(cache_file: Path, image_size: tuple[int, int]):
    """``load_cached_sample`` (reference ``dataset.py:86-105``) without the float conversion."""
    with np.load(cache_file) as cached:
        if not {"left", "right", "disparity"}.issubset(cached.files):
            return None
        left, right, disp = cached["left"], cached["right"], cached["disparity"]
    if left.ndim != 3 or right.ndim != 3 or disp.ndim != 2:
        return None
    if left.shape[:2] != image_size or right.shape[:2] != image_size or disp.shape != image_size:
        return None
    return left.astype(np.uint8, copy=False), right.astype(np.uint8, copy=False), disp.astype(np.float16, copy=False)


class FoundationStereoDataset(Dataset):
    """Same constructor, validation and cache behaviour as the reference (``dataset.py:131-311``);
    items are uint8 (plus sampled augmentation factors) for :class:`DeviceLoader`."""

    def __init__(
        self,
        samples: Iterable[StereoSample],
        image_size: tuple[int, int] = (240, 320),
        augment: bool = False,
        brightness_jitter: float = 0.0,
        contrast_jitter: float = 0.0,
        saturation_jitter: float = 0.0,
        hue_jitter: float = 0.0,
        gamma_jitter: float = 0.0,
        noise_std_max: float = 0.0,
        blur_prob: float = 0.0,
        blur_sigma_max: float = 0.0,
        blur_kernel_size: int = 5,
        cache_root: str | Path | None = None,
        require_cache: bool = False,
    ) -> None:
        self.samples = list(samples)
        self.image_size = tuple(image_size)
        self.augment = augment
        self.brightness_jitter = brightness_jitter
        self.contrast_jitter = contrast_jitter
        self.saturation_jitter = saturation_jitter
        self.hue_jitter = hue_jitter
        self.gamma_jitter = gamma_jitter
        self.noise_std_max = noise_std_max
        self.blur_prob = blur_prob
        self.blur_sigma_max = blur_sigma_max
        self.blur_kernel_size = blur_kernel_size
        self.cache_root = Path(cache_root).expanduser().resolve() if cache_root is not None else None
        self.require_cache = require_cache
        if not 0.0 <= self.blur_prob <= 1.0:
            raise ValueError(f"blur_prob must be in [0, 1], got {self.blur_prob}")
        if self.blur_kernel_size < 3 or self.blur_kernel_size % 2 == 0:
            raise ValueError(f"blur_kernel_size must be odd and >= 3, got {self.blur_kernel_size}")
        if self.saturation_jitter < 0.0:
            raise ValueError(f"saturation_jitter must be >= 0, got {self.saturation_jitter}")
        if self.gamma_jitter < 0.0:
            raise ValueError(f"gamma_jitter must be >= 0, got {self.gamma_jitter}")
        if len(self.samples) == 0:
            raise ValueError("No samples were provided.")

    def __len__(self) -> int:
        return len(self.samples)

    # --- augmentation factors: same generator calls, same order as dataset.py:214-270 ---------
    def _sample_jitter_factor(self, jitter: float) -> float:
        if jitter <= 0.0:
            return 1.0
        return float(torch.empty(1).uniform_(max(0.0, 1.0 - jitter), 1.0 + jitter).item())

    def _sample_hue_shift(self) -> float:
        if self.hue_jitter <= 0.0:
            return 0.0
        return float(torch.empty(1).uniform_(-self.hue_jitter, self.hue_jitter).item())

    def _sample_gamma_factor(self) -> float:
        if self.gamma_jitter <= 0.0:
            return 1.0
        low = max(0.1, 1.0 - self.gamma_jitter)
        return float(torch.empty(1).uniform_(low, max(low, 1.0 + self.gamma_jitter)).item())

    def _sample_noise_std(self) -> float:
        if self.noise_std_max <= 0.0:
            return 0.0
        return float(torch.empty(1).uniform_(0.0, self.noise_std_max).item())

    def _should_apply_blur(self) -> bool:
        if self.blur_prob <= 0.0 or self.blur_sigma_max <= 0.0:
            return False
        return bool(torch.rand(1).item() < self.blur_prob)

    def _sample_blur_sigma(self) -> float:
        return float(torch.empty(1).uniform_(0.1, max(self.blur_sigma_max, 0.1)).item())

    def sample_augment_params(self) -> np.ndarray:
        """Factors of one ``_augment_rgb`` call: [brightness, contrast, saturation, hue, gamma,
        blur sigma (0 = none), noise std]. Raises as torchvision would for an invalid hue shift."""
        b = self._sample_jitter_factor(self.brightness_jitter)
        c = self._sample_jitter_factor(self.contrast_jitter)
        s = self._sample_jitter_factor(self.saturation_jitter)
        h = self._sample_hue_shift()
        if not -0.5 <= h <= 0.5:
            raise ValueError(f"hue_factor ({h}) is not in [-0.5, 0.5].")
        g = self._sample_gamma_factor()
        sigma = self._sample_blur_sigma() if self._should_apply_blur() else 0.0
        n = self._sample_noise_std()
        return np.array([b, c, s, h, g, sigma, n], dtype=np.float32)

    def __getitem__(self, index: int) -> dict:
        sample = self.samples[index]
        item: dict = {"cache_file": ""}
        if self.cache_root is not None:
            cache_file = self.cache_root / sample_cache_relpath(sample)
            if cache_file.exists():
                loaded = _load_cached_uint8(cache_file, self.image_size)
                if loaded is not None:
                    item.update(kind=1, left=loaded[0], right=loaded[1], disparity=loaded[2])
                elif self.require_cache:
                    raise ValueError(f"Cache entry is invalid or shape-mismatched for sample: {cache_file}")
            elif self.require_cache:
                raise FileNotFoundError(f"Required cache entry not found: {cache_file}")
            if "kind" not in item:
                item["cache_file"] = str(cache_file)  # DeviceLoader writes it after preprocessing
        if "kind" not in item:
            item.update(kind=0, left=read_rgb_uint8(sample.left_rgb_path), right=read_rgb_uint8(sample.right_rgb_path),
                        disparity=read_rgb_uint8(sample.disparity_path))
            if not (item["left"].shape == item["right"].shape == item["disparity"].shape):
                raise ValueError(f"left/right/disparity sizes differ for sample {sample.disparity_path}")
        if self.augment:
            item["aug"] = np.stack([self.sample_augment_params(), self.sample_augment_params()])
        return item


def collate_uint8(items: list[dict]) -> list[dict]:
    """Stack items into homogeneous groups (same kind and source size), keeping batch positions."""
    groups: dict[tuple, list[int]] = {}
    for i, it in enumerate(items):
        groups.setdefault((it["kind"],) + tuple(it["left"].shape), []).append(i)
    out = []
    for (kind, *shape), idx in groups.items():
        g = {
            "kind": kind,
            "index": torch.tensor(idx, dtype=torch.int64),
            "left": torch.from_numpy(np.stack([items[i]["left"] for i in idx])),
            "right": torch.from_numpy(np.stack([items[i]["right"] for i in idx])),
            "disparity": torch.from_numpy(np.stack([items[i]["disparity"] for i in idx])),
            "cache_file": [items[i]["cache_file"] for i in idx],
        }
        if kind == 1:
            g["disparity"] = g["disparity"].view(torch.int16)  # f16 bits; pinned transfer as 2-byte words
        if "aug" in items[idx[0]]:
            g["aug"] = torch.from_numpy(np.stack([items[i]["aug"] for i in idx]))
        out.append(g)
    return out


def _pin(t: torch.Tensor) -> torch.Tensor:
    return t if t.is_pinned() else t.pin_memory()


def save_cached_sample(cache_file: Path, left: np.ndarray, right: np.ndarray, target: np.ndarray) -> None:
    """Reference cache format (``dataset.py:108-128``): uint8 HWC of clip(x*255), f16 disparity."""
    lnp = np.clip(left.transpose(1, 2, 0) * 255.0, 0, 255).astype(np.uint8)
    rnp = np.clip(right.transpose(1, 2, 0) * 255.0, 0, 255).astype(np.uint8)
    cache_file.parent.mkdir(parents=True, exist_ok=True)
    np.savez(cache_file, left=lnp, right=rnp, disparity=target[0].astype(np.float16))


def read_cache_batch(paths, image_size: tuple[int, int], left: torch.Tensor, right: torch.Tensor, disparity: torch.Tensor,
                     threads: int = 16) -> None:
    """Native (``sd_read_cache_batch``) read of reference-format cache files (``load_cached_sample``, reference
    ``dataset.py:86-105``) into host tensors: left/right uint8 [n,H,W,3], disparity int16 [n,H,W] (the f16 bits).
    A host thread pool inside the call, the GIL released (ctypes); no worker processes, no pickling."""
    H, W = image_size
    n = len(paths)
    for t, shape, dt in ((left, (n, H, W, 3), torch.uint8), (right, (n, H, W, 3), torch.uint8),
                         (disparity, (n, H, W), torch.int16)):
        if tuple(t.shape) != shape or t.dtype != dt or not t.is_contiguous() or t.device.type != "cpu":
            raise ValueError(f"read_cache_batch: expected a contiguous CPU {dt} tensor of {shape}, got {t.dtype} "
                             f"{tuple(t.shape)}")
    arr = (ctypes.c_char_p * max(n, 1))(*[os.fsencode(str(p)) for p in paths])
    err = ctypes.create_string_buffer(1024)
    rc = L.load().sd_read_cache_batch(ctypes.cast(arr, ctypes.c_void_p), n, H, W, left.data_ptr(), right.data_ptr(),
                                      disparity.data_ptr(), threads, err, len(err))
    if rc != 0:
        msg = err.value.decode(errors="replace")
        if rc > 0 and not Path(paths[rc - 1]).exists():
            raise FileNotFoundError(f"Required cache entry not found: {msg}")
        raise ValueError(f"Cache entry is invalid or shape-mismatched: {msg}")


def read_png_batch(paths, size: tuple[int, int], out: torch.Tensor, threads: int = 16) -> bool:
    """Native (``sd_read_png_batch``) decode of n PNG frames of one source size into a uint8 [n,H,W,3] host tensor,
    as ``read_rgb_uint8`` (PIL ``convert("RGB")``) returns them. False when a file is not an 8-bit RGB/RGBA,
    non-interlaced PNG of that size (the caller reads that batch with PIL); missing files raise."""
    H, W = size
    n = len(paths)
    if tuple(out.shape) != (n, H, W, 3) or out.dtype != torch.uint8 or not out.is_contiguous():
        raise ValueError(f"read_png_batch: expected a contiguous uint8 tensor of {(n, H, W, 3)}")
    arr = (ctypes.c_char_p * max(n, 1))(*[os.fsencode(str(p)) for p in paths])
    err = ctypes.create_string_buffer(1024)
    rc = L.load().sd_read_png_batch(ctypes.cast(arr, ctypes.c_void_p), n, H, W, out.data_ptr(), threads, err, len(err))
    if rc > 0 and not Path(paths[rc - 1]).exists():
        raise FileNotFoundError(err.value.decode(errors="replace"))
    return rc == 0


def png_size(path) -> tuple[int, int] | None:
    """(H, W) from a PNG's IHDR, None if it is not a PNG."""
    h, w = ctypes.c_int(0), ctypes.c_int(0)
    rc = L.load().sd_png_size(os.fsencode(str(path)), ctypes.addressof(h), ctypes.addressof(w))
    return (h.value, w.value) if rc == 0 else None


class DeviceLoader:
    """Iterates device batch dicts ``{"input","target","valid_mask"}`` for ``run_epoch``.

    Wraps a ``torch.utils.data.DataLoader`` over a :class:`FoundationStereoDataset` (uint8
    collate, pinned memory, the reference's worker options). Each host batch is copied to the
    device on a side HIP stream (DMA engines) and turned into the reference's tensors there by the
    HIP kernels, beside the training step of the batch before it; the consumer's stream waits on
    an event.
    """

    def __init__(self, dataset: FoundationStereoDataset, batch_size: int, shuffle: bool = False, num_workers: int = 0,
                 device: torch.device | str = "cuda", drop_last: bool = False, persistent_workers: bool = False,
                 generator: torch.Generator | None = None, sampler=None, native: bool | None = None,
                 read_threads: int = 16):
        """native: read batches with the in-process native cache reader (``read_cache_batch``) instead of DataLoader
        worker processes; without a cache_root (native=True only), PNG frames decoded by ``read_png_batch``. Default
        (None): on for datasets served entirely from the cache (require_cache). Same batch
        order (the DataLoader's own batch sampler) and bytes; augmentation factors are drawn in the main process in
        the order of a num_workers=0 DataLoader (worker processes draw them from per-worker RNG streams instead)."""
        self.dataset = dataset
        if native is None:
            native = dataset.cache_root is not None and dataset.require_cache
        if native and dataset.cache_root is not None and not dataset.require_cache:
            raise ValueError("DeviceLoader(native=True) serves a cache_root dataset only with require_cache "
                             "(the worker path writes cache misses)")
        self.native, self.read_threads = native, read_threads
        self.device = torch.device(device)
        if self.device.type != "cuda":
            raise RuntimeError(f"DeviceLoader prepares batches with HIP kernels; got device {self.device}")
        self.loader = DataLoader(dataset, batch_size=batch_size, shuffle=shuffle if sampler is None else False,
                                 sampler=sampler, num_workers=num_workers, collate_fn=collate_uint8, pin_memory=True,
                                 drop_last=drop_last, persistent_workers=persistent_workers and num_workers > 0,
                                 generator=generator)
        self._stream = None
        self._batches = 0
        self._seed_drawn = False
        # the decode / augment kernels on the side stream beside the previous step (default), or on the consumer's
        # stream right before the step (SD_LOADER_PREP_SIDE=0): 640x480 B=16 loader-fed training 1634 vs 1615 pairs/s
        self._prep_side = os.environ.get("SD_LOADER_PREP_SIDE", "1") == "1"

    def __len__(self) -> int:
        return len(self.loader)

    def _upload(self, groups: list[dict]) -> list[dict]:
        """Side stream: the pinned uint8 frames (and augmentation factors) of a host batch to the device. The copies run
        on the DMA engines; the seeds of the augmentation noise are drawn here, in batch order."""
        dev = self.device
        staged = []
        for g in groups:
            n = len(g["index"])
            st = {"g": g, "left": _pin(g["left"]).to(dev, non_blocking=True),
                  "right": _pin(g["right"]).to(dev, non_blocking=True),
                  "disparity": _pin(g["disparity"]).to(dev, non_blocking=True)}
            if "aug" in g:
                st["params"] = _pin(g["aug"].reshape(n * 2, AUG_PARAMS).contiguous()).to(dev, non_blocking=True)
                st["seed"] = int(torch.randint(0, 2**62, (1,)).item())
            staged.append(st)
        return staged

    def _finish(self, staged, ev, consumer) -> dict:
        if isinstance(staged, dict):  # prepared on the side stream (SD_LOADER_PREP_SIDE=1)
            consumer.wait_event(ev)
            for t in staged.values():
                t.record_stream(consumer)
            return staged
        return self._kernels(staged, ev, consumer)

    def _kernels(self, staged: list[dict], ev, consumer) -> dict:
        """Decode / resize / augment the uploaded uint8 frames into the reference's tensors on stream `consumer` (the
        side stream by default, after the copies; ev = None) or on the training stream after the copy event."""
        L.load()
        if ev is not None:
            consumer.wait_event(ev)
        H, W = self.dataset.image_size
        B = sum(len(st["g"]["index"]) for st in staged)
        dev = self.device
        s = L.stream_handle(dev)
        inp = torch.empty(B, 6, H, W, device=dev)
        tgt = torch.empty(B, 1, H, W, device=dev)
        val = torch.empty(B, 1, H, W, device=dev, dtype=torch.bool)
        for st in staged:
            g = st["g"]
            for k in ("left", "right", "disparity", "params"):
                if k in st:
                    st[k].record_stream(consumer)
            left, right, disp = st["left"], st["right"], st["disparity"]
            n = len(g["index"])
            contiguous = bool((g["index"] == torch.arange(g["index"][0], g["index"][0] + n)).all())
            gi = inp[g["index"][0]:g["index"][0] + n] if contiguous else torch.empty(n, 6, H, W, device=dev)
            gt = tgt[g["index"][0]:g["index"][0] + n] if contiguous else torch.empty(n, 1, H, W, device=dev)
            gv = val[g["index"][0]:g["index"][0] + n] if contiguous else torch.empty(n, 1, H, W, device=dev, dtype=torch.bool)
            if g["kind"] == 0:
                Hs, Ws = g["left"].shape[1:3]
                L.call("sd_stereo_preprocess", left.data_ptr(), right.data_ptr(), disp.data_ptr(), n, Hs, Ws, H, W,
                       gi.data_ptr(), gt.data_ptr(), gv.data_ptr(), s)
            else:
                L.call("sd_stereo_from_cache", left.data_ptr(), right.data_ptr(), disp.data_ptr(), n, H, W,
                       gi.data_ptr(), gt.data_ptr(), gv.data_ptr(), s)
            if any(g["cache_file"]):
                # the cache holds the un-augmented sample (the reference saves before _augment_rgb,
                # dataset.py:297-303): write it now (first epoch with a cache root; synchronises)
                gi_h, gt_h = gi.cpu().numpy(), gt.cpu().numpy()
                for k, f in enumerate(g["cache_file"]):
                    if f:
                        save_cached_sample(Path(f), gi_h[k, :3], gi_h[k, 3:], gt_h[k])
            if "params" in st:
                work = torch.empty(n * 6 * H * W + 128 * n, device=dev)
                L.call("sd_augment_rgb", gi.data_ptr(), n, H, W, st["params"].data_ptr(), self.dataset.blur_kernel_size,
                       st["seed"], work.data_ptr(), s)
            if not contiguous:
                inp[g["index"].to(dev)] = gi
                tgt[g["index"].to(dev)] = gt
                val[g["index"].to(dev)] = gv
        return {"input": inp, "target": tgt, "valid_mask": val}

    def _native_groups(self):
        """Host batches from the native reader, in collate_uint8's format: a one-thread executor reads batch i+1 into
        one of two pinned buffer sets while batch i is copied and prepared; a set is refilled only after the
        event of its last H2D copy (recorded by __iter__ in self._h2d_done) has completed."""
        H, W = self.dataset.image_size
        root, samples = self.dataset.cache_root, self.dataset.samples
        bmax = self.loader.batch_size

        def alloc():
            return (torch.empty(bmax, H, W, 3, dtype=torch.uint8).pin_memory(),
                    torch.empty(bmax, H, W, 3, dtype=torch.uint8).pin_memory(),
                    torch.empty(bmax, H, W, dtype=torch.int16).pin_memory())

        bufs = [alloc(), alloc()] if root is not None else [None, None]
        self._h2d_done = [None, None]

        def read_png(idxs):  # frames of the un-cached source (pinned by torch's caching host allocator)
            """collate_uint8's groups: one per source frame size, in order of first occurrence in the batch."""
            sm = [samples[i] for i in idxs]
            attrs = ("left_rgb_path", "right_rgb_path", "disparity_path")
            by_size: dict = {}
            for j, x in enumerate(sm):
                by_size.setdefault(png_size(x.left_rgb_path), []).append(j)
            parts = []  # (batch positions, left, right, disparity)
            for hw, pos in by_size.items():
                outs = []
                for attr in attrs if hw is not None else ():
                    t = torch.empty(len(pos), *hw, 3, dtype=torch.uint8, pin_memory=True)
                    if not read_png_batch([getattr(sm[j], attr) for j in pos], hw, t, self.read_threads):
                        break
                    outs.append(t)
                if len(outs) == 3:
                    parts.append((pos, *outs))
                    continue
                # PIL for these frames (not 8-bit RGB/RGBA PNGs), regrouped by their decoded size
                dec: dict = {}
                for j in pos:
                    f = [read_rgb_uint8(getattr(sm[j], a)) for a in attrs]
                    if not (f[0].shape == f[1].shape == f[2].shape):
                        raise ValueError(f"left/right/disparity sizes differ for sample {sm[j].disparity_path}")
                    dec.setdefault(f[0].shape, []).append((j, f))
                for items in dec.values():
                    parts.append(([j for j, _ in items], *(torch.from_numpy(np.stack([f[a] for _, f in items]))
                                                            .pin_memory() for a in range(3))))
            first = {}
            for pos, left, right, disp in parts:  # merge same-size parts, keeping first-occurrence order
                if not (left.shape == right.shape == disp.shape):
                    raise ValueError(f"left/right/disparity sizes differ in the batch of {sm[pos[0]].disparity_path}")
                first.setdefault(tuple(left.shape[1:]), []).append((pos, left, right, disp))
            groups = []
            for ps in sorted(first.values(), key=lambda ps: min(min(p[0]) for p in ps)):
                pos = [j for p in ps for j in p[0]]
                order = sorted(range(len(pos)), key=lambda i: pos[i])
                cat = [torch.cat([p[k] for p in ps])[order] if len(ps) > 1 else ps[0][k] for k in (1, 2, 3)]
                groups.append({"kind": 0, "index": torch.tensor(sorted(pos), dtype=torch.int64), "left": cat[0],
                               "right": cat[1], "disparity": cat[2], "cache_file": [""] * len(pos)})
            return groups

        def read(k, idxs):
            if root is None:
                return read_png(idxs)
            n = len(idxs)
            left, right, disp = (t[:n] for t in bufs[k])
            read_cache_batch([root / sample_cache_relpath(samples[i]) for i in idxs], (H, W), left, right, disp,
                             self.read_threads)
            return [{"kind": 1, "index": torch.arange(n), "left": left, "right": right, "disparity": disp,
                     "cache_file": [""] * n}]

        with ThreadPoolExecutor(1) as ex:
            # a DataLoader iterator draws its workers' base seed from the generator (or the global RNG) before the
            # sampler's permutation: the same draw keeps the shuffle order, and the RNG stream after it, identical.
            # A persistent-workers DataLoader draws it once, when it first creates its iterator (_reset draws no more)
            if not (self.loader.persistent_workers and self._seed_drawn):
                torch.empty((), dtype=torch.int64).random_(generator=self.loader.generator)
                self._seed_drawn = True
            it = iter(self.loader.batch_sampler)
            nxt = next(it, None)
            fut = ex.submit(read, 0, nxt) if nxt is not None else None
            k = 0
            while fut is not None:
                gs = fut.result()
                nxt = next(it, None)
                fut = None
                if nxt is not None:
                    if self._h2d_done[k ^ 1] is not None:
                        self._h2d_done[k ^ 1].synchronize()
                    fut = ex.submit(read, k ^ 1, nxt)
                if self.dataset.augment:
                    # drawn here, as batch k is handed over, so the main-process RNG sees the order of a
                    # num_workers=0 DataLoader: factors of batch k (per item in batch order, in __getitem__'s calls),
                    # then the noise seeds _upload draws for batch k's groups, then batch k+1's factors
                    ds = self.dataset
                    n = sum(len(g["index"]) for g in gs)
                    aug = np.stack([np.stack([ds.sample_augment_params(), ds.sample_augment_params()]) for _ in range(n)])
                    for g in gs:
                        g["aug"] = torch.from_numpy(aug[g["index"].numpy()])
                self._slot = k
                yield gs
                k ^= 1

    def __iter__(self):
        if self._stream is None:
            self._stream = torch.cuda.Stream(self.device)
        consumer = torch.cuda.current_stream(self.device)
        pending = None
        for groups in (self._native_groups() if self.native else self.loader):
            self._stream.wait_stream(consumer)  # reuse of freed buffers is ordered after their last use
            with torch.cuda.stream(self._stream):
                staged = self._upload(groups)
                if self._prep_side:  # A/B: the kernels beside the step instead of before it
                    staged = self._kernels(staged, None, self._stream)
                ev = torch.cuda.Event()
                ev.record(self._stream)
            if self.native:
                self._h2d_done[self._slot] = ev  # the pinned set may be refilled once its copies are done
            if pending is not None:
                yield self._finish(*pending, consumer)
            pending = (staged, ev)
        if pending is not None:
            yield self._finish(*pending, consumer)
