"""Training CLI of the HIP path — mirror of reference ``train.py:main`` (``train.py:60-212,480-690``).

    python -m stereo_depth_estimation_amd.cli --dataset-root DIR [reference flags] [--resume last.pt]
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 -m stereo_depth_estimation_amd.cli ...

Same flags, defaults, seeding, sample split, datasets, epoch loop, metrics keys and checkpoint
files (``checkpoints/last.pt`` every epoch, ``best.pt`` on the lowest val MAE) with the reference's
checkpoint dict ``{"epoch", "model_state_dict", "optimizer_state_dict", "args", "metrics"}``
(``train.py:421-436``), so checkpoints load in the reference's live app and through
``load_state_dict_compat``. Differences:

* batches come from :class:`~stereo_depth_estimation_amd.dataset.DeviceLoader` (uint8 H2D,
  decode/resize/augment on the GPU);
* ``--resume CKPT`` (new) restores model, AdamW state, epoch, global step,
  best metric and the RNG states saved with each checkpoint (extra keys the reference ignores),
  so a resumed run continues exactly where the saved one was: weights, AdamW moments, step,
  shuffle order and the GPU noise seeds. One exception: with ``--num-workers > 0`` and
  ``--augment``, the jitter factors are drawn in the persistent worker processes, whose RNG
  restarts in a resumed run (same distribution, different draws). Checkpoints are read with
  ``torch.load(weights_only=True)``: everything in them is tensors and plain Python values;
* with ``WORLD_SIZE > 1`` (torchrun) samples are sharded across ranks and gradients are summed
  over RCCL (``ddp.DataParallel``); rank 0 writes checkpoints and logs;
* MLflow is used when importable; otherwise metrics go to ``<run dir>/metrics.jsonl``;
* ``--device cpu`` and ``--compile`` are rejected: there is no CPU path and no tracing compiler
  (the reference's CPU path is the parity oracle in ``oracle/``); epoch previews are not written.
"""

from __future__ import annotations

import argparse
import json
import os
import random
import time
from dataclasses import asdict, dataclass
from pathlib import Path

import numpy as np
import torch

from .dataset import DeviceLoader, FoundationStereoDataset, discover_samples, split_samples
from .model import StereoUNet
from .optim import FusedAdamW
from .train import MLFLOW_TRAIN_LOG_EVERY_BATCHES, run_epoch


@dataclass
class TrainConfig:  # reference train.py:38-58, plus the HIP path's options at the end
    dataset_root: str
    height: int
    width: int
    epochs: int
    batch_size: int
    lr: float
    weight_decay: float
    num_workers: int
    val_fraction: float
    max_samples: int
    seed: int
    device: str
    mlflow_tracking_uri: str
    mlflow_experiment: str
    run_name: str | None
    output_dir: str
    cache_root: str | None
    require_cache: bool
    compile: bool
    compile_mode: str
    compile_backend: str
    augment: bool
    brightness_jitter: float
    contrast_jitter: float
    saturation_jitter: float
    hue_jitter: float
    gamma_jitter: float
    noise_std_max: float
    blur_prob: float
    blur_sigma_max: float
    blur_kernel_size: int
    resume: str | None = None
    precision: str = "fp32"
    sync_bn: bool = False


def build_parser() -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(description="Train stereo disparity model on FoundationStereo (MI355X HIP path).")
    p.add_argument("--dataset-root", type=str, default="/mnt/bulk2/NVidia Foundation Stereo")
    p.add_argument("--height", type=int, default=240)
    p.add_argument("--width", type=int, default=320)
    p.add_argument("--epochs", type=int, default=100)
    p.add_argument("--batch-size", type=int, default=30)
    p.add_argument("--lr", type=float, default=1e-3)
    p.add_argument("--weight-decay", type=float, default=1e-4)
    p.add_argument("--num-workers", type=int, default=4)
    p.add_argument("--val-fraction", type=float, default=0.1)
    p.add_argument("--max-samples", type=int, default=0)
    p.add_argument("--seed", type=int, default=42)
    p.add_argument("--device", type=str, default="auto")
    p.add_argument("--mlflow-tracking-uri", type=str, default="sqlite:///mlflow.db")
    p.add_argument("--mlflow-experiment", type=str, default="foundation-stereo-depth")
    p.add_argument("--run-name", type=str, default=None)
    p.add_argument("--output-dir", type=str, default="./outputs")
    p.add_argument("--cache-root", type=str, default=None)
    p.add_argument("--require-cache", action="store_true")
    p.add_argument("--compile", action=argparse.BooleanOptionalAction, default=False)
    p.add_argument("--compile-mode", type=str, default="default", choices=("default", "reduce-overhead", "max-autotune"))
    p.add_argument("--compile-backend", type=str, default="inductor")
    p.add_argument("--augment", action="store_true")
    p.add_argument("--brightness-jitter", type=float, default=0.0)
    p.add_argument("--contrast-jitter", type=float, default=0.0)
    p.add_argument("--saturation-jitter", type=float, default=0.0)
    p.add_argument("--hue-jitter", type=float, default=0.0)
    p.add_argument("--gamma-jitter", type=float, default=0.0)
    p.add_argument("--noise-std-max", type=float, default=0.0)
    p.add_argument("--blur-prob", type=float, default=0.0)
    p.add_argument("--blur-sigma-max", type=float, default=0.0)
    p.add_argument("--blur-kernel-size", type=int, default=5)
    p.add_argument("--resume", type=str, default=None, help="Checkpoint (last.pt) to continue from.")
    p.add_argument("--precision", type=str, default="fp32", choices=("bf16", "fp32"),
                   help="fp32: the reference's arithmetic (default); bf16: opt-in fast path (bf16 activations, fp32 accumulation)")
    p.add_argument("--sync-bn", action="store_true",
                   help="multi-GPU: BatchNorm statistics over the global batch (SyncBatchNorm) instead of per rank")
    return p


def parse_args(argv=None) -> TrainConfig:
    return TrainConfig(**vars(build_parser().parse_args(argv)))


def set_seed(seed: int) -> None:  # train.py:215-220
    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)
    if torch.cuda.is_available():
        torch.cuda.manual_seed_all(seed)


def resolve_device(device_arg: str, local_rank: int) -> torch.device:
    if device_arg == "auto":
        if not torch.cuda.is_available():
            raise RuntimeError("No HIP device: this trainer runs only on MI355X (no CPU path).")
        return torch.device("cuda", local_rank)
    dev = torch.device(device_arg)
    if dev.type != "cuda":
        raise RuntimeError(f"--device {device_arg}: this trainer runs only on a HIP device (no CPU path).")
    return dev


# ---------------------------------------------------------------- RNG state as tensors / plain values
def rng_state() -> dict:
    ver, mt, gauss = random.getstate()
    np_name, np_keys, np_pos, np_has_gauss, np_gauss = np.random.get_state()
    return {
        "python": [ver, list(mt), gauss],
        "numpy": {"name": np_name, "keys": torch.from_numpy(np_keys.astype(np.int64)), "pos": int(np_pos),
                  "has_gauss": int(np_has_gauss), "cached_gaussian": float(np_gauss)},
        "torch": torch.get_rng_state(),
        "cuda": torch.cuda.get_rng_state_all() if torch.cuda.is_available() else [],
    }


def set_rng_state(st: dict) -> None:
    ver, mt, gauss = st["python"]
    random.setstate((ver, tuple(mt), gauss))
    n = st["numpy"]
    np.random.set_state((n["name"], n["keys"].numpy().astype(np.uint32), n["pos"], n["has_gauss"],
                         n["cached_gaussian"]))
    torch.set_rng_state(st["torch"])
    if st.get("cuda") and torch.cuda.is_available():
        torch.cuda.set_rng_state_all(st["cuda"])


def save_checkpoint(checkpoint_path: Path, epoch: int, model: StereoUNet, optimizer: FusedAdamW, args: TrainConfig,
                    metrics: dict[str, float], *, global_step: int = 0, best_val_mae: float = float("inf"),
                    best_epoch: int = -1) -> None:
    """The reference's checkpoint dict (train.py:421-436) plus resume state under extra keys."""
    checkpoint = {
        "epoch": epoch,
        "model_state_dict": model.state_dict(),
        "optimizer_state_dict": optimizer.state_dict(),
        "args": asdict(args),
        "metrics": metrics,
        "global_step": global_step,
        "best_val_mae": best_val_mae,
        "best_epoch": best_epoch,
        "rng_state": rng_state(),
    }
    tmp = checkpoint_path.with_suffix(checkpoint_path.suffix + ".tmp")
    torch.save(checkpoint, tmp)
    os.replace(tmp, checkpoint_path)  # never leave a torn last.pt behind


def load_checkpoint(path: str | Path, model: StereoUNet, optimizer: FusedAdamW | None, device) -> dict:
    """Restore a checkpoint written by :func:`save_checkpoint` (or by the reference: model and
    optimizer only; the RNG / global-step keys are then absent). Safe loader only."""
    ck = torch.load(path, map_location="cpu", weights_only=True)
    model.load_state_dict(ck["model_state_dict"])
    model.to(device)
    if optimizer is not None and "optimizer_state_dict" in ck:
        optimizer.load_state_dict(ck["optimizer_state_dict"])
    if "rng_state" in ck:
        set_rng_state(ck["rng_state"])
    return ck


class _JsonlLogger:
    def __init__(self, path: Path):
        self.path = path

    def log_metrics(self, metrics, step=None):
        with open(self.path, "a") as f:
            f.write(json.dumps({"step": step, **metrics}) + "\n")


class _NullLogger:
    def log_metrics(self, metrics, step=None):
        pass


def _epoch_metrics(train_metrics, val_metrics, seconds):
    m = {f"train_{k}": train_metrics[k] for k in ("loss", "nll", "mae", "rmse", "sigma")}
    m["epoch_seconds"] = seconds
    if val_metrics is not None:
        m.update({f"val_{k}": val_metrics[k] for k in ("loss", "nll", "mae", "rmse", "sigma")})
    return m


def main(argv=None) -> dict:
    args = parse_args(argv)
    if args.compile:
        raise RuntimeError("--compile: the HIP path has no tracing compiler (north star); drop the flag.")
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    device = resolve_device(args.device, local_rank)
    torch.cuda.set_device(device)
    ddp = None
    if world > 1:
        import torch.distributed as dist

        from .ddp import DataParallel, ShardSampler

        os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        if not dist.is_initialized():
            dist.init_process_group("nccl", device_id=device)
    set_seed(args.seed)
    if rank == 0:
        print(f"Using device: {device} (world size {world})")

    all_samples = discover_samples(args.dataset_root)
    if args.max_samples > 0:
        all_samples = all_samples[: args.max_samples]
    if len(all_samples) < 2:
        raise ValueError("Need at least two samples to create train/validation splits.")
    train_samples, val_samples = split_samples(all_samples, args.val_fraction, args.seed)
    if rank == 0:
        print(f"Discovered {len(all_samples)} samples: train={len(train_samples)}, val={len(val_samples)}")
    image_size = (args.height, args.width)
    train_ds = FoundationStereoDataset(
        train_samples, image_size=image_size, augment=args.augment, brightness_jitter=args.brightness_jitter,
        contrast_jitter=args.contrast_jitter, saturation_jitter=args.saturation_jitter, hue_jitter=args.hue_jitter,
        gamma_jitter=args.gamma_jitter, noise_std_max=args.noise_std_max, blur_prob=args.blur_prob,
        blur_sigma_max=args.blur_sigma_max, blur_kernel_size=args.blur_kernel_size, cache_root=args.cache_root,
        require_cache=args.require_cache)
    val_ds = (FoundationStereoDataset(val_samples, image_size=image_size, cache_root=args.cache_root,
                                      require_cache=args.require_cache) if val_samples else None)
    sampler = val_sampler = None
    if world > 1:
        from torch.utils.data.distributed import DistributedSampler

        sampler = DistributedSampler(train_ds, num_replicas=world, rank=rank, shuffle=True, seed=args.seed)
        if val_ds is not None:  # exact shards: no padded duplicates in the summed val metrics (best.pt selection)
            val_sampler = ShardSampler(len(val_ds), world, rank)
    persistent = args.num_workers > 0
    loader_gen = None
    if persistent:
        # The worker base seed is drawn once per process (when the persistent iterator is created): from
        # its own generator, so the main-process RNG stream (shuffle order, GPU noise seeds) is the same
        # in a resumed run as in the run it continues. The shuffle keeps the reference's source, the
        # global RNG (a DataLoader generator would also drive the sampler).
        loader_gen = torch.Generator().manual_seed(args.seed)
        if sampler is None:
            sampler = torch.utils.data.RandomSampler(train_ds)
    train_loader = DeviceLoader(train_ds, args.batch_size, shuffle=True, num_workers=args.num_workers, device=device,
                                persistent_workers=persistent, sampler=sampler, generator=loader_gen)
    val_loader = (DeviceLoader(val_ds, args.batch_size, shuffle=False, num_workers=args.num_workers, device=device,
                               persistent_workers=persistent, sampler=val_sampler) if val_ds is not None else None)

    model = StereoUNet(in_channels=6, out_channels=1, precision=args.precision).to(device)
    optimizer = FusedAdamW(model.parameters(), lr=args.lr, weight_decay=args.weight_decay)
    start_epoch, global_step, best_val_mae, best_epoch = 1, 0, float("inf"), -1
    if args.resume:
        ck = load_checkpoint(args.resume, model, optimizer, device)
        start_epoch = int(ck["epoch"]) + 1
        global_step = int(ck.get("global_step", (start_epoch - 1) * len(train_loader)))
        best_val_mae = float(ck.get("best_val_mae", float("inf")))
        best_epoch = int(ck.get("best_epoch", -1))
        if rank == 0:
            print(f"Resumed from {args.resume}: epoch {start_epoch - 1}, global step {global_step}")
    if world > 1:
        ddp = DataParallel(model, sync_bn=args.sync_bn)

    # run directory and logger (MLflow when available, else JSON lines)
    logger, run_ctx, run_id = _NullLogger(), None, args.run_name or time.strftime("run-%Y%m%d-%H%M%S")
    mlflow = None
    if rank == 0:
        try:
            import mlflow  # noqa: F811

            mlflow.set_tracking_uri(args.mlflow_tracking_uri)
            mlflow.set_experiment(args.mlflow_experiment)
            run_ctx = mlflow.start_run(run_name=args.run_name)
            run_id = mlflow.active_run().info.run_id
            logger = mlflow
        except ImportError:
            mlflow = None
    if args.resume:
        output_dir = Path(args.resume).expanduser().resolve().parent.parent  # keep writing into the same run
    else:
        output_dir = Path(args.output_dir).expanduser().resolve() / run_id
    checkpoints_dir = output_dir / "checkpoints"
    if rank == 0:
        checkpoints_dir.mkdir(parents=True, exist_ok=True)
        (output_dir / "config.json").write_text(json.dumps(asdict(args), indent=2), encoding="utf-8")
        if mlflow is None:
            logger = _JsonlLogger(output_dir / "metrics.jsonl")

    history = []
    try:
        for epoch in range(start_epoch, args.epochs + 1):
            if hasattr(sampler, "set_epoch"):
                sampler.set_epoch(epoch)
            t0 = time.time()
            train_metrics, global_step = run_epoch(model, train_loader, device, optimizer=optimizer,
                                                   global_step=global_step,
                                                   log_every_batches=MLFLOW_TRAIN_LOG_EVERY_BATCHES,
                                                   logger=logger, ddp=ddp)
            if ddp is not None:  # evaluate and checkpoint with rank 0's BN running statistics on every rank
                ddp.sync_buffers()
            val_metrics = run_epoch(model, val_loader, device, optimizer=None, ddp=ddp)[0] if val_loader else None
            metrics = _epoch_metrics(train_metrics, val_metrics, time.time() - t0)
            candidate = (val_metrics or train_metrics)["mae"]
            improved = candidate < best_val_mae
            if improved:
                best_val_mae, best_epoch = candidate, epoch
            if rank == 0:
                logger.log_metrics(metrics, step=epoch)
                kw = dict(global_step=global_step, best_val_mae=best_val_mae, best_epoch=best_epoch)
                save_checkpoint(checkpoints_dir / "last.pt", epoch, model, optimizer, args, metrics, **kw)
                if improved:
                    save_checkpoint(checkpoints_dir / "best.pt", epoch, model, optimizer, args, metrics, **kw)
                vm = f", val_mae={val_metrics['mae']:.4f}" if val_metrics else ""
                print(f"Epoch {epoch}/{args.epochs}: train_mae={train_metrics['mae']:.4f}{vm}, "
                      f"train_rmse={train_metrics['rmse']:.4f}")
            history.append(metrics)
    finally:
        if run_ctx is not None:
            mlflow.set_tag("best_epoch", best_epoch)
            mlflow.set_tag("best_val_mae", best_val_mae)
            mlflow.end_run()
    if rank == 0:
        print(f"Best validation MAE: {best_val_mae:.4f} at epoch {best_epoch}")
        print(f"Checkpoints saved to: {checkpoints_dir}")
    return {"history": history, "best_val_mae": best_val_mae, "best_epoch": best_epoch, "output_dir": str(output_dir),
            "global_step": global_step}


if __name__ == "__main__":
    main()
