"""Training step and epoch loop of the HIP path — mirror of reference ``train.py:292-418``.

``run_epoch(model, loader, device, optimizer=None, global_step=0, log_every_batches=None)``
keeps the reference's signature, batch-dict contract ({"input","target","valid_mask"},
dataset.py:305-311), metrics dict ({"loss","nll","mae","rmse","sigma"}), MLflow step keys
and the ``RuntimeError("No valid target pixels found for this epoch.")``.

What changes is underneath: one fused HIP train step per batch (forward with BN-stat
epilogues -> heads + masked NLL + its gradient -> hand-scheduled backward -> AdamW) with
no host synchronisation; metric sums accumulate on the device in fp64 and are read once
per MLflow log interval and once per epoch, instead of ~10 ``.item()`` per batch.
The zero-valid batch skip (train.py:331-332) is a device-side gate on the AdamW kernel.
"""

from __future__ import annotations

import math
from typing import Callable

import torch

from . import _lib as L
from .model import StereoUNet
from .optim import FusedAdamW

MLFLOW_TRAIN_LOG_EVERY_BATCHES = 10


class _NullLogger:
    def log_metrics(self, metrics, step=None):
        pass


def _metric_means(sums: torch.Tensor) -> dict[str, float] | None:
    s = sums.tolist()
    n = s[4]
    if n <= 0:
        return None
    nll = s[0] / n
    return {"loss": nll, "nll": nll, "mae": s[1] / n, "rmse": math.sqrt(s[2] / n), "sigma": s[3] / n}


def train_step(model: StereoUNet, optimizer: FusedAdamW | None, inputs, targets, valid_mask,
               grad_hook: Callable[[str], None] | None = None, count_hook: Callable[[torch.Tensor], None] | None = None,
               before_step: Callable[[], None] | None = None):
    """One fused step (train.py:320-343) if optimizer is given, else an eval pass (train.py:301,327-340).

    Accumulates (sum nll, sum |d|, sum d^2, sum sigma, n) into ``model._engine.metrics``.
    grad_hook(name) is called as each top-level module's gradients become final (DDP buckets);
    count_hook(count) may all-reduce the valid count before the loss normalisation; if it returns a handle
    (an async collective), the handle is waited on after the forward, which the collective then overlaps.
    """
    eng = model.engine(inputs.device)
    with torch.cuda.device(eng.device):
        _train_step(model, eng, optimizer, inputs, targets, valid_mask, grad_hook, count_hook, before_step)


def _train_step(model, eng, optimizer, inputs, targets, valid_mask, grad_hook, count_hook, before_step):
    training = optimizer is not None
    mask_u8 = valid_mask.contiguous().view(torch.uint8)
    targets = targets.contiguous()
    # the valid count depends on the batch only: counted (and all-reduced) ahead of the forward; with the weight packs
    # and the input pack in one launch where it applies
    fused = eng.step_prologue(inputs, targets, mask_u8, training)
    if not fused:
        eng.count_valid(targets, mask_u8)
    try:
        pending = count_hook(eng.count) if count_hook is not None else None
    except BaseException:
        eng._xin_ready = None  # the packed input belongs to this step's forward only
        raise
    if not fused:
        eng.pack_weights(train=training)
    eng.forward(inputs, train=training)
    if pending is not None:
        pending.wait()
    if not training:
        eng.heads(L.SD_HEADS_LOSS, target=targets, valid=mask_u8, no_grad=True)
        return
    eng.heads(L.SD_HEADS_LOSS, target=targets, valid=mask_u8)
    if grad_hook is not None:
        grad_hook("heads")
    eng.backward(grad_hook)
    if before_step is not None:
        before_step()
    optimizer.fused_step(gather_grads=False, gate_on_count=True)


def run_epoch(model: StereoUNet, loader, device: torch.device, optimizer: FusedAdamW | None = None,
              global_step: int = 0, log_every_batches: int | None = None, logger=None, ddp=None):
    """train.py:292-418 on the HIP path. Returns (metrics, global_step)."""
    is_training = optimizer is not None
    model.train(is_training)
    logger = logger or _NullLogger()
    eng = model.engine(device)
    eng.metrics.zero_()
    interval = torch.zeros(5, dtype=torch.float64, device=eng.device)
    for batch in loader:
        if is_training:
            global_step += 1
        inputs = batch["input"].to(device, non_blocking=True)
        targets = batch["target"].to(device, non_blocking=True)
        valid_mask = batch["valid_mask"].to(device, non_blocking=True)
        if ddp is not None:
            ddp.step(model, optimizer, inputs, targets, valid_mask)
        else:
            train_step(model, optimizer, inputs, targets, valid_mask)
        if (is_training and log_every_batches is not None and log_every_batches > 0
                and global_step % log_every_batches == 0):
            cur = eng.metrics.clone()
            if ddp is not None:
                cur = ddp.sum_metrics(cur)
            means = _metric_means(cur - interval)
            if means is not None:
                logger.log_metrics({f"train_{k}_step": v for k, v in means.items()}, step=global_step)
                interval = cur
    total = eng.metrics.clone()
    if ddp is not None:
        total = ddp.sum_metrics(total)
    if total[4].item() == 0:
        raise RuntimeError("No valid target pixels found for this epoch.")
    if is_training:
        means = _metric_means(total - interval)
        if means is not None:
            logger.log_metrics({f"train_{k}_step": v for k, v in means.items()}, step=global_step)
    return _metric_means(total), global_step
