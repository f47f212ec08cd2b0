"""Data parallelism for the HIP training path (one process per GPU, RCCL over xGMI).

The reference is single-process (no torch.distributed anywhere); this adds the
one strategy the north star asks for.  Semantics chosen to match the single-process
reference on the global batch:
  * the valid-pixel count is all-reduced BEFORE the loss normalisation, so every rank's
    gradient is d(global mean NLL)/dθ and the gradient all-reduce is a plain SUM
    (train.py:334-340 on the concatenated global batch);
  * the zero-valid skip (train.py:331-332) is decided on the global count, identically on
    every rank, so parameters never diverge;
  * BatchNorm uses per-rank batch statistics (standard DDP). The running statistics
    drift apart per rank during an epoch; ``sync_buffers()`` broadcasts rank 0's before every
    evaluation epoch and checkpoint (torch DDP's broadcast_buffers, once per epoch instead of per
    forward: nothing reads them between training forwards), so every rank evaluates, and
    best.pt is chosen, with the statistics that are saved. ``sync_bn=True`` instead normalises with
    the global batch's statistics (SyncBatchNorm: two fp64 all-reduces per BN layer per step), which
    reproduces the single-process reference on the concatenated batch.
Gradient buckets are contiguous slices of the flat gradient buffer (the model stores
parameters in backward-production order), each all-reduced asynchronously on RCCL's stream
as soon as backward finalises its last module — the collective overlaps the rest of
backward; AdamW waits for all buckets.  Nothing here synchronises the host.
"""

from __future__ import annotations

import torch
import torch.distributed as dist

# top-level modules in the order the engine finalises their gradients
GRAD_EVENTS = ("heads", "dec1", "up1", "dec2", "up2", "dec3", "up3", "dec4", "up4", "bottleneck", "enc4", "enc3",
               "enc2", "enc1")


def plan_buckets(ranges: list[tuple[str, int, int]], cap_elems: int) -> list[tuple[tuple[str, ...], int, int]]:
    """Group (module, start, end) flat ranges (backward order) into contiguous buckets of
    >= cap_elems elements (the last one may be smaller).  Heads' two modules map to 'heads'."""
    merged: list[tuple[str, int, int]] = []
    for name, a, b in ranges:
        key = "heads" if name in ("disparity_head", "logvar_head") else name
        if merged and merged[-1][0] == key:
            merged[-1] = (key, merged[-1][1], b)
        else:
            merged.append((key, a, b))
    buckets, cur, start = [], [], None
    for key, a, b in merged:
        if start is None:
            start = a
        cur.append(key)
        if b - start >= cap_elems:
            buckets.append((tuple(cur), start, b))
            cur, start = [], None
    if cur:
        buckets.append((tuple(cur), start, merged[-1][2]))
    return buckets


class BucketAllReduce:
    """Launch an async SUM all-reduce per bucket when its last module's grads are final."""

    def __init__(self, flat: torch.Tensor, buckets, group=None):
        self.flat, self.buckets, self.group = flat, buckets, group
        self.last_of = {names[-1]: i for i, (names, _, _) in enumerate(buckets)}
        self.handles = []
        # measurement (bench.py): (start, end) HIP events around each wait, on the stream that waits. With RCCL the
        # wait makes the current stream wait for RCCL's, so end - start is the all-reduce time backward did not hide
        self.wait_events: list | None = None

    def on_grads_ready(self, name: str):
        i = self.last_of.get(name)
        if i is not None:
            _, a, b = self.buckets[i]
            self.handles.append(dist.all_reduce(self.flat[a:b], op=dist.ReduceOp.SUM, group=self.group, async_op=True))

    def wait(self):
        ev = None
        if self.wait_events is not None:
            ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            ev[0].record()
        for h in self.handles:
            h.wait()
        self.handles.clear()
        if ev is not None:
            ev[1].record()
            self.wait_events.append(ev)


class ShardSampler(torch.utils.data.Sampler):
    """Exact, unpadded shard of a dataset for evaluation: rank r takes indices r, r + world, ... . Every sample is
    seen by exactly one rank, so the all-reduced metric sums equal the single-process epoch's (the reference's
    validation, train.py:617-620), where torch's DistributedSampler pads the shards with repeated samples."""

    def __init__(self, n: int, world: int, rank: int):
        self.n, self.world, self.rank = n, world, rank

    def __iter__(self):
        return iter(range(self.rank, self.n, self.world))

    def __len__(self) -> int:
        return len(range(self.rank, self.n, self.world))


class DataParallel:
    def __init__(self, model, group=None, bucket_cap_mb: float = 8.0, broadcast: bool = True, sync_bn: bool = False):
        """sync_bn: global-batch BatchNorm statistics (torch.nn.SyncBatchNorm semantics; SURVEY §8e "--sync-bn"):
        one fp64 all-reduce of per-channel (sum, sumsq) per BN layer in the forward and of (sum dz, sum dz*xhat) in
        the backward, 2 x 18 small collectives per step. Each carries the rank's pixel count, so ranks may hold
        batches of different sizes (the last batch of an epoch)."""
        self.model, self.group = model, group
        self.world = dist.get_world_size(group)
        self.cap = int(bucket_cap_mb * 1024 * 1024 / 4)
        self._ar = None
        self.sync_bn = sync_bn
        if broadcast:
            self.broadcast_state()
        if sync_bn:
            eng = model.engine(next(model.parameters()).device)
            eng.bn_sync = lambda t: dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)

    def broadcast_state(self):
        dev = next(self.model.parameters()).device
        self.model.engine(dev)
        flat_p, _ = self.model.flat_buffers()
        dist.broadcast(flat_p, src=0, group=self.group)
        self.sync_buffers()

    def sync_buffers(self):
        """BatchNorm running statistics (and num_batches_tracked) from rank 0 to every rank."""
        for b in self.model.buffers():
            dist.broadcast(b, src=0, group=self.group)
        if self.model._engine is not None:
            self.model._engine.touch_state()  # eval forwards must recompute the BN coefficients / re-pack

    def _reducer(self):
        flat_p, flat_g = self.model.flat_buffers()
        if self._ar is None or self._ar.flat is not flat_g:
            self._ar = BucketAllReduce(flat_g, plan_buckets(self.model.bucket_ranges(), self.cap), self.group)
        return self._ar

    def step(self, model, optimizer, inputs, targets, valid_mask):
        from .train import train_step

        if optimizer is None:
            # evaluation: no loss normaliser is needed (the metric sums count this rank's pixels, summed once per epoch
            # by sum_metrics), so no per-batch collective either: ranks may hold different numbers of batches
            train_step(model, None, inputs, targets, valid_mask)
            return
        ar = self._reducer()
        train_step(model, optimizer, inputs, targets, valid_mask, grad_hook=ar.on_grads_ready,
                   count_hook=self._allreduce_count, before_step=ar.wait)

    def _allreduce_count(self, count: torch.Tensor):
        """count := the global valid count (sd_count_valid wrote this rank's into both of the engine's counters; the
        SUM all-reduce turns `count` into the global one, `count_local` keeps this rank's for the metric sums). Async:
        train_step waits on the handle after the forward, so the collective's latency overlaps it."""
        eng = getattr(getattr(self, "model", None), "_engine", None)
        if eng is not None and count.data_ptr() == eng.count_local.data_ptr():
            raise RuntimeError("DDP count all-reduce on the engine's per-rank counter (count aliases count_local)")
        return dist.all_reduce(count, op=dist.ReduceOp.SUM, group=self.group, async_op=True)

    def sum_metrics(self, t: torch.Tensor) -> torch.Tensor:
        t = t.clone()
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)
        return t
