"""World-size-2 `gloo` tests of the data-parallel host logic (stereo_depth_estimation_amd/ddp.py).

The reference trains single-process; the DDP semantics added here are:
contiguous gradient buckets in backward order, an async SUM all-reduce per bucket fired when
its last module's gradients are final, and a SUM all-reduce of the valid-pixel count before the
loss normalisation (so the zero-valid skip of train.py:331-332 is decided globally).
These run on CPU; the GPU test (test_gpu_ddp.py) checks the same path end to end.
"""

from __future__ import annotations

import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from stereo_depth_estimation_amd.ddp import GRAD_EVENTS, BucketAllReduce, DataParallel, ShardSampler, plan_buckets
from stereo_depth_estimation_amd.model import StereoUNet


def _ranges(base=32):
    return StereoUNet(in_channels=6, out_channels=1, base_channels=base).bucket_ranges()


@pytest.mark.parametrize("cap", [1, 10_000, 2_000_000, 10**9])
def test_plan_buckets_contiguous_cover_in_backward_order(cap):
    ranges = _ranges()
    total = ranges[-1][2]
    buckets = plan_buckets(ranges, cap)
    assert buckets[0][1] == 0 and buckets[-1][2] == total
    for (_, _, e0), (_, a1, _) in zip(buckets, buckets[1:]):
        assert e0 == a1  # contiguous slices of the flat gradient buffer
    assert all(e - a >= cap for _, a, e in buckets[:-1])
    names = [n for ns, _, _ in buckets for n in ns]
    assert names == list(GRAD_EVENTS)  # every module once, heads merged, in the engine's finalise order
    if cap == 1:
        assert len(buckets) == len(GRAD_EVENTS)
    if cap == 10**9:
        assert len(buckets) == 1


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank: int, world: int, port: int, cap: int, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        ranges = _ranges(base=8)
        total = ranges[-1][2]
        buckets = plan_buckets(ranges, cap)
        flat = torch.arange(total, dtype=torch.float32) * (rank + 1)
        ar = BucketAllReduce(flat, buckets)
        # a bucket's collective starts exactly when its last module is final, not before
        launched = []
        for i, name in enumerate(GRAD_EVENTS):
            ar.on_grads_ready(name)
            done = set(GRAD_EVENTS[: i + 1])
            launched.append(len(ar.handles) == sum(1 for ns, _, _ in buckets if ns[-1] in done))
        ar.wait()
        scale = sum(r + 1 for r in range(world))
        ok_sum = torch.equal(flat, torch.arange(total, dtype=torch.float32) * scale) and not ar.handles
        # host-side reducers (no engine needed): global valid count, metric sums
        dp = DataParallel.__new__(DataParallel)
        dp.group = None
        count = torch.tensor([0 if rank == 0 else 7], dtype=torch.int32)  # rank 0 alone would skip
        dp._allreduce_count(count).wait()  # async (train_step waits after the forward)
        met = torch.tensor([1.0, 2.5, 4.0], dtype=torch.float64) * (rank + 1)
        before = met.clone()
        s = dp.sum_metrics(met)
        ok_met = torch.equal(s, torch.tensor([1.0, 2.5, 4.0], dtype=torch.float64) * scale) and torch.equal(met, before)
        q.put((rank, all(launched), ok_sum, int(count.item()), ok_met))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("cap", [1, 50_000])
def test_bucket_allreduce_count_and_metrics_world2(cap):
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, cap, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, launched_in_order, ok_sum, count, ok_met in sorted(results):
        assert launched_in_order, f"rank {rank}: bucket launched before its last module was final"
        assert ok_sum, f"rank {rank}: bucketed SUM all-reduce wrong"
        assert count == 7, f"rank {rank}: global valid count {count} (zero-valid skip must be global)"
        assert ok_met, f"rank {rank}: metric sums wrong"


def _val_sums(net, batches):
    """Eval-mode metric sums (train.py:345-356) of the oracle over the given batches, in the engine's
    metrics layout [sum nll, sum |d|, sum d^2, sum sigma, n] (fp64)."""
    from oracle import unet_ref as U

    tot = torch.zeros(5, dtype=torch.float64)
    for b in batches:
        with torch.no_grad():
            d, lv = net.forward(torch.as_tensor(b["input"]), train=False)
        _, s = U.masked_nll(d, lv, torch.as_tensor(b["target"]), torch.as_tensor(b["valid_mask"]))
        tot += torch.tensor([s["nll"], s["abs"], s["sq"], s["sigma"], s["n"]], dtype=torch.float64)
    return tot


def _collate(items):
    import numpy as np

    return {k: np.concatenate([it[k] for it in items]) for k in items[0]}


def _val_worker(rank: int, world: int, port: int, n: int, bs: int, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from torch.utils.data.distributed import DistributedSampler

        from oracle import unet_ref as U
        from stereo_depth_estimation_amd.train import _metric_means

        torch.set_num_threads(2)
        items = [U.make_batch(1, 32, 48, seed=100 + i) for i in range(n)]
        net = U.Net(U.make_state(8, seed=0), base_channels=8)
        dp = DataParallel.__new__(DataParallel)
        dp.group = None
        out = {}
        for name, sampler in (("exact", ShardSampler(n, world, rank)),
                              ("padded", DistributedSampler(range(n), num_replicas=world, rank=rank, shuffle=False))):
            idx = list(sampler)
            batches = [_collate([items[i] for i in idx[j:j + bs]]) for j in range(0, len(idx), bs)]
            out[name] = (idx, _metric_means(dp.sum_metrics(_val_sums(net, batches))))
        q.put((rank, out, None))
    except Exception as e:  # report instead of hanging the parent
        q.put((rank, None, repr(e)))
        raise
    finally:
        dist.destroy_process_group()


def test_val_shards_exact_metrics_equal_single_process_world2():
    """Validation under DDP (cli.py): exact unpadded shards (ShardSampler) + one SUM all-reduce of the metric sums give
    the single-process epoch's metrics on an odd-sized val set (the reference's val epoch, train.py:617-620, and so
    its best.pt choice on val mae, :656-662); torch's DistributedSampler pads a duplicate sample and does not."""
    import math

    from oracle import unet_ref as U

    world, n, bs = 2, 5, 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_val_worker, args=(r, world, port, n, bs, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = sorted((q.get(timeout=180) for _ in range(world)), key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
    items = [U.make_batch(1, 32, 48, seed=100 + i) for i in range(n)]
    net = U.Net(U.make_state(8, seed=0), base_channels=8)
    ref, _ = U.run_epoch(net, [_collate(items[j:j + bs]) for j in range(0, n, bs)], None)
    shards = []
    for rank, out, err in results:
        assert err is None, f"rank {rank}: {err}"
        shards.append(out["exact"][0])
        for k, v in ref.items():
            assert math.isclose(out["exact"][1][k], v, rel_tol=1e-6), (rank, k, out["exact"][1][k], v)
        assert any(not math.isclose(out["padded"][1][k], v, rel_tol=1e-6) for k, v in ref.items())
    assert sorted(i for s in shards for i in s) == list(range(n))  # every sample exactly once
    assert all(p.exitcode == 0 for p in procs)
