"""Data-parallel train step end to end on the GPU: two ranks, either `gloo` over device tensors with
both ranks on cuda:0 (the single-GPU box has one card), or the production path — RCCL (`nccl`
backend) with one rank per GPU and the async bucket all-reduces on RCCL's stream overlapping
backward — when the box has two or more GPUs (skipped otherwise).

* Both ranks train on the SAME batch: per-rank BN statistics then equal the single-process ones,
  the global valid count is 2x, and the SUM of the two gradients normalised by it equals the
  single-process gradient — so after two DDP steps the parameters must match two plain
  single-process steps (fp32 path; only reduction order differs).
* Rank 0 gets a batch with no valid pixel, rank 1 a normal one: the skip of train.py:331-332 is
  decided on the global count, so both ranks step and stay bit-identical.
* Different batches per rank: the per-rank BN running statistics differ after a step and are equal
  again after ``DataParallel.sync_buffers()`` (called by the CLI before evaluation / checkpoints).
"""

from __future__ import annotations

import os
import socket

import pytest
import torch

pytestmark = pytest.mark.gpu


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank: int, world: int, port: int, q, backend: str = "gloo"):
    import torch.distributed as dist

    from stereo_depth_estimation_amd.data import synthetic_batch
    from stereo_depth_estimation_amd.ddp import DataParallel
    from stereo_depth_estimation_amd.model import StereoUNet
    from stereo_depth_estimation_amd.optim import FusedAdamW
    from stereo_depth_estimation_amd.train import train_step

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
    dev = torch.device("cuda", rank if backend == "nccl" else 0)
    torch.cuda.set_device(dev)
    if backend == "nccl":
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    else:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    try:

        def make():
            torch.manual_seed(0)
            m = StereoUNet(in_channels=6, out_channels=1, base_channels=8, precision="fp32").to(dev)
            return m, FusedAdamW(m.parameters(), lr=1e-3, weight_decay=1e-4)

        b = synthetic_batch(2, 32, 48, seed=5, device=dev)
        # 1) same batch on both ranks == single process
        m_ddp, o_ddp = make()
        dp = DataParallel(m_ddp, bucket_cap_mb=0.05)
        m_ref, o_ref = make()
        for _ in range(2):
            dp.step(m_ddp, o_ddp, b["input"], b["target"], b["valid_mask"])
            train_step(m_ref, o_ref, b["input"], b["target"], b["valid_mask"])
        torch.cuda.synchronize()
        diff = max(float((p - r).abs().max()) for p, r in zip(m_ddp.parameters(), m_ref.parameters()))
        # 2) rank 0 has no valid pixel: both ranks still step, in lockstep
        m2, o2 = make()
        dp2 = DataParallel(m2)
        mask = b["valid_mask"].clone()
        if rank == 0:
            mask.zero_()
        p0 = torch.cat([p.detach().flatten().clone() for p in m2.parameters()])
        dp2.step(m2, o2, b["input"], b["target"], mask)
        torch.cuda.synchronize()
        p1 = torch.cat([p.detach().flatten() for p in m2.parameters()])
        moved = bool((p1 != p0).any())
        gathered = [torch.empty_like(p1) for _ in range(world)]
        dist.all_gather(gathered, p1)
        in_sync = all(torch.equal(gathered[0], g) for g in gathered)
        # 3) different batches per rank: BN running statistics drift apart until sync_buffers()
        m3, o3 = make()
        dp3 = DataParallel(m3)
        b3 = synthetic_batch(2, 32, 48, seed=11 + rank, device=dev)
        dp3.step(m3, o3, b3["input"], b3["target"], b3["valid_mask"])
        bufs = torch.cat([t.detach().double().flatten() for t in m3.buffers()])
        gathered = [torch.empty_like(bufs) for _ in range(world)]
        dist.all_gather(gathered, bufs)
        drifted = not all(torch.equal(gathered[0], g) for g in gathered)
        dp3.sync_buffers()
        bufs = torch.cat([t.detach().double().flatten() for t in m3.buffers()])
        dist.all_gather(gathered, bufs)
        synced = all(torch.equal(gathered[0], g) for g in gathered)
        q.put((rank, diff, moved, in_sync and drifted and synced, None))
    except Exception as e:  # report instead of hanging the parent
        q.put((rank, None, None, None, repr(e)))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("backend", ["gloo", "nccl"])
def test_ddp_two_ranks_match_single_process_and_skip_globally(backend):
    import torch.multiprocessing as mp

    if backend == "nccl" and torch.cuda.device_count() < 2:
        pytest.skip("RCCL two-rank test needs two GPUs (one rank per device)")
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, backend)) for r in range(world)]
    for p in procs:
        p.start()
    results = sorted(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=120)
    for rank, diff, moved, in_sync, err in results:
        assert err is None, f"rank {rank}: {err}"
        assert diff <= 1e-6, f"rank {rank}: DDP params differ from single-process by {diff}"
        assert moved, f"rank {rank}: zero-local-valid rank skipped the step (skip must use the global count)"
        assert in_sync, f"rank {rank}: ranks diverged, or BN buffers not re-synced by sync_buffers()"
    assert all(p.exitcode == 0 for p in procs)


def _sync_bn_worker(rank: int, world: int, port: int, q, precision: str = "fp32"):
    import torch.distributed as dist

    from stereo_depth_estimation_amd.data import synthetic_batch
    from stereo_depth_estimation_amd.ddp import DataParallel
    from stereo_depth_estimation_amd.model import StereoUNet
    from stereo_depth_estimation_amd.optim import FusedAdamW
    from stereo_depth_estimation_amd.train import train_step

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY="0")
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        def make():
            torch.manual_seed(0)
            m = StereoUNet(in_channels=6, out_channels=1, base_channels=base, precision=precision).to(dev)
            return m, FusedAdamW(m.parameters(), lr=1e-3, weight_decay=1e-4)

        # fp32: the small parity configuration; bf16: the product kernels (halo convs, fused BN-backward sums from
        # the pool backward / dgrad epilogues / heads, all feeding the synced finalizes)
        base, H, W = (8, 32, 48) if precision == "fp32" else (32, 64, 96)
        b = synthetic_batch(2 * world, H, W, seed=21, device=dev)
        shard = {k: v[2 * rank:2 * rank + 2] for k, v in b.items()}
        m_ref, o_ref = make()
        train_step(m_ref, o_ref, b["input"], b["target"], b["valid_mask"])  # one process, the whole batch
        g_ref = m_ref.flat_buffers()[1].double().clone()
        bufs_ref = [t.detach().double().clone() for t in m_ref.buffers()]
        out = {}
        for sync in (True, False):  # sync-BN, and per-rank BN as the control the test must tell apart
            m, o = make()
            dp = DataParallel(m, bucket_cap_mb=0.05, sync_bn=sync)
            dp.step(m, o, shard["input"], shard["target"], shard["valid_mask"])
            torch.cuda.synchronize()
            g = m.flat_buffers()[1].double()
            rel = float((g - g_ref).norm() / g_ref.norm())
            bd = max(float((t.detach().double() - r).abs().max() / (r.abs().max() + 1e-12))
                     for t, r in zip(m.buffers(), bufs_ref) if t.is_floating_point())
            out[sync] = (rel, bd)
        diff, bdiff = out[True]
        ctrl, bctrl = out[False]
        print(f"sync-bn {precision} rank {rank}: grad rel {diff:.3e} (per-rank BN {ctrl:.3e}), "
              f"running stats rel {bdiff:.3e} (per-rank BN {bctrl:.3e})", flush=True)
        q.put((rank, diff, bdiff, ctrl, bctrl, None))
    except Exception as e:
        q.put((rank, None, None, None, repr(e)))
        raise
    finally:
        dist.destroy_process_group()


# bound on (gradient rel. error, running-statistics rel. error) against the single process on the whole batch
SYNC_TOL = {"fp32": (1e-5, 1e-5), "bf16": (5e-3, 1e-5)}  # measured: 3.6e-7 / 4.0e-7, 5.0e-4 / 0


@pytest.mark.parametrize("precision", ["fp32", "bf16"])
def test_sync_bn_two_ranks_match_single_process_on_the_global_batch(precision):
    """DataParallel(sync_bn=True): two ranks on half a batch each normalise with the global batch's BatchNorm
    statistics, so the all-reduced gradient of one step equals the single-process gradient on the whole batch (the
    reference's semantics) within fp32 rounding, and so do the BN running statistics (incl. the unbiased variance
    over the global count). Per-rank BN on the same shards is the control: it must be far off. bf16: bf16 storage of
    every activation and gradient rounds differently when the batch is split, hence the looser bounds."""
    import torch.multiprocessing as mp

    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_sync_bn_worker, args=(r, world, port, q, precision)) for r in range(world)]
    for p in procs:
        p.start()
    results = sorted(q.get(timeout=300) for _ in range(world))
    for p in procs:
        p.join(timeout=120)
    gtol, btol = SYNC_TOL[precision]
    for rank, diff, bdiff, ctrl, bctrl, err in results:
        assert err is None, f"rank {rank}: {err}"
        assert diff <= gtol, f"rank {rank}: sync-BN gradient differs from the single-process global batch by {diff} (rel)"
        assert bdiff <= btol, f"rank {rank}: sync-BN running statistics differ by {bdiff} (rel)"
        assert bctrl > 1e3 * btol, f"rank {rank}: per-rank BN stats ({bctrl}) not distinguishable from sync-BN"
        assert ctrl > 10 * gtol, f"rank {rank}: per-rank BN ({ctrl}) not distinguishable from sync-BN ({diff})"
    assert all(p.exitcode == 0 for p in procs)
