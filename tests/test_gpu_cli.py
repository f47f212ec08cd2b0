"""Training CLI end to end on the GPU (cli.main, reference train.py:480-690 loop) on a small
FoundationStereo-layout PNG tree: checkpoints in the reference format, best.pt on val MAE, and
--resume continuing a run exactly: 3 epochs straight == 2 epochs + resume for
the 3rd, bit for bit (the kernels are deterministic; data order, augmentation factors and noise
seeds come from the RNG states saved in the checkpoint)."""

from __future__ import annotations

import json

import pytest
import torch

from conftest import write_stereo_tree

pytestmark = pytest.mark.gpu


def _args(root, out, run, epochs, extra=(), workers=0, augment=True):
    aug = ["--augment", "--brightness-jitter", "0.2", "--noise-std-max", "0.02"] if augment else []
    return ["--dataset-root", str(root), "--height", "32", "--width", "48", "--epochs", str(epochs),
            "--batch-size", "2", "--num-workers", str(workers), "--val-fraction", "0.25", "--output-dir", str(out),
            "--run-name", run, *aug, *extra]


def test_cli_checkpoints_and_exact_resume(tmp_path):
    from stereo_depth_estimation_amd import cli

    write_stereo_tree(tmp_path / "data", scenes=2, frames=4, hw=(40, 52), seed=9)
    straight = cli.main(_args(tmp_path / "data", tmp_path / "out", "straight", 3))
    ck_dir = tmp_path / "out" / "straight" / "checkpoints"
    assert (ck_dir / "last.pt").exists() and (ck_dir / "best.pt").exists()
    last = torch.load(ck_dir / "last.pt", map_location="cpu", weights_only=True)
    assert last["epoch"] == 3 and last["global_step"] == straight["global_step"] == 9
    assert set(last["metrics"]) >= {"train_mae", "val_mae", "epoch_seconds"}
    lines = (tmp_path / "out" / "straight" / "metrics.jsonl").read_text().splitlines()
    assert any(json.loads(x)["step"] == 3 and "val_mae" in json.loads(x) for x in lines)

    cli.main(_args(tmp_path / "data", tmp_path / "out", "resumed", 2))
    part = tmp_path / "out" / "resumed" / "checkpoints" / "last.pt"
    resumed = cli.main(_args(tmp_path / "data", tmp_path / "out", "resumed", 3, ["--resume", str(part)]))
    assert resumed["global_step"] == 9
    a = torch.load(ck_dir / "last.pt", map_location="cpu", weights_only=True)
    b = torch.load(part, map_location="cpu", weights_only=True)
    assert b["epoch"] == 3
    for k, v in a["model_state_dict"].items():
        assert torch.equal(v, b["model_state_dict"][k]), k
    for pid, st in a["optimizer_state_dict"]["state"].items():
        for k, v in st.items():
            assert torch.equal(torch.as_tensor(v), torch.as_tensor(b["optimizer_state_dict"]["state"][pid][k])), (pid, k)
    assert a["metrics"]["train_mae"] == b["metrics"]["train_mae"]


def test_cli_exact_resume_with_persistent_workers(tmp_path):
    """--num-workers 2 (persistent workers, the reference's loader setup): the worker base seed comes
    from its own generator, so the shuffle order and everything downstream continue exactly after
    --resume (augmentation off: its jitter is drawn inside the workers, see cli.py)."""
    from stereo_depth_estimation_amd import cli

    write_stereo_tree(tmp_path / "data", scenes=2, frames=4, hw=(40, 52), seed=9)
    kw = dict(workers=2, augment=False)
    cli.main(_args(tmp_path / "data", tmp_path / "out", "straight", 3, **kw))
    cli.main(_args(tmp_path / "data", tmp_path / "out", "resumed", 2, **kw))
    part = tmp_path / "out" / "resumed" / "checkpoints" / "last.pt"
    cli.main(_args(tmp_path / "data", tmp_path / "out", "resumed", 3, ["--resume", str(part)], **kw))
    a = torch.load(tmp_path / "out" / "straight" / "checkpoints" / "last.pt", map_location="cpu", weights_only=True)
    b = torch.load(part, map_location="cpu", weights_only=True)
    for k, v in a["model_state_dict"].items():
        assert torch.equal(v, b["model_state_dict"][k]), k
    assert a["metrics"]["train_mae"] == b["metrics"]["train_mae"]
