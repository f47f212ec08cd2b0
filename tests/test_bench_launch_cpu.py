"""bench.py's multi-GPU launcher logic on CPU.

`python bench.py --gpus N` without WORLD_SIZE (the driver's BENCH command form) must start N rank processes through a
child torch.distributed.run BEFORE anything touches a GPU, and a --gpus / WORLD_SIZE mismatch must fail instead of
measuring one GPU. SD_BENCH_PROBE=1 makes each rank join a gloo group and report instead of running the step.
"""

import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO))

import bench  # noqa: E402


def test_launch_plan_single_and_ranked():
    assert bench.launch_plan(1, {}, ["--gpus", "1"]) is None
    assert bench.launch_plan(4, {"WORLD_SIZE": "4"}, ["--gpus", "4"]) is None  # a rank of torch.distributed.run


def test_launch_plan_spawns_ranks_without_world_size():
    cmd = bench.launch_plan(8, {}, ["--gpus", "8", "--steps", "3"])
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in cmd and "127.0.0.1" in cmd
    assert cmd[-4:] == ["--gpus", "8", "--steps", "3"]


@pytest.mark.parametrize("world,gpus", [("1", 8), ("2", 4), ("8", 1)])
def test_launch_plan_mismatch_is_an_error(world, gpus):
    with pytest.raises(SystemExit):
        bench.launch_plan(gpus, {"WORLD_SIZE": world}, [])


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                             "MASTER_PORT")}
    env.update(SD_BENCH_PROBE="1", PYTHONDONTWRITEBYTECODE="1", **kw)
    return env


def test_bench_gpus_2_starts_two_ranks():
    r = subprocess.run([sys.executable, str(REPO / "bench.py"), "--gpus", "2"], env=_env(), capture_output=True,
                       text=True, timeout=300, cwd=REPO)
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line == {"probe": True, "n_gpus": 2, "gpus_arg": 2, "rank_sum": 3.0, "local_ranks": "2"}


def test_bench_world_size_mismatch_exits_nonzero():
    r = subprocess.run([sys.executable, str(REPO / "bench.py"), "--gpus", "4"], env=_env(WORLD_SIZE="2", RANK="0"),
                       capture_output=True, text=True, timeout=300, cwd=REPO)
    assert r.returncode != 0
    assert "WORLD_SIZE=2" in r.stderr
    assert not r.stdout.strip()


def test_step_roofline_prices_surveys_85_gflop_step():
    """the whole-step conv roofline. Its GEMM table must carry the survey's
    85.025 GFLOP per training pair at 320x240 (fwd 28.430 + dgrad 28.165 + wgrad 28.430), and the attainable time at
    B = 64 must give the survey's ~20.6-20.9 k pairs/s ceiling; frac = attainable / measured."""
    r = bench.step_roofline(8.0, 64, 240, 320)
    assert abs(r["gflop_per_pair"] - 85.025) < 0.01
    assert 20_000 < r["ceiling_pairs_s"] < 21_500
    assert r["frac"] == round(r["attainable_ms_per_step"] / 8.0, 4)
    assert len(r["layers_us"]) == 23 and "dgrad" not in r["layers_us"]["enc1.0"]
    assert r["layers_us"]["dec4.0"]["wgrad"][1] == "mfma" and r["layers_us"]["dec1.1"]["fwd"][1] == "hbm"
