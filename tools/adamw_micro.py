"""Micro-benchmark of sd_adamw over a flat buffer of the model's size (StereoUNet base 32: 7.76 M parameters).

    SD_ADAM_BLOCKS=2048 python tools/adamw_micro.py [--n=50]

Prints us per call (HIP events, median of 3 rounds of n calls) and checks the device step counter advanced once per
call (the last-block hand-off of k_adamw).
"""

from __future__ import annotations

import json
import os
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import torch  # noqa: E402

from stereo_depth_estimation_amd import _lib as L  # noqa: E402


def main():
    n = next((int(a.split("=")[1]) for a in sys.argv[1:] if a.startswith("--n=")), 50)
    dev = "cuda"
    P = 7_762_465
    p, g, m, v = (torch.randn(P, device=dev) for _ in range(4))
    v.abs_()
    step = torch.zeros(1, dtype=torch.int32, device=dev)
    count = torch.ones(1, dtype=torch.int32, device=dev)
    scratch = torch.zeros(4, device=dev)
    s = torch.cuda.current_stream().cuda_stream

    def call():
        L.call("sd_adamw", p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr(), P, 1e-3, 1e-4, 0.9, 0.999, 1e-8,
               step.data_ptr(), count.data_ptr(), scratch.data_ptr(), s)

    for _ in range(5):
        call()
    rounds = []
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(n):
            call()
        e1.record()
        torch.cuda.synchronize()
        rounds.append(round(e0.elapsed_time(e1) * 1000 / n, 1))
    assert int(step.item()) == 5 + 3 * n, int(step.item())
    assert float(scratch.abs().sum()) == 0.0
    print(json.dumps({"blocks": os.environ.get("SD_ADAM_BLOCKS", "default"), "us": sorted(rounds)[1], "rounds": rounds}))


if __name__ == "__main__":
    main()
