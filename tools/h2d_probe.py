"""Does a pinned host -> device copy on a side stream run on a copy engine (SDMA) or as a blit kernel on the CUs?
    rocprofv3 --kernel-trace --memory-copy-trace -d out -o run -- python3 tools/h2d_probe.py
A blit kernel (__amd_rocclr_copyBuffer*) in the kernel trace during the copy means the data path's H2D competes with
the training kernels for CUs."""

import time

import torch


def main():
    dev = torch.device("cuda:0")
    n = 39 << 20  # one C4 batch of uint8 frames + f16 disparity
    host = torch.empty(n, dtype=torch.uint8).pin_memory()
    dst = torch.empty(n, dtype=torch.uint8, device=dev)
    side = torch.cuda.Stream(dev)
    for _ in range(3):
        with torch.cuda.stream(side):
            dst.copy_(host, non_blocking=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(10):
        with torch.cuda.stream(side):
            dst.copy_(host, non_blocking=True)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / 10
    print(f"H2D {n / 2**20:.0f} MiB: {dt * 1e3:.3f} ms, {n / dt / 1e9:.1f} GB/s", flush=True)


if __name__ == "__main__":
    main()
