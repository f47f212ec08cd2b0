"""hipBLASLt (torch.mm) time of the up3/up4 ConvTranspose GEMM shapes at B = 64, as a bound on what a tiled GEMM
reaches there (plain [M, K] x [K, N] bf16, no gather / BN transform / pixel-shuffle epilogue)."""
import torch

SHAPES = {"up4 fwd": (19200, 512, 1024), "up4 dgrad": (19200, 1024, 512), "up3 fwd": (76800, 256, 512),
          "up3 dgrad": (76800, 512, 256), "up4 wgrad (K=P)": (512, 76800, 256 * 4 // 4 * 4 // 4 * 1024 // 256),
          "up3 wgrad (K=P)": (256, 307200, 512)}
for name, (m, k, n) in SHAPES.items():
    a = torch.randn(m, k, device="cuda", dtype=torch.bfloat16)
    b = torch.randn(k, n, device="cuda", dtype=torch.bfloat16)
    for _ in range(5):
        c = a @ b
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(50):
        c = a @ b
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / 50 * 1e3
    print(f"{name:18s} M={m} K={k} N={n}: {us:7.1f} us  {2 * m * n * k / us / 1e6:7.1f} TFLOP/s", flush=True)
