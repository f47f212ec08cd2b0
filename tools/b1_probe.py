"""Per-launch cost of the eval convs at batch 1, 960x720 (the live app's forward), inside a HIP graph.

    python tools/b1_probe.py [reps]

For each layer shape: REPS launches of the same conv captured in one graph, replayed, time / REPS (HIP events). Also a
1-element torch add (the per-kernel floor of a graph node). Prints us per launch.
"""

from __future__ import annotations

import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import torch  # noqa: E402

from stereo_depth_estimation_amd import _lib as L  # noqa: E402

SHAPES = [  # (H, W, cin, cout): the live app's 960x720 forward, one shape per U-Net level
    (16, 32, 32, 32),
    (720, 960, 32, 32),
    (360, 480, 64, 64),
    (180, 240, 128, 128),
    (90, 120, 256, 256),
    (90, 120, 512, 256),
    (45, 60, 512, 512),
]


def graph_time(fn, reps: int, s: torch.cuda.Stream) -> float:
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for _ in range(reps):
            fn()
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = 1e9
    for _ in range(5):
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) * 1e3 / reps)
    return best


def main() -> None:
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    dev = torch.device("cuda:0")
    L.load()
    s = torch.cuda.Stream()
    sp = s.cuda_stream
    t = torch.zeros(1, device=dev)
    print(f"torch add (1 element): {graph_time(lambda: t.add_(1.0), reps, s):7.2f} us")
    # chained full-resolution pair (enc1.0 -> enc1.1): singles vs the pair in one graph
    H, W = 720, 960
    x8 = torch.randn(H * W, 8, device=dev).to(torch.bfloat16)
    w1 = (torch.randn(32 * 128, device=dev) * 0.05).to(torch.bfloat16)
    w2 = (torch.randn(32 * 320, device=dev) * 0.05).to(torch.bfloat16)
    o1 = torch.empty(H * W, 32, device=dev, dtype=torch.bfloat16)
    o2 = torch.empty(H * W, 32, device=dev, dtype=torch.bfloat16)
    sc32, sh32 = torch.rand(32, device=dev) + 0.5, torch.randn(32, device=dev) * 0.1
    s1 = L.make_src(x8, 8, H, W, taps=9)
    s2 = L.make_src(o1, 32, H, W, taps=9, bn0=(sc32, sh32))

    def c1():
        L.call("sd_conv_gemm", L.SD_BF16, s1, 1, H, W, w1.data_ptr(), 32, 128, L.SD_EPI_STORE, o1.data_ptr(),
               None, 0, None, None, sp)

    def c2():
        L.call("sd_conv_gemm", L.SD_BF16, s2, 1, H, W, w2.data_ptr(), 32, 320, L.SD_EPI_STORE, o2.data_ptr(),
               None, 0, None, None, sp)

    def pair():
        c1()
        c2()

    print(f"enc1.0 {graph_time(c1, reps, s):7.2f} us  enc1.1 {graph_time(c2, reps, s):7.2f} us  "
          f"pair {graph_time(pair, reps, s):7.2f} us  "
          f"({L.kernel_name('sd_conv_gemm_kernel_name', L.SD_BF16, s1, 1, H, W, 32, L.SD_EPI_STORE)}, "
          f"{L.kernel_name('sd_conv_gemm_kernel_name', L.SD_BF16, s2, 1, H, W, 32, L.SD_EPI_STORE)})")
    for H, W, ci, co in SHAPES:
        torch.manual_seed(0)
        y = torch.randn(H * W, ci, device=dev).to(torch.bfloat16)
        sc = torch.rand(ci, device=dev) + 0.5
        sh = torch.randn(ci, device=dev) * 0.1
        kpad = ((9 * ci + 63) // 64) * 64
        w = (torch.randn(co * kpad, device=dev) * 0.05).to(torch.bfloat16)
        o = torch.empty(H * W, co, device=dev, dtype=torch.bfloat16)
        src = L.make_src(y, ci, H, W, taps=9, bn0=(sc, sh))

        hb = L.call("sd_conv3x3_ex_ws_bytes", src, 1, H, W, co, L.SD_EPI_STORE, 0)
        hws = torch.empty(max(hb // 4, 4), device=dev)

        def bf16():
            L.call("sd_conv3x3_ex_ws", src, 1, H, W, w.data_ptr(), co, kpad, L.SD_EPI_STORE, 0, None, None,
                   o.data_ptr(), None, hws.data_ptr(), 4 * hws.numel(), sp)

        name = L.kernel_name("sd_conv_gemm_kernel_name", L.SD_BF16, src, 1, H, W, co, L.SD_EPI_STORE)
        tb = graph_time(bf16, reps, s)
        srcq = L.make_src(y, ci, H, W, taps=9, bn0=(sc, sh), xform0=L.SD_BNRELU)
        ctap = (ci + 15) // 16 * 16
        kq = ((9 * ctap + 63) // 64) * 64
        wq = torch.randint(0, 0x70, (co * kq,), device=dev, dtype=torch.uint8)
        wsc = torch.full((co,), 1e-2, device=dev)
        asc = torch.ones(1, device=dev)

        def q8():
            L.call("sd_conv3x3_q8", srcq, 1, H, W, wq.data_ptr(), wsc.data_ptr(), asc.data_ptr(), co, kq,
                   o.data_ptr(), sp)

        tq = graph_time(q8, reps, s)
        qn = L.kernel_name("sd_conv3x3_q8_kernel_name", 1, H, W, co, ci, 0)
        # cold: every launch of the graph on its own input, weights and output (as the layers of one forward)
        ys = [torch.randn(H * W, ci, device=dev).to(torch.bfloat16) for _ in range(reps)]
        wqs = [torch.randint(0, 0x70, (co * kq,), device=dev, dtype=torch.uint8) for _ in range(reps)]
        os_ = [torch.empty(H * W, co, device=dev, dtype=torch.bfloat16) for _ in range(reps)]
        srcs = [L.make_src(yy, ci, H, W, taps=9, bn0=(sc, sh), xform0=L.SD_BNRELU) for yy in ys]
        it = [0]

        def q8c():
            i = it[0] % reps
            it[0] += 1
            L.call("sd_conv3x3_q8", srcs[i], 1, H, W, wqs[i].data_ptr(), wsc.data_ptr(), asc.data_ptr(), co, kq,
                   os_[i].data_ptr(), sp)

        tqc = graph_time(q8c, reps, s)
        print(f"{H:3d}x{W:3d} {ci:3d}->{co:3d}  bf16 {tb:7.2f} us {name}   q8 {tq:7.2f} us  cold {tqc:7.2f} us {qn}")


if __name__ == "__main__":
    main()
