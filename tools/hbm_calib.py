"""Achievable HBM rate on this box: PyTorch copy (read + write), fill (write only) and sum (read only) over buffers far
larger than the 256 MB MALL, timed with HIP events. The bench's roofline `peak` stays the 8 TB/s spec figure; this
gives the practical ceiling the HBM-bound kernels' rates compare against.
    python tools/hbm_calib.py [GiB]"""

import ctypes
import json
import sys
from pathlib import Path

import torch


def timed(fn, iters=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters * 1e-3


def main():
    gib = float(sys.argv[1]) if len(sys.argv) > 1 else 2.0
    n = int(gib * (1 << 30)) // 2
    src = torch.randn(n, device="cuda", dtype=torch.float32).to(torch.bfloat16)
    dst = torch.empty_like(src)
    nbytes = n * 2
    out = {"bytes_per_buffer": nbytes}
    t = timed(lambda: dst.copy_(src))
    out["copy_TBps"] = round(2 * nbytes / t / 1e12, 3)
    t = timed(lambda: dst.fill_(1.0))
    out["fill_TBps"] = round(nbytes / t / 1e12, 3)
    t = timed(lambda: torch.sum(src, dtype=torch.float32))
    out["sum_read_TBps"] = round(nbytes / t / 1e12, 3)
    # hand-written streaming kernels (tools/hbm_copy.hip, 16-B loads/stores, 4 in flight per lane), by grid size
    lib = ctypes.CDLL(str(Path(__file__).resolve().parent / "_hbm_copy.so"))
    lib.hbm_run.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_longlong, ctypes.c_int,
                            ctypes.c_void_p, ctypes.c_void_p]
    flag = torch.zeros(1, dtype=torch.int32, device="cuda")
    n16 = nbytes // 16
    st = torch.cuda.current_stream().cuda_stream
    # 3-7: no bounds checks (2 GiB is a multiple of every grid's pass), plain / nontemporal, 4 or 8 loads in flight
    for kind, name, mult in ((0, "hip_copy", 2), (1, "hip_read", 1), (2, "hip_fill", 1), (3, "hip_copy_nb", 2),
                             (4, "hip_copy_nb_nt", 2), (5, "hip_copy_nb_nt_u8", 2), (6, "hip_fill_nb_nt", 1),
                             (7, "hip_fill_nb", 1)):
        best = 0.0
        for blocks in (1024, 2048, 4096, 8192, 16384):
            if kind >= 3 and n16 % (blocks * 256 * 8):
                continue
            def run():
                rc = lib.hbm_run(kind, src.data_ptr(), dst.data_ptr(), n16, blocks, flag.data_ptr(), st)
                assert rc == 0, rc
            rate = mult * nbytes / timed(run) / 1e12
            out[f"{name}_{blocks}_TBps"] = round(rate, 3)
            best = max(best, rate)
        out[f"{name}_best_TBps"] = round(best, 3)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
