"""Per-step GPU busy time from a rocprofv3 kernel trace of bench.py (steps delimited by the step prologue:
k_step_prologue, or k_pack_multi in traces of builds before it / SD_PROLOGUE=0).

    python tools/step_busy.py gpurun_out/<tag>/prof/run_kernel_trace.csv [...]
"""
import csv
import statistics
import sys


def step_busy(path):
    rows = list(csv.DictReader(open(path)))
    names = [r["Kernel_Name"] for r in rows]
    idx = [i for i, n in enumerate(names) if "k_step_prologue" in n]
    if len(idx) < 6:
        idx = [i for i, n in enumerate(names) if "k_pack_multi" in n]
    busy, wall = [], []
    for a, b in zip(idx[3:-2], idx[4:-1]):  # regular training steps (skip warmup and the tail)
        busy.append(sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows[a:b]) / 1e3)
        wall.append((int(rows[b]["Start_Timestamp"]) - int(rows[a]["Start_Timestamp"])) / 1e3)
    return statistics.median(busy), statistics.median(wall), len(busy)


if __name__ == "__main__":
    for p in sys.argv[1:]:
        b, w, n = step_busy(p)
        print(f"{p}: busy {b:.0f} us, wall {w:.0f} us per step (median of {n})")
