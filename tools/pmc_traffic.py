"""Per-kernel HBM traffic from two rocprofv3 PMC passes of the same bench command.

    cd /tmp && export TMPDIR=/tmp
    rocprofv3 --pmc FETCH_SIZE --output-format csv -d OUT/f -o fetch -- python3 bench.py --steps 2 --warmup 1
    rocprofv3 --pmc WRITE_SIZE --output-format csv -d OUT/w -o write -- python3 bench.py --steps 2 --warmup 1
    python tools/pmc_traffic.py OUT/f/fetch_counter_collection.csv OUT/w/write_counter_collection.csv \
        > profiles/<round>_pmc_traffic.json

Units and gfx950 corrections (MI355X_MICROARCH.md, HBM section), checked here on kernels with
known byte counts (k_bn_bwd_apply, k_pack_input, k_count_valid): both counters are in KiB;
WRITE_SIZE is exact for 16-B-per-lane stores; FETCH_SIZE reports half the bytes of wide
coalesced reads, so it is doubled. bytes/launch = 1024 * (2 * FETCH_SIZE + WRITE_SIZE),
averaged over a kernel's launches (the same averaging as bench.py's per-kernel timing).
"""

from __future__ import annotations

import csv
import json
import re
import sys
from collections import defaultdict


def short_name(name: str) -> str:
    """'void (anonymous namespace)::k_halo_conv<2, 8>((anonymous namespace)::HFwdArgs)' -> 'k_halo_conv<2, 8>'."""
    n = name.replace("(anonymous namespace)::", "")
    n = re.sub(r"^void ", "", n)
    depth, out = 0, []
    for ch in n:  # cut the argument list, keep template arguments
        if ch == "(" and depth == 0:
            break
        depth += ch == "<"
        depth -= ch == ">"
        out.append(ch)
    return "".join(out).strip()


def per_dispatch(path: str, counter: str) -> dict[int, tuple[str, float]]:
    out = {}
    with open(path) as f:
        for r in csv.DictReader(f):
            if r["Counter_Name"] == counter:
                out[int(r["Dispatch_Id"])] = (short_name(r["Kernel_Name"]), float(r["Counter_Value"]))
    return out


def main(fetch_csv: str, write_csv: str):
    fetch = per_dispatch(fetch_csv, "FETCH_SIZE")
    write = per_dispatch(write_csv, "WRITE_SIZE")
    agg = defaultdict(lambda: [0, 0.0, 0])
    for _, (k, v) in fetch.items():
        agg[k][0] += 1
        agg[k][1] += 2.0 * 1024.0 * v
    wagg = defaultdict(lambda: [0, 0.0])
    for _, (k, v) in write.items():
        wagg[k][0] += 1
        wagg[k][1] += 1024.0 * v
    res = {}
    for k in sorted(set(agg) | set(wagg)):
        nf, fb, _ = agg.get(k, [0, 0.0, 0])
        nw, wb = wagg.get(k, [0, 0.0])
        rd = fb / nf if nf else None
        wr = wb / nw if nw else None
        res[k] = {"launches_fetch_pass": nf, "launches_write_pass": nw, "read_bytes_per_launch": rd,
                  "write_bytes_per_launch": wr,
                  "hbm_bytes_per_launch": (rd or 0.0) + (wr or 0.0) if rd is not None and wr is not None else None}
    import hashlib
    import os

    lib = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "stereo_depth_estimation_amd", "libstereo_hip.so")
    with open(lib, "rb") as f:
        sha = hashlib.sha256(f.read()).hexdigest()
    # bench.py reports a kernel's traffic only when this matches the library it loaded (same build)
    json.dump({"source": [fetch_csv, write_csv], "correction": "bytes = 1024*(2*FETCH_SIZE + WRITE_SIZE)",
               "lib_sha256": sha, "kernels": res}, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
