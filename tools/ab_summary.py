"""Summarise a tools/ab_lib.sh directory: per-layer micro times (mean of the two runs per arm) and bench values."""
import json
import re
import sys
from pathlib import Path

d = Path(sys.argv[1])


def micro(arm_files):
    rows = {}
    for f in arm_files:
        if not f.exists():
            continue
        for line in f.read_text().splitlines():
            m = re.match(r"^(wgrad .*?|\d+x\d+ .*?)[:|] .*?(\d+\.\d+) us", line)
            if m:
                rows.setdefault(m.group(1).strip(), []).append(float(m.group(2)))
    return {k: sum(v) / len(v) for k, v in rows.items()}


for kind in ("micro", "wgrad"):
    a = micro([d / f"{kind}_new.log", d / f"{kind}_new2.log"])
    b = micro([d / f"{kind}_old.log", d / f"{kind}_old2.log"])
    for k in a:
        if k in b:
            print(f"{k:40s} new {a[k]:8.1f} us  old {b[k]:8.1f} us  {100 * (b[k] / a[k] - 1):+5.1f}%")
for arm in ("new", "old", "new2", "old2"):
    j = json.loads((d / f"bench_{arm}.json").read_text())
    print(arm, j["value"], j["ms_per_step"])
