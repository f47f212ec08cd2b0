#!/bin/bash
# Conv and wgrad micro-benchmarks of several builds (build_ab/<name>.so), in-tree first and last.
#   gpurun -- 'bash tools/ab_variants2.sh TAG name1 name2 ...'
TAG=${1:-var}
shift 1
OUT=$(pwd)/gpurun_out/$TAG
mkdir -p "$OUT"
run() {  # $1 = label, $2 = library path or empty
    SD_HIP_LIB=$2 timeout -k 10 100 python -u tools/conv_micro.py > "$OUT/$1.conv.log" 2>&1 || exit 1
    SD_HIP_LIB=$2 timeout -k 10 100 python -u tools/conv_micro.py --wgrad > "$OUT/$1.wgrad.log" 2>&1 || exit 2
}
run intree ""
for v in "$@"; do run "$v" "$(pwd)/build_ab/$v.so"; done
run intree2 ""
python3 - "$OUT" "$@" <<'PY'
import re, sys
from pathlib import Path
d = Path(sys.argv[1]); arms = ["intree"] + sys.argv[2:] + ["intree2"]
def rows(a):
    r = {}
    for kind in ("conv", "wgrad"):
        for line in (d / f"{a}.{kind}.log").read_text().splitlines():
            m = re.match(r"^(wgrad .*?|\d+x\d+ .*?)[:|] .*?(\d+\.\d+) us", line)
            if m: r[m.group(1).strip()] = float(m.group(2))
    return r
R = {a: rows(a) for a in arms}
print(f"{'layer':34s}" + "".join(f"{a[:16]:>17s}" for a in arms))
for k in R["intree"]:
    print(f"{k:34s}" + "".join(f"{R[a].get(k, float('nan')):17.1f}" for a in arms))
PY
