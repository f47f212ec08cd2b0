#!/bin/bash
# conv micro-benchmark of the in-tree build and of build_ab/<variant>.so builds, one log each
#   gpurun -- 'bash tools/micro_variants.sh TAG libstereo_hip_a.so libstereo_hip_b.so ...'
TAG=$1; shift
OUT=$(pwd)/gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 150 python -u tools/conv_micro.py > "$OUT/micro_intree.log" 2>&1 || exit 2
for v in "$@"; do
    SD_HIP_LIB=$(pwd)/build_ab/$v timeout -k 10 150 python -u tools/conv_micro.py > "$OUT/micro_$v.log" 2>&1 || exit 3
done
python - "$OUT" "$@" <<'PY'
import sys, re
out, names = sys.argv[1], ["intree"] + sys.argv[2:]
data = {}
for n in names:
    for line in open(f"{out}/micro_{n}.log"):
        m = re.match(r"(\S+ \S+ \S+)\s*\|.*?>\s+([\d.]+) us", line)
        if m: data.setdefault(m.group(1), []).append(float(m.group(2)))
print("layer".ljust(24), " ".join(n[-14:].rjust(14) for n in names))
for k, v in data.items(): print(k.ljust(24), " ".join(f"{x:14.1f}" for x in v))
print("sum".ljust(24), " ".join(f"{sum(v[i] for v in data.values()):14.1f}" for i in range(len(names))))
PY
