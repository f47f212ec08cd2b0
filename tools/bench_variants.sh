#!/bin/bash
# per-layer GEMM times (bench SD_BENCH_LAYERS) of the in-tree build and of build_ab/<variant>.so builds
#   gpurun -- 'bash tools/bench_variants.sh TAG lib_a.so lib_b.so ...'
TAG=$1; shift
OUT=$(pwd)/gpurun_out/$TAG
mkdir -p "$OUT"
for v in intree "$@"; do
    if [ "$v" = intree ]; then unset SD_HIP_LIB; else export SD_HIP_LIB=$(pwd)/build_ab/$v; fi
    SD_BENCH_LAYERS=1 timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-infer \
        > "$OUT/b_$v.json" 2> "$OUT/b_$v.err" || exit 3
    grep -o '"value": [0-9.]*' "$OUT/b_$v.json" | head -1
done
unset SD_HIP_LIB
python - "$OUT" intree "$@" <<'PY'
import sys, json
out, names = sys.argv[1], sys.argv[2:]
data = {}
for n in names:
    for l in open(f"{out}/b_{n}.err"):
        if '{"layer"' in l:
            r = json.loads(l[l.index("{"):])
            data.setdefault(r["layer"], {})[n] = r["ms_per_step"] * 1000
print("layer".ljust(42), " ".join(n[-12:].rjust(12) for n in names))
for k, v in sorted(data.items(), key=lambda kv: -kv[1].get("intree", 0)):
    print(k.ljust(42), " ".join(f"{v.get(n, 0):12.1f}" for n in names))
PY
