#!/bin/bash
# Bench lines of the in-tree library and build_ab/ variants, alternating for R rounds (same box), then a summary.
#   gpurun -- 'bash tools/ab_bench_libs.sh TAG R libstereo_hip_a.so ...'
TAG=$1; R=$2; shift 2
OUT=$(pwd)/gpurun_out/$TAG
mkdir -p "$OUT"
for r in $(seq 1 "$R"); do
    for v in intree "$@"; do
        if [ "$v" = intree ]; then unset SD_HIP_LIB; else export SD_HIP_LIB=$(pwd)/build_ab/$v; fi
        timeout -k 10 200 python -u bench.py --steps 30 --warmup 5 --no-cpu-baseline --no-infer --epe-steps 0 \
            > "$OUT/bench_${v}_$r.json" 2> "$OUT/bench_${v}_$r.err" || exit 4
    done
done
unset SD_HIP_LIB
python - "$OUT" "$R" intree "$@" <<'P'
import json, sys
out, R, names = sys.argv[1], int(sys.argv[2]), sys.argv[3:]
for n in names:
    v = [json.load(open(f"{out}/bench_{n}_{r}.json"))["value"] for r in range(1, R + 1)]
    print(f"{n:32s} " + " ".join(f"{x:8.1f}" for x in v) + f"   best {max(v):8.1f}")
P
