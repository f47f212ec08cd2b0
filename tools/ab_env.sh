#!/bin/bash
# bench A/B of environment settings on one box, alternating (per-layer GEMM times in the .err files)
#   gpurun -- 'bash tools/ab_env.sh TAG "SD_X=1" "SD_X=0" [rounds]'
TAG=$1; A=$2; B=$3; R=${4:-2}
OUT=$(pwd)/gpurun_out/$TAG; mkdir -p "$OUT"
for r in $(seq 1 $R); do
  for arm in A B; do
    if [ $arm = A ]; then SET=$A; else SET=$B; fi
    env $SET SD_BENCH_LAYERS=1 timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-infer \
        > "$OUT/b_${arm}_$r.json" 2> "$OUT/b_${arm}_$r.err" || exit 3
    echo "$arm ($SET) round $r: $(grep -o '"value": [0-9.]*' "$OUT/b_${arm}_$r.json" | head -1)"
  done
done
