#!/bin/bash
# bench A/B/C/... of environment settings on one box, arms alternating per round (per-layer GEMM times in the .err)
#   gpurun -- 'bash tools/ab_arms.sh TAG ROUNDS "SD_X=1" "SD_X=0" "SD_Y=2" ...'   ("-" = no extra setting)
TAG=$1; R=$2; shift 2
OUT=$(pwd)/gpurun_out/$TAG; mkdir -p "$OUT"
for r in $(seq 1 $R); do
  i=0
  for SET in "$@"; do
    i=$((i + 1))
    [ "$SET" = "-" ] && SET="SD_NONE=1"
    env $SET SD_BENCH_LAYERS=1 timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-infer \
        > "$OUT/b_${i}_$r.json" 2> "$OUT/b_${i}_$r.err" || exit 3
    echo "arm $i ($SET) round $r: $(grep -o '"value": [0-9.]*' "$OUT/b_${i}_$r.json" | head -1)"
  done
done
