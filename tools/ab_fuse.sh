#!/bin/bash
# per-layer GEMM times with the fused BN-backward wgrad on / off, alternating, same box
OUT=gpurun_out/ab_fuse; mkdir -p $OUT
for r in 1 2; do
for f in 1 0; do
  SD_BN_FUSE=$f SD_BENCH_LAYERS=1 timeout -k 10 200 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-infer > $OUT/b_${f}_$r.json 2> $OUT/b_${f}_$r.err || exit $?
  grep -o '"value": [0-9.]*' $OUT/b_${f}_$r.json
done
done
