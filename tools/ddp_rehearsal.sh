#!/bin/bash
# The bench's N > 1 path (DataParallel buckets, async count all-reduce, barriers, max-over-ranks timing, rank-0 JSON)
# rehearsed on a one-GPU box: 2 ranks over gloo, both on cuda:0. Not a scaling measurement.
#   gpurun -- 'bash tools/ddp_rehearsal.sh TAG'
OUT=$(pwd)/gpurun_out/${1:-ddp}
EXTRA=${2:-}  # e.g. --sync-bn
mkdir -p "$OUT"
SD_BENCH_SHARE_DEVICE=1 timeout -k 10 300 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 5 --warmup 2 $EXTRA \
    > "$OUT/bench2.json" 2> "$OUT/bench2.err"
rc=$?; echo "ddp rehearsal exit $rc"; cat "$OUT/bench2.json"; exit $rc
