#!/bin/bash
# Micro-benchmark several builds of the C ABI (build_ab/<name>.so) against the in-tree one.
#   gpurun -- 'bash tools/ab_variants.sh TAG "--wgrad" name1 name2 ...'
TAG=${1:-var}
ARGS=${2:-}
shift 2
OUT=$(pwd)/gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 100 python -u tools/conv_micro.py $ARGS > "$OUT/intree.log" 2>&1 || exit 1
for v in "$@"; do
    SD_HIP_LIB=$(pwd)/build_ab/$v.so timeout -k 10 100 python -u tools/conv_micro.py $ARGS > "$OUT/$v.log" 2>&1 || exit 2
done
timeout -k 10 100 python -u tools/conv_micro.py $ARGS > "$OUT/intree2.log" 2>&1 || exit 3
for f in "$OUT"/*.log; do echo "== $(basename $f)"; cat "$f"; done
