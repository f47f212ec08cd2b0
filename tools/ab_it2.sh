#!/bin/bash
# halo conv two-items-per-pass (SD_HALO_IT=2) : GPU conv tests under it, then bench A/B on one box
OUT=$(pwd)/gpurun_out/ab_it2; mkdir -p "$OUT"
SD_HALO_IT=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py -x -q --timeout 120 --timeout-method thread > "$OUT/tests.log" 2>&1
rc=$?; tail -2 "$OUT/tests.log"; [ $rc -eq 0 ] || exit $rc
bash tools/ab_env.sh ab_it2b "SD_HALO_IT=2" "SD_HALO_IT=1" 2
