#!/bin/bash
# GPU tests of the conv kernels, the conv micro-benchmark of the in-tree build against build_ab/<old>.so, and
# the per-wave cycle counters of the timing build build_ab/libstereo_hip_e1024.so (-DWG_EXP=1024).
#   gpurun -- 'bash tools/conv_diag.sh TAG [build_ab/libstereo_hip_prev.so]'
TAG=${1:-diag}
OLD=$(pwd)/${2:-build_ab/libstereo_hip_prev.so}
OUT=$(pwd)/gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -k "conv3x3 or halo" --timeout 120 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1 || { echo "tests rc $?"; tail -n 30 "$OUT/gpu_tests.log"; exit 1; }
tail -n 1 "$OUT/gpu_tests.log"
for arm in new old; do
    case $arm in old*) export SD_HIP_LIB=$OLD ;; *) unset SD_HIP_LIB ;; esac
    timeout -k 10 150 python -u tools/conv_micro.py > "$OUT/micro_$arm.log" 2>&1 || exit 2
done
SD_HIP_LIB=$(pwd)/build_ab/libstereo_hip_e1024.so SD_WG_DIAG=1 timeout -k 10 150 python -u tools/conv_micro.py > "$OUT/diag.log" 2>&1 || exit 3
unset SD_HIP_LIB
paste -d'|' <(cut -c1-60 "$OUT/micro_new.log") <(cut -c30-60 "$OUT/micro_old.log")
grep diag "$OUT/diag.log"
