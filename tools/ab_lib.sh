#!/bin/bash
# A/B of the in-tree library against another build of the same C ABI (build_ab/<name>.so):
# conv/wgrad micro-benchmarks and bench lines, alternating, then the GPU tests of the in-tree build.
#   gpurun -- 'bash tools/ab_lib.sh TAG build_ab/libstereo_hip_old.so [pytest -k expr]'
TAG=${1:-ab}
OLD=$(pwd)/${2:-build_ab/libstereo_hip_old.so}
K=${3:-}
OUT=$(pwd)/gpurun_out/$TAG
mkdir -p "$OUT"
for arm in new old new2 old2; do
    case $arm in old*) export SD_HIP_LIB=$OLD ;; *) unset SD_HIP_LIB ;; esac
    timeout -k 10 150 python -u tools/conv_micro.py > "$OUT/micro_$arm.log" 2>&1 || { echo "micro $arm rc $?"; tail -n 20 "$OUT/micro_$arm.log"; exit 2; }
done
for arm in new old new2 old2; do
    case $arm in old*) export SD_HIP_LIB=$OLD ;; *) unset SD_HIP_LIB ;; esac
    timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-infer --epe-steps 0 > "$OUT/bench_$arm.json" 2> "$OUT/bench_$arm.err" || exit 4
done
unset SD_HIP_LIB
python tools/ab_summary.py "$OUT"
timeout -k 10 400 python -u -m pytest tests -m gpu -q ${K:+-k "$K"} --timeout 120 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
rc=$?; echo "tests rc $rc"; tail -n 15 "$OUT/gpu_tests.log"; exit $rc
