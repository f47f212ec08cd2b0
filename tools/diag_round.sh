#!/bin/bash
# One box session of diagnostics: B=1 960x720 inference kernel traces (fp8, bf16), the HBM calibration, and the conv
# micro-benchmark of the in-tree build beside phase-removal / cycle-counter builds (build_ab/, tools/build_variant.sh).
#   gpurun --timeout 1200 -- 'bash tools/diag_round.sh TAG [variant.so ...]'
TAG=${1:-diag}; shift
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
bash tools/infer_prof.sh "$TAG/inf" || exit $?
timeout -k 10 120 python -u tools/hbm_calib.py > "$OUT/hbm_calib.json" 2> "$OUT/hbm_calib.err" || exit 3
cat "$OUT/hbm_calib.json"
timeout -k 10 150 python -u tools/conv_micro.py > "$OUT/micro_intree.log" 2>&1 || exit 4
for v in "$@"; do
    if [ "$v" = "libstereo_hip_diag.so" ]; then
        SD_WG_DIAG=1 SD_HIP_LIB=$ROOT/build_ab/$v timeout -k 10 150 python -u tools/conv_micro.py > "$OUT/micro_$v.log" 2>&1 || exit 5
    else
        SD_HIP_LIB=$ROOT/build_ab/$v timeout -k 10 150 python -u tools/conv_micro.py > "$OUT/micro_$v.log" 2>&1 || exit 5
    fi
done
echo done
