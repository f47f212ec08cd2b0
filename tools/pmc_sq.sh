#!/bin/bash
# One rocprofv3 PMC pass (SQ + GRBM counters, kernel trace only) of a short bench, summarised into
# MFMA-busy / LDS-busy fractions per kernel by tools/pmc_sq.py.
#   gpurun --timeout 600 -- 'bash tools/pmc_sq.sh TAG'
TAG=${1:-sq}
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > "$OUT/avail.txt" 2>&1
for c in SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE; do
    grep -q "$c" "$OUT/avail.txt" || { echo "counter $c not listed"; exit 3; }
done
timeout -k 10 240 rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_LDS_BANK_CONFLICT \
    SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE --output-format csv -d "$OUT/sq" -o sq -- \
    python3 "$ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --no-infer --no-roofline --epe-steps 0 > "$OUT/sq.log" 2>&1
rc=$?; echo "sq exit $rc" | tee -a "$OUT/status.txt"; [ $rc -eq 0 ] || exit $rc
cd "$ROOT" && python3 tools/pmc_sq.py $(ls "$OUT"/sq/*counter_collection.csv) $(ls "$OUT"/sq/*kernel_trace.csv) > "$OUT/pmc_sq.json"
