#!/bin/bash
# Two rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE; separate runs, kernel trace only) of a short
# bench, summarised into profiles/pmc_traffic.json by tools/pmc_traffic.py.
#   gpurun --timeout 600 -- 'bash tools/pmc_round.sh TAG'
TAG=${1:-pmc}
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/f" -o fetch -- \
    python3 "$ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --no-infer --no-roofline --epe-steps 0 > "$OUT/fetch.log" 2>&1
rc=$?; echo "fetch exit $rc" | tee -a "$OUT/status.txt"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/w" -o write -- \
    python3 "$ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --no-infer --no-roofline --epe-steps 0 > "$OUT/write.log" 2>&1
rc=$?; echo "write exit $rc" | tee -a "$OUT/status.txt"; [ $rc -eq 0 ] || exit $rc
cd "$ROOT" && python3 tools/pmc_traffic.py $(ls "$OUT"/f/*counter_collection.csv) $(ls "$OUT"/w/*counter_collection.csv) > "$OUT/pmc_traffic.json"
