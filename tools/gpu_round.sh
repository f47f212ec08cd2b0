#!/bin/bash
# One GPU-box session: GPU tests, the bench line, and a rocprofv3 kernel-trace summary of the bench.
#   gpurun --timeout 1200 -- 'bash tools/gpu_round.sh TAG [pytest selection]'
# Every GPU step has its own time limit; a fault / abort / timeout ends the script there.
TAG=${1:-run}
SEL=${2:-tests}
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
stop_on_fault() {  # pytest: 0 = pass, 1 = test failures (continue); anything else ends the session
    local rc=$1 what=$2
    echo "$what exit $rc" | tee -a "$OUT/status.txt"
    if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then exit "$rc"; fi
}
timeout -k 10 480 python -u -m pytest $SEL -m gpu -v --timeout 120 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
stop_on_fault $? pytest
tail -3 "$OUT/gpu_tests.log"
timeout -k 10 300 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; echo "bench exit $rc" | tee -a "$OUT/status.txt"; [ $rc -eq 0 ] || exit $rc
cat "$OUT/bench.json"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
    python3 "$ROOT/bench.py" --steps 10 --warmup 3 --no-cpu-baseline --no-infer --epe-steps 0 > "$OUT/prof.log" 2>&1
rc=$?; echo "rocprof exit $rc" | tee -a "$OUT/status.txt"; exit $rc
