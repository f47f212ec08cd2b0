#!/bin/bash
# The round's committed evidence from one GPU session, all from the same library build:
# bench line (full: EPE, inference, CPU baseline), rocprofv3 kernel-trace stats of a 10-step bench, the PMC
# traffic passes (tools/pmc_round.sh), the SQ pass (tools/pmc_sq.sh) and the stall pass (tools/pmc_stall.sh).
#   gpurun --timeout 1200 -- 'bash tools/profile_round.sh TAG'
# Every GPU step has its own time limit; a failure ends the script there.
TAG=${1:-prof}
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
timeout -k 10 300 python -u bench.py > "$OUT/bench.json" 2> "$OUT/bench.err" || exit $?
tail -c 400 "$OUT/bench.json"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
    python3 "$ROOT/bench.py" --steps 10 --warmup 3 --no-cpu-baseline --no-infer --epe-steps 0 > "$OUT/prof.log" 2>&1 || exit $?
cd "$ROOT"
bash tools/pmc_round.sh "${TAG}_tr" || exit $?
bash tools/pmc_sq.sh "${TAG}_sq" || exit $?
bash tools/pmc_stall.sh "${TAG}_st" || exit $?
echo "profile_round done"
