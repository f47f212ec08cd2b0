#!/bin/bash
# One rocprofv3 PMC pass (kernel trace only) of the issue-stall counters of a short bench: where the waves' cycles go
# (SQ_WAIT_INST_ANY issue stalls, of them SQ_WAIT_INST_LDS; SQ_ACTIVE_INST_*; LDS FIFO-full cycles), per kernel.
#   gpurun --timeout 600 -- 'bash tools/pmc_stall.sh TAG'
TAG=${1:-stall}
ROOT=$(pwd)
OUT=$ROOT/gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY \
    SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL GRBM_GUI_ACTIVE --output-format csv \
    -d "$OUT/st" -o st -- \
    python3 "$ROOT/bench.py" --steps 2 --warmup 1 --no-cpu-baseline --no-infer --no-roofline --epe-steps 0 > "$OUT/st.log" 2>&1
rc=$?; echo "stall exit $rc" | tee -a "$OUT/status.txt"; [ $rc -eq 0 ] || exit $rc
cd "$ROOT" && python3 - "$OUT" <<'PY' > "$OUT/pmc_stall.json"
import csv, glob, json, sys
from collections import defaultdict
sys.path.insert(0, "tools")
from pmc_traffic import short_name
out = sys.argv[1]
per, names = defaultdict(lambda: defaultdict(float)), {}
for r in csv.DictReader(open(glob.glob(out + "/st/*counter_collection.csv")[0])):
    d = int(r["Dispatch_Id"]); names[d] = short_name(r["Kernel_Name"])
    per[d][r["Counter_Name"]] += float(r["Counter_Value"])
agg = defaultdict(lambda: defaultdict(float)); n = defaultdict(int)
for d, cs in per.items():
    n[names[d]] += 1
    for k, v in cs.items(): agg[names[d]][k] += v
res = {}
for k, cs in agg.items():
    wc = cs.get("SQ_WAVE_CYCLES", 0.0)
    if wc <= 0: continue
    gui = cs.get("GRBM_GUI_ACTIVE", 0.0) / 8
    res[k] = {"launches": n[k], "wait_inst_any": cs["SQ_WAIT_INST_ANY"] / wc, "wait_inst_lds": cs["SQ_WAIT_INST_LDS"] / wc,
              "active_inst_any": cs["SQ_ACTIVE_INST_ANY"] / wc, "active_inst_lds": cs["SQ_ACTIVE_INST_LDS"] / wc,
              "active_inst_valu": cs["SQ_ACTIVE_INST_VALU"] / wc,
              "lds_data_fifo_full_per_cu_cycle": cs["SQ_LDS_DATA_FIFO_FULL"] / (256 * gui) if gui else None,
              "lds_cmd_fifo_full_per_cu_cycle": cs["SQ_LDS_CMD_FIFO_FULL"] / (256 * gui) if gui else None}
print(json.dumps({"source": "rocprofv3 --pmc (kernel trace only), bench.py --steps 2; ratios to SQ_WAVE_CYCLES "
                  "(quad-cycles summed over waves), FIFO-full counts per CU cycle (GRBM_GUI_ACTIVE / 8 XCDs)",
                  "kernels": dict(sorted(res.items(), key=lambda kv: -kv[1]["launches"]))}, indent=1))
PY
