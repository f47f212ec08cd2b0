#!/bin/bash
# Kernel-trace A/B of the in-tree library against another build (same C ABI): rocprofv3 --kernel-trace --stats of a
# short bench for each, alternating twice, then per-kernel average durations side by side.
#   gpurun -- 'bash tools/prof_ab.sh TAG build_ab/lib_old.so'
TAG=${1:-pab}; OLD=$(pwd)/${2:-build_ab/lib_old.so}
ROOT=$(pwd); OUT=$ROOT/gpurun_out/$TAG; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for r in 1 2; do
  for arm in new old; do
    if [ $arm = old ]; then export SD_HIP_LIB=$OLD; else unset SD_HIP_LIB; fi
    timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/${arm}_$r" -o run -- \
        python3 "$ROOT/bench.py" --steps 10 --warmup 3 --no-cpu-baseline --no-infer --no-roofline > "$OUT/${arm}_$r.log" 2>&1
    rc=$?; echo "$arm $r exit $rc"; [ $rc -eq 0 ] || exit $rc
  done
done
unset SD_HIP_LIB
cd "$ROOT" && python3 - "$OUT" <<'PY'
import csv, glob, re, sys
out = sys.argv[1]
def load(arm):
    acc = {}
    for r in (1, 2):
        f = glob.glob(f"{out}/{arm}_{r}/**/*kernel_stats.csv", recursive=True)[0]
        for row in csv.DictReader(open(f)):
            c, t = acc.get(row["Name"], (0, 0.0))
            acc[row["Name"]] = (c + int(row["Calls"]), t + float(row["TotalDurationNs"]))
    return acc
a, b = load("old"), load("new")
rows = []
for k in set(a) | set(b):
    (ca, ta), (cb, tb) = a.get(k, (0, 0.0)), b.get(k, (0, 0.0))
    rows.append((tb - ta, k, ta / max(ca, 1), tb / max(cb, 1), ca, cb))
for d, k, ua, ub, ca, cb in sorted(rows)[:25]:
    name = re.sub(r"\(\(anonymous namespace\)::\w+\)", "", k).replace("(anonymous namespace)::", "")[:90]
    print(f"{d / 1e3:+10.1f} us total  avg {ua / 1e3:8.1f} -> {ub / 1e3:8.1f} us  calls {ca}->{cb}  {name}")
print("total ms", round(sum(v[1] for v in a.values()) / 1e6, 2), "->", round(sum(v[1] for v in b.values()) / 1e6, 2))
PY
