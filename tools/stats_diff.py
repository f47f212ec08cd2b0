"""Per-kernel time difference between two rocprofv3 kernel-stats runs of the bench profile
(gpurun_out/<tag>/prof/**/*kernel_stats.csv), per profiled step."""
import csv, glob, re, sys

def load(tag):
    f = glob.glob(f"gpurun_out/{tag}/prof/**/*kernel_stats.csv", recursive=True)[0]
    return {r["Name"]: (int(r["Calls"]), float(r["TotalDurationNs"])) for r in csv.DictReader(open(f))}

def short(n):
    n = re.sub(r"\(\(anonymous namespace\)::\w+\)", "", n)
    return n.replace("(anonymous namespace)::", "")[:80]

a, b = load(sys.argv[1]), load(sys.argv[2])
steps = float(sys.argv[3]) if len(sys.argv) > 3 else 23.0
rows = []
for k in set(a) | set(b):
    ca, ta = a.get(k, (0, 0.0))
    cb, tb = b.get(k, (0, 0.0))
    rows.append((tb - ta, k, ta, tb, ca, cb))
for d, k, ta, tb, ca, cb in sorted(rows):
    if abs(d) / 1e3 / steps > 2:
        print(f"{d / 1e3 / steps:+8.1f} us/step  {ta / 1e3 / steps:8.1f} -> {tb / 1e3 / steps:8.1f}  calls {ca}->{cb}  {short(k)}")
print("total ms/step", round(sum(v[1] for v in a.values()) / 1e6 / steps, 3), "->",
      round(sum(v[1] for v in b.values()) / 1e6 / steps, 3))
