OUT=gpurun_out/r03_e4; mkdir -p $OUT
run() { if [ "$1" = intree ]; then timeout -k 10 150 python -u tools/conv_micro.py > $OUT/micro_$2.log 2>&1; else SD_HIP_LIB=$PWD/build_ab/libstereo_hip_$1.so timeout -k 10 150 python -u tools/conv_micro.py > $OUT/micro_$2.log 2>&1; fi; }
run intree a1 && run epl0 b1 && run epl0nt c1 && run epl1nt d1 && run epl0noepi e1 && run intree a2 && run epl0 b2 && run epl0nt c2 && run epl1nt d2 || exit 3
python - <<'P'
import re
out="gpurun_out/r03_e4"; names=["a1","b1","c1","d1","e1","a2","b2","c2","d2"]
data={}
for n in names:
    for line in open(f"{out}/micro_{n}.log"):
        m=re.match(r"(\S+ \S+ \S+)\s*\|.*?>\s+([\d.]+) us", line)
        if m: data.setdefault(m.group(1),[]).append(float(m.group(2)))
print("layer".ljust(22)," ".join(n.rjust(7) for n in names))
for k,v in data.items(): print(k.ljust(22)," ".join(f"{x:7.1f}" for x in v))
print("sum".ljust(22)," ".join(f"{sum(v[i] for v in data.values()):7.1f}" for i in range(len(names))))
P
