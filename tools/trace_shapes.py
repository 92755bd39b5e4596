"""Per-(kernel, grid) time from a rocprofv3 kernel trace: python tools/trace_shapes.py trace.csv N [filter...]
(N = forward / step count the trace holds, to print per-unit times)."""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
n = float(sys.argv[2])
flt = sys.argv[3:]
d = collections.defaultdict(list)
for r in rows:
    name = r["Kernel_Name"]
    if flt and not any(f in name for f in flt):
        continue
    short = name.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0][:60]
    d[(short, r["Grid_Size_X"], r["Grid_Size_Y"], r["Grid_Size_Z"], r["VGPR_Count"])].append(
        int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
tot = sum(sum(v) for v in d.values())
print(f"total {tot / n / 1e3:.1f} us per unit")
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1]))[:40]:
    print(f"{sum(v) / n / 1e3:8.1f} us  n={len(v) / n:5.1f}  avg={sum(v) / len(v) / 1e3:7.2f} us  {k}")
