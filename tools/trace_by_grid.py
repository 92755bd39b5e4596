"""Per (kernel, grid) average duration from a rocprofv3 kernel_trace CSV:
python tools/trace_by_grid.py trace.csv [name-substring] [last-N-dispatches]"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
pat = sys.argv[2] if len(sys.argv) > 2 else ""
if len(sys.argv) > 3:
    rows = rows[-int(sys.argv[3]):]
agg = defaultdict(list)
for r in rows:
    if pat in r["Kernel_Name"]:
        key = (r["Kernel_Name"][:60], r["Grid_Size_X"], r["Grid_Size_Y"], r["Grid_Size_Z"], r["Workgroup_Size_X"])
        agg[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
    print(f"{sum(v):9.1f} us  n={len(v):4d} avg {sum(v)/len(v):7.1f}  {k}")
