"""Per-kernel-family time of the last full training step in a rocprofv3
kernel_trace CSV (steps delimited by the AdamW launches):
python tools/step_families.py trace.csv [top-N]"""
import collections
import csv
import re
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "adamw" in r["Kernel_Name"]]
step = rows[idx[-3] + 1:idx[-1] + 1]
dur = lambda r: (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
c, n = collections.defaultdict(float), collections.Counter()
for r in step:
    m = re.search(r"(\w+_kernel)", r["Kernel_Name"])
    key = re.sub(r"^_ZN12_GLOBAL__N_1\d+", "", m.group(1)) if m else r["Kernel_Name"][:40]
    c[key] += dur(r)
    n[key] += 1
wall = (int(step[-1]["End_Timestamp"]) - int(step[0]["Start_Timestamp"])) / 1e3
print(f"wall {wall:.0f} us, kernel sum {sum(c.values()):.0f} us, launches {len(step)}")
for k, v in sorted(c.items(), key=lambda kv: -kv[1])[:int(sys.argv[2]) if len(sys.argv) > 2 else 25]:
    print(f"{v:8.0f} us {n[k]:4d}  {k}")
