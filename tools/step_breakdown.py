"""Per-category kernel time of the last training step in a rocprofv3 kernel trace
(steps delimited by the AdamW launches)."""
import collections
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if "adamw" in r["Kernel_Name"]]
ends, prev = [], None
for i in idx:
    if prev is None or i - prev > 5:
        ends.append(i)
    prev = i
step = rows[ends[-2] + 2:ends[-1] + 2]
t0, t1 = int(step[0]["Start_Timestamp"]), int(step[-1]["End_Timestamp"])
print(f"launches {len(step)}  wall {(t1 - t0) / 1e3:.1f} us")


def cat(n):
    for k, key in (("conv_fwd", "conv_fwd"), ("wgrad", "wgrad"), ("gn_", "gn"), ("pack_weight", "pack"),
                   ("xattn", "xattn"), ("fold", "fold"), ("mqa", "mqa"), ("CUDAFunctor_add", "torch-add"),
                   ("at::native", "torch-other"), ("rocclr", "copy")):
        if k in n:
            return key
    return "other"


agg, per = collections.defaultdict(lambda: [0.0, 0]), collections.defaultdict(list)
for r in step:
    t = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    c = cat(r["Kernel_Name"])
    agg[c][0] += t
    agg[c][1] += 1
    per[(r["Kernel_Name"].replace("(anonymous namespace)::", "")[:60], r["Grid_Size_X"], r["Grid_Size_Y"],
         r["Grid_Size_Z"])].append(t)
for k, v in sorted(agg.items(), key=lambda kv: -kv[1][0]):
    print(f"{v[0]:9.1f} us {v[1]:4d}  {k}")
if len(sys.argv) > 2:
    for k, v in sorted(per.items(), key=lambda kv: -sum(kv[1]))[:int(sys.argv[2])]:
        print(f"{sum(v):8.1f} n={len(v):3d} avg {sum(v) / len(v):6.1f} {k}")
