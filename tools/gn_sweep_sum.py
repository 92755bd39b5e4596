"""Summarise tools/gn_sweep.sh: per config and gnbench case, average duration
of the four GroupNorm kernels (positional: 2 + 23x2 fwd, 23x2 bwd per case)."""
import csv
import glob
import os
import sys

CASES = ["64x64 C64", "32x32 C64", "32x32 C128", "16x16 C128", "16x16 C256", "8x8 C256", "8x8 C512"]
for d in sorted(glob.glob(os.path.join(sys.argv[1], "gns_*"))):
    f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    if not f:
        continue
    rows = [r for r in csv.DictReader(open(f[0])) if "gn_" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rows]
    print(os.path.basename(d), len(rows))
    tot = [0.0] * 4
    for i, name in enumerate(CASES):
        c = dur[i * 94:(i + 1) * 94]
        if len(c) < 94:
            break
        fw, bw = c[2 + 6:48], c[48 + 6:94]  # skip warm-up launches
        v = [sum(fw[0::2]) / len(fw[0::2]), sum(fw[1::2]) / len(fw[1::2]),
             sum(bw[0::2]) / len(bw[0::2]), sum(bw[1::2]) / len(bw[1::2])]
        tot = [a + b for a, b in zip(tot, v)]
        print(f"  {name:12s} fred {v[0]:6.1f} fapp {v[1]:6.1f} bred {v[2]:6.1f} bapp {v[3]:6.1f}")
    print(f"  {'sum':12s} fred {tot[0]:6.1f} fapp {tot[1]:6.1f} bred {tot[2]:6.1f} bapp {tot[3]:6.1f}  all {sum(tot):6.1f}")
