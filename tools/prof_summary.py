"""Summarise a rocprofv3 --kernel-trace --stats CSV: per-kernel ms/step."""
import csv
import sys

path, steps = sys.argv[1], float(sys.argv[2])
rows = list(csv.DictReader(open(path)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total kernel time per step: {tot / 1e6 / steps:.3f} ms over {int(sum(int(r['Calls']) for r in rows) / steps)} launches")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[: int(sys.argv[3]) if len(sys.argv) > 3 else 25]:
    print(f"{float(r['TotalDurationNs']) / 1e6 / steps:8.3f} ms/step  {int(r['Calls']) / steps:6.1f}/step  "
          f"avg {float(r['AverageNs']) / 1e3:7.1f} us  {r['Name'][:100]}")
