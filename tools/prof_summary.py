"""Per-kernel time of the REPLAYED training step from a rocprofv3
--kernel-trace CSV: steps are delimited by the AdamW launch that ends each
update; the last N complete steps (default 3: the graph replays of
`bench.py --steps 5 --warmup 2 --no-roofline --no-sampling --no-fp32`) are
averaged, so warm-up, capture, the fp32 / sampling legs and the per-launch
timing steps never leak into the per-step numbers.

  python tools/prof_summary.py run_kernel_trace.csv [top-N] [N-steps]
"""
import collections
import csv
import re
import sys

path = sys.argv[1]
top = int(sys.argv[2]) if len(sys.argv) > 2 else 40
nsteps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
ends = [i for i, r in enumerate(rows) if "adamw" in r["Kernel_Name"]]
# an update launches one AdamW kernel per parameter group: a step ends at the
# last AdamW launch before the next forward
step_ends = [i for j, i in enumerate(ends) if j + 1 == len(ends) or ends[j + 1] - i > 8]
if len(step_ends) < nsteps + 1:
    sys.exit(f"only {len(step_ends)} steps in the trace")
lo, hi = step_ends[-nsteps - 1] + 1, step_ends[-1] + 1
sel = rows[lo:hi]
dur = lambda r: (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
tot, cnt = collections.defaultdict(float), collections.Counter()
for r in sel:
    name = r["Kernel_Name"]
    m = re.search(r"(\w+_kernel)(<[^(]*>)?", name)
    key = (re.sub(r"^_ZN12_GLOBAL__N_1\d+", "", m.group(1)) + (m.group(2) or "")) if m else name[:60]
    tot[key] += dur(r)
    cnt[key] += 1
wall = (int(sel[-1]["End_Timestamp"]) - int(sel[0]["Start_Timestamp"])) / 1e3 / nsteps
ksum = sum(tot.values()) / nsteps
print(f"replayed training step (mean of the last {nsteps}): wall {wall:.0f} us, kernel sum {ksum:.0f} us, "
      f"{len(sel) / nsteps:.0f} launches")
for k, v in sorted(tot.items(), key=lambda kv: -kv[1])[:top]:
    print(f"{v / nsteps:9.1f} us/step {cnt[k] / nsteps:6.1f}/step  avg {v / cnt[k]:7.1f} us  {k[:110]}")
