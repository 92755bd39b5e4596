"""Per-kernel PMC table from a rocprofv3 SQ/GRBM counter pass (+ optional
traffic JSON of tools/pmc_traffic.py):

  python tools/pmc_sq.py sq_counter_collection.csv [traffic.json]

Columns per kernel (averages per dispatch):
  mfma_busy  SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 * 1024 SIMDs):
             the fraction of the chip's SIMD-cycles during the dispatch the
             MFMA pipe was busy (GRBM_GUI_ACTIVE sums the 8 XCDs;
             SQ_VALU_MFMA_BUSY_CYCLES counts cycles, 32 per 32x32x16 bf16 MFMA,
             MI355X_MICROARCH.md §per-instruction constants)
  valu/mfma  SQ_INSTS_VALU / SQ_INSTS_MFMA (VALU instructions per MFMA)
  lds/mfma   SQ_INSTS_LDS / SQ_INSTS_MFMA
  conflict   SQ_LDS_BANK_CONFLICT cycles per LDS instruction
  wait_inst  SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES (issue-stall share of wave time)
  MB         HBM bytes per dispatch (2*FETCH_SIZE + WRITE_SIZE, traffic JSON)
"""
import csv
import json
import re
import sys
from collections import defaultdict

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from pmc_traffic import norm  # noqa: E402

rows = defaultdict(lambda: defaultdict(list))
disp = defaultdict(set)
for r in csv.DictReader(open(sys.argv[1])):
    k = norm(r["Kernel_Name"])
    rows[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    disp[k].add(r.get("Dispatch_Id", r.get("Correlation_Id", "")))
traffic = json.load(open(sys.argv[2])) if len(sys.argv) > 2 else {}
tmap = {norm(k): v for k, v in traffic.items()}


def avg(d, n):
    v = d.get(n)
    return sum(v) / len(v) if v else float("nan")


out = []
for k, d in rows.items():
    mfma = avg(d, "SQ_VALU_MFMA_BUSY_CYCLES")
    gui = avg(d, "GRBM_GUI_ACTIVE")
    imf = avg(d, "SQ_INSTS_MFMA")
    ivalu = avg(d, "SQ_INSTS_VALU")
    ilds = avg(d, "SQ_INSTS_LDS")
    busy = mfma / (gui / 8 * 1024) if gui == gui and gui > 0 else float("nan")
    t = tmap.get(k, {}).get("traffic_bytes")
    out.append((gui, k, len(disp[k]), busy, ivalu / imf if imf else float("nan"),
                ilds / imf if imf else float("nan"),
                avg(d, "SQ_LDS_BANK_CONFLICT") / ilds if ilds else float("nan"),
                avg(d, "SQ_WAIT_INST_ANY") / avg(d, "SQ_WAVE_CYCLES"), t))
print(f"{'kernel':46s} {'n':>4s} {'gui_cyc':>9s} {'mfma_busy':>9s} {'valu/mfma':>9s} {'lds/mfma':>8s} "
      f"{'confl':>6s} {'waitI':>6s} {'MB':>8s}")
for gui, k, n, busy, vm, lm, cf, wi, t in sorted(out, key=lambda r: -r[0] * len(r)):
    name = f"{k[0]}<{','.join(map(str, k[1]))}>" if k[1] else k[0]
    print(f"{name[:46]:46s} {n:4d} {gui:9.0f} {busy:9.3f} {vm:9.2f} {lm:8.2f} {cf:6.2f} {wi:6.2f} "
          f"{(t or 0) / 1e6:8.2f}")
