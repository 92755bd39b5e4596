"""Per (kernel, grid) averages of the counters tools/frame_pmc.sh collects over
tools/frame_ab.py, with the window conv's chip-time fractions:

  python tools/frame_pmc.py pass1_counter_collection.csv pass2_counter_collection.csv

  mfma     SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 * 1024 SIMDs)
  lds/cu   SQ_LDS_IDX_ACTIVE / (GRBM_GUI_ACTIVE / 8 * 256 CUs): LDS-array busy
           share if the counter sums cycles over CUs (x4 if it counts quads)
  ldsI     SQ_INSTS_LDS per dispatch (LDS instructions, all waves)
  wLDS     SQ_WAIT_INST_LDS / SQ_WAVE_CYCLES (LDS issue stall share)
  wAny     SQ_WAIT_ANY / SQ_WAVE_CYCLES (parked at s_waitcnt / barrier)
  wInst    SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES (any issue stall)
  act      SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES"""
import csv
import sys
from collections import defaultdict

acc = defaultdict(lambda: defaultdict(list))
for path in sys.argv[1:]:
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"]
        if "frame" not in name and "stripe" not in name:
            continue
        # mangled: keep the kernel name and its template arguments
        short = (name.split("N_1")[-1].split("EvNS_")[0] if "_ZN" in name
                 else name.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0])[-60:]
        grid = r.get("Grid_Size", r.get("Grid_Size_X", "?"))
        acc[(short, grid)][r["Counter_Name"]].append(float(r["Counter_Value"]))


def a(d, n):
    v = d.get(n)
    return sum(v) / len(v) if v else float("nan")


print(f"{'kernel':60s} {'grid':>8s} {'n':>4s} {'mfma':>6s} {'lds/cu':>7s} {'ldsI':>9s} {'confl':>8s} "
      f"{'wLDS':>6s} {'wAny':>6s} {'wInst':>6s} {'act':>6s} {'actLDS':>7s} {'dFIFO':>8s} {'cFIFO':>8s}")
for (k, g), d in sorted(acc.items()):
    gui = a(d, "GRBM_GUI_ACTIVE")
    wc = a(d, "SQ_WAVE_CYCLES")
    n = max(len(v) for v in d.values())
    print(f"{k:60s} {g:>8s} {n:4d} {a(d, 'SQ_VALU_MFMA_BUSY_CYCLES') / (gui / 8 * 1024):6.3f} "
          f"{a(d, 'SQ_LDS_IDX_ACTIVE') / (gui / 8 * 256):7.3f} {a(d, 'SQ_INSTS_LDS'):9.0f} "
          f"{a(d, 'SQ_LDS_BANK_CONFLICT'):8.0f} {a(d, 'SQ_WAIT_INST_LDS') / wc:6.3f} {a(d, 'SQ_WAIT_ANY') / wc:6.3f} "
          f"{a(d, 'SQ_WAIT_INST_ANY') / wc:6.3f} {a(d, 'SQ_ACTIVE_INST_ANY') / wc:6.3f} "
          f"{a(d, 'SQ_ACTIVE_INST_LDS') / wc:7.3f} {a(d, 'SQ_LDS_DATA_FIFO_FULL'):8.0f} {a(d, 'SQ_LDS_CMD_FIFO_FULL'):8.0f}")
