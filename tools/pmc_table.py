"""Per (kernel, grid) averages of rocprofv3 --pmc counters from one or more
counter_collection CSVs, with derived shares:

  python tools/pmc_table.py <kernel-substring> a.csv [b.csv ...]

  mfma   SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 * 1024 SIMDs)
  wAny   SQ_WAIT_ANY / SQ_WAVE_CYCLES (parked at s_waitcnt / barrier)
  wInst  SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES (issue stall)
  act    SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES
  hit    TCC_HIT_sum / (TCC_HIT_sum + TCC_MISS_sum)
  fetchMB  2 * FETCH_SIZE KB (the gfx950 half-count correction) / 1e6 * 1024
  dram   TCC_EA0_RDREQ_DRAM_sum / TCC_EA0_RDREQ_sum"""
import csv
import sys
from collections import defaultdict

filt = sys.argv[1]
acc = defaultdict(lambda: defaultdict(list))
for path in sys.argv[2:]:
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"]
        if filt not in name:
            continue
        short = (name.split("N_1")[-1].split("EvNS_")[0] if "_ZN" in name
                 else name.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0])[-48:]
        grid = r.get("Grid_Size", r.get("Grid_Size_X", "?"))
        acc[(short, grid)][r["Counter_Name"]].append(float(r["Counter_Value"]))


def a(d, n):
    v = d.get(n)
    return sum(v) / len(v) if v else float("nan")


def div(x, y):
    return x / y if y == y and y else float("nan")


print(f"{'kernel':48s} {'grid':>8s} {'mfma':>6s} {'wAny':>6s} {'wInst':>6s} {'act':>6s} {'dFIFO':>8s} "
      f"{'ldsI':>8s} {'hit':>6s} {'fetchMB':>8s} {'dram':>6s} {'taAddrTC':>9s} {'taDataTC':>9s}")
for (k, g), d in sorted(acc.items()):
    gui = a(d, "GRBM_GUI_ACTIVE")
    wc = a(d, "SQ_WAVE_CYCLES")
    hit, miss = a(d, "TCC_HIT_sum"), a(d, "TCC_MISS_sum")
    print(f"{k:48s} {g:>8s} {div(a(d, 'SQ_VALU_MFMA_BUSY_CYCLES'), gui / 8 * 1024):6.3f} "
          f"{div(a(d, 'SQ_WAIT_ANY'), wc):6.3f} {div(a(d, 'SQ_WAIT_INST_ANY'), wc):6.3f} "
          f"{div(a(d, 'SQ_ACTIVE_INST_ANY'), wc):6.3f} {a(d, 'SQ_LDS_DATA_FIFO_FULL'):8.0f} {a(d, 'SQ_INSTS_LDS'):8.0f} "
          f"{div(hit, hit + miss):6.3f} {2 * a(d, 'FETCH_SIZE') * 1024 / 1e6:8.2f} "
          f"{div(a(d, 'TCC_EA0_RDREQ_DRAM_sum'), a(d, 'TCC_EA0_RDREQ_sum')):6.3f} "
          f"{a(d, 'TA_ADDR_STALLED_BY_TC_CYCLES_sum'):9.0f} {a(d, 'TA_DATA_STALLED_BY_TC_CYCLES_sum'):9.0f}")
