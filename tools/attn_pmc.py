"""Issue-slot ceiling of the MQA kernels from two rocprofv3 SQ passes over
tools/attnbench.py (tools/gpu_attn_pmc.sh):

  python tools/attn_pmc.py pass1_counter_collection.csv pass2_counter_collection.csv

Per kernel (and grid, so the config-2 and 8,192-token forwards stay apart),
averages per dispatch:
  mfma_busy   SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 * 1024 SIMDs)
  issue_busy  vector issue cycles / the same SIMD-cycles, with the per-wave
              issue costs of MI355X_MICROARCH.md (constants table, 'vector-
              instruction ISSUE cost'): transcendental 8, other VALU 4, an MFMA
              holds issue for 8 of its 32 cycles
  ceiling     the MFMA-busy the same instruction mix allows when the vector
              issue port is the binding resource: mfma_cycles / issue_cycles
              (a SIMD cannot run the MFMA pipe faster than it can issue the
              VALU work the kernel pairs with each MFMA)
"""
import csv
import sys
from collections import defaultdict


def load(path, rows, disp):
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"]
        for tag in ("mqa_fwd_fa_stream_kernel", "mqa_fwd_fa_kernel", "mqa_fwd_pp_kernel", "mqa_dq_fa_kernel",
                    "mqa_dkdv_fa_kernel", "mqa_finish_fa_kernel", "mqa_prep_kernel"):
            if tag in name:
                break
        else:
            continue
        k = (tag, r.get("Grid_Size", r.get("Grid_Size_X", "")))
        rows[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
        disp[k].add(r.get("Dispatch_Id", ""))


rows = defaultdict(lambda: defaultdict(list))
disp = defaultdict(set)
for p in sys.argv[1:]:
    load(p, rows, disp)


def avg(d, n):
    v = d.get(n)
    return sum(v) / len(v) if v else float("nan")


print(f"{'kernel':28s} {'grid':>8s} {'n':>3s} {'mfma_busy':>9s} {'issue_busy':>10s} {'ceiling':>8s} "
      f"{'busy/ceil':>9s} {'valu/mfma':>9s} {'trans/mfma':>10s}")
for k, d in sorted(rows.items()):
    gui = avg(d, "GRBM_GUI_ACTIVE")
    simd_cyc = gui / 8 * 1024
    mf_cyc = avg(d, "SQ_VALU_MFMA_BUSY_CYCLES")
    n_mfma = avg(d, "SQ_INSTS_MFMA")
    n_valu = avg(d, "SQ_INSTS_VALU")
    n_trans = avg(d, "SQ_INSTS_VALU_TRANS_F32")
    if n_trans != n_trans:
        n_trans = 0.0
    plain = n_valu - n_mfma - n_trans  # SQ_INSTS_VALU counts MFMAs too
    issue = 8 * n_trans + 4 * plain + 8 * n_mfma
    busy = mf_cyc / simd_cyc
    ceil = mf_cyc / max(issue, mf_cyc, 1.0)
    print(f"{k[0]:28s} {k[1]:>8s} {len(disp[k]):3d} {busy:9.3f} {issue / simd_cyc:10.3f} {ceil:8.3f} "
          f"{busy / ceil if ceil else float('nan'):9.3f} {n_valu / n_mfma if n_mfma else float('nan'):9.2f} "
          f"{n_trans / n_mfma if n_mfma else float('nan'):10.2f}")
