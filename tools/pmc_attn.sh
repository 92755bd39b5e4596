# PMC passes (one counter group per run) over tools/attnbench.py, averaged per fa kernel
export TMPDIR=/tmp
rocprofv3 -L > gpurun_out/pmc_list.txt 2>&1 || true
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_ANY --output-format csv -d gpurun_out/apmc1 -o run -- python3 tools/attnbench.py > gpurun_out/apmc1.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_MFMA SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d gpurun_out/apmc2 -o run -- python3 tools/attnbench.py > gpurun_out/apmc2.log 2>&1 ; \
python3 - <<'PY'
import csv, collections, os
for d in ("apmc1", "apmc2"):
    f = f"gpurun_out/{d}/run_counter_collection.csv"
    if not os.path.exists(f):
        print(d, "missing"); continue
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if "fa::" in r["Kernel_Name"] or "fa_kernel" in r["Kernel_Name"]:
            k = r["Kernel_Name"].split("::")[-1][:20]
            agg[(k, r["Counter_Name"])].append(float(r["Counter_Value"]))
    for k, v in sorted(agg.items()):
        print(d, k, f"{sum(v) / len(v):.4g}")
PY
