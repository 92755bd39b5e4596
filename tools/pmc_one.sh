export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_INSTS_LDS --output-format csv -d gpurun_out/pmc1 -o run -- python3 tools/kbench.py fwd1 > gpurun_out/pmc1.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d gpurun_out/pmc2 -o run -- python3 tools/kbench.py fwd1 > gpurun_out/pmc2.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pmc3 -o run -- python3 tools/kbench.py fwd1 > gpurun_out/pmc3.log 2>&1
python3 - <<'PY'
import csv, collections
for d in ("pmc1", "pmc2"):
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f"gpurun_out/{d}/run_counter_collection.csv")):
        if "stripe" in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, v in agg.items():
        print(d, k, sum(v) / len(v))
PY
grep stripe gpurun_out/pmc3/run_kernel_stats.csv | cut -c1-200
