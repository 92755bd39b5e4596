# PMC passes over the 8x8-stage 512->512 forward conv (tools/kbench.py fwd8)
export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_WAIT_ANY --output-format csv -d gpurun_out/cpmc1 -o run -- python3 tools/kbench.py fwd8 > gpurun_out/cpmc1.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LDS_UNALIGNED_STALL SQ_INSTS_VALU SQ_INSTS_MFMA SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d gpurun_out/cpmc2 -o run -- python3 tools/kbench.py fwd8 > gpurun_out/cpmc2.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum SQ_INSTS_VMEM SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_VMEM --output-format csv -d gpurun_out/cpmc4 -o run -- python3 tools/kbench.py fwd8 > gpurun_out/cpmc4.log 2>&1 ; \
timeout -s KILL 90 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/cpmc3 -o run -- python3 tools/kbench.py fwd8 > gpurun_out/cpmc3.log 2>&1
python3 - <<'PY'
import csv, collections, os
for d in ("cpmc1", "cpmc2", "cpmc4"):
    f = f"gpurun_out/{d}/run_counter_collection.csv"
    if not os.path.exists(f):
        print(d, "missing"); continue
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if "conv" in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, v in agg.items():
        print(d, k, f"{sum(v) / len(v):.4g}")
PY
grep conv gpurun_out/cpmc3/run_kernel_stats.csv | cut -c1-160
