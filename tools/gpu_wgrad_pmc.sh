#!/bin/bash
# window wgrad: timing A/B of the XCD tile dealing + counters of the default form
export TMPDIR=/tmp
tag=${1:-wgpmc}
mkdir -p gpurun_out
for rep in 1 2; do
  for v in 0 1; do
    DV_WG_XCD=$v timeout -k 10 120 python tools/wgrad_ab.py 2>/dev/null | sed "s/^/XCD=$v /" >> gpurun_out/${tag}.log || exit 1
  done
done
grep total gpurun_out/${tag}.log
B="python3 tools/wgrad_ab.py"
for x in 0 1; do
export DV_WG_XCD=$x
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_LDS_DATA_FIFO_FULL SQ_INSTS_LDS GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/${tag}_x${x}_1 -o run -- $B > /dev/null 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/${tag}_x${x}_2 -o run -- $B > /dev/null 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${tag}_x${x}_3 -o run -- $B > /dev/null 2>&1 || exit 1
timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_RDREQ_DRAM_sum TCC_EA0_RDREQ_sum --output-format csv -d gpurun_out/${tag}_x${x}_4 -o run -- $B > /dev/null 2>&1 || exit 1
echo "== DV_WG_XCD=$x" >> gpurun_out/${tag}_pmc.txt
python3 tools/pmc_table.py wgrad gpurun_out/${tag}_x${x}_{1,2,3,4}/run_counter_collection.csv >> gpurun_out/${tag}_pmc.txt || exit 1
done
cat gpurun_out/${tag}_pmc.txt
