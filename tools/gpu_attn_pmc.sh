#!/bin/bash
# MQA kernel counters over tools/attnbench.py (two SQ passes) -> issue-slot ceiling table
export TMPDIR=/tmp
tag=${1:-attnpmc}
mkdir -p gpurun_out
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_INSTS_SALU GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/apmc1_$tag -o run -- python3 tools/attnbench.py > gpurun_out/apmc1_$tag.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_TRANS_F32 SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/apmc2_$tag -o run -- python3 tools/attnbench.py > gpurun_out/apmc2_$tag.log 2>&1
python3 tools/attn_pmc.py gpurun_out/apmc1_$tag/run_counter_collection.csv $(ls gpurun_out/apmc2_$tag/run_counter_collection.csv 2>/dev/null) > gpurun_out/attn_pmc_$tag.txt
cat gpurun_out/attn_pmc_$tag.txt
