#!/bin/bash
# LDS / issue counters of the window / stripe / row-window wgrad convs over two eager bench steps,
# two SQ passes, counters picked from what rocprofv3 -L lists on the box:
#   bash tools/step_conv_pmc.sh <tag>   -> gpurun_out/<tag>.log
export TMPDIR=/tmp
tag=${1:-spmc}
mkdir -p gpurun_out
out=gpurun_out/${tag}.log
timeout -k 10 120 rocprofv3 -L > gpurun_out/${tag}_counters.txt 2>&1 || exit 1
pick() { local o=""; for c in $1; do grep -qw "$c" gpurun_out/${tag}_counters.txt && o="$o $c"; done; echo $o; }
p1=$(pick "SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY")
p2=$(pick "SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_MISC SQ_INSTS_MFMA SQ_INSTS_VALU SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL")
echo "pass1: $p1" > $out
echo "pass2: $p2" >> $out
timeout -s KILL 240 rocprofv3 --pmc $p1 GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/${tag}_1 -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-roofline --no-graphs --no-sampling --no-fp32 >> $out 2>&1 || exit 1
timeout -s KILL 240 rocprofv3 --pmc $p2 GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/${tag}_2 -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-roofline --no-graphs --no-sampling --no-fp32 >> $out 2>&1 || exit 1
python3 tools/frame_pmc.py gpurun_out/${tag}_1/run_counter_collection.csv gpurun_out/${tag}_2/run_counter_collection.csv >> $out 2>&1
