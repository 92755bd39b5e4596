# PMC evidence per kernel (eager bench, 2 steps): HBM traffic (FETCH_SIZE, WRITE_SIZE
# in separate passes) and MFMA / VALU / LDS activity (one SQ + GRBM pass).
#   bash tools/gpu_pmc_families.sh <tag>
export TMPDIR=/tmp
tag=$1
B="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-roofline --no-graphs --no-sampling --no-fp32 --no-config3"
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmcf_$tag -o run -- $B > gpurun_out/pmcf_$tag.log 2>&1 && \
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmcw_$tag -o run -- $B > gpurun_out/pmcw_$tag.log 2>&1 && \
timeout -s KILL 240 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d gpurun_out/pmcs_$tag -o run -- $B > gpurun_out/pmcs_$tag.log 2>&1 && \
python3 tools/pmc_traffic.py gpurun_out/pmcf_$tag/run_counter_collection.csv gpurun_out/pmcw_$tag/run_counter_collection.csv gpurun_out/pmc_traffic_$tag.json && \
python3 tools/pmc_sq.py gpurun_out/pmcs_$tag/run_counter_collection.csv gpurun_out/pmc_traffic_$tag.json > gpurun_out/pmc_families_$tag.txt && cat gpurun_out/pmc_families_$tag.txt
