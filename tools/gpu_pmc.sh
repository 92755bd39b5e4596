# HBM traffic per kernel: two separate rocprofv3 PMC passes (FETCH_SIZE, then
# WRITE_SIZE — never combined with tracing) over the eager bench, summarised by
# tools/pmc_traffic.py into gpurun_out/pmc_traffic_<tag>.json.
#   bash tools/gpu_pmc.sh <tag>
export TMPDIR=/tmp
tag=$1
mkdir -p gpurun_out
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmcf_$tag -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-roofline --no-graphs --no-sampling --no-fp32 > gpurun_out/pmcf_$tag.log 2>&1 && \
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmcw_$tag -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-roofline --no-graphs --no-sampling --no-fp32 > gpurun_out/pmcw_$tag.log 2>&1 && \
python tools/pmc_traffic.py gpurun_out/pmcf_$tag/run_counter_collection.csv gpurun_out/pmcw_$tag/run_counter_collection.csv gpurun_out/pmc_traffic_$tag.json
