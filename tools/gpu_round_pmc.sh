# Round evidence: PMC HBM-traffic passes -> profiles/pmc_traffic_r01<tag>.json
# (read by bench.py for roofline.traffic), then tests, default bench with
# cpu_baseline and the rocprofv3 kernel stats (tools/gpu_round.sh).
set -o pipefail
tag=$1
bash tools/gpu_pmc.sh $tag && \
python tools/pmc_traffic.py gpurun_out/pmcf_$tag/run_counter_collection.csv gpurun_out/pmcw_$tag/run_counter_collection.csv gpurun_out/pmc_traffic_r01$tag.json && \
cp gpurun_out/pmc_traffic_r01$tag.json profiles/ && \
bash tools/gpu_round.sh $tag
