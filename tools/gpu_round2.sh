# Round-2 evidence: PMC HBM-traffic passes -> profiles/pmc_traffic_r02<tag>.json
# (read by bench.py for roofline.traffic), then tests (+ parity log), the
# default bench (all legs) and the rocprofv3 kernel stats (tools/gpu_round.sh).
set -o pipefail
tag=$1
bash tools/gpu_pmc.sh $tag && \
python tools/pmc_traffic.py gpurun_out/pmcf_$tag/run_counter_collection.csv gpurun_out/pmcw_$tag/run_counter_collection.csv gpurun_out/pmc_traffic_r02$tag.json && \
cp gpurun_out/pmc_traffic_r02$tag.json profiles/ && \
bash tools/gpu_round.sh $tag
