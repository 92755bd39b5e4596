#!/bin/bash
# round evidence: GPU tests + smoke, default bench, rocprof trace of the replayed step, PMC families
set -o pipefail
export TMPDIR=/tmp
tag=$1
bash tools/gpu_round.sh $tag || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$tag.log 2>&1 || exit 1
bash tools/gpu_pmc_families.sh $tag > /dev/null 2>&1 || exit 1
# keep the summaries and the rocprof stats table; drop the raw traces (gpurun_out/ must stay under 64 MiB)
cp gpurun_out/prof_$tag/run_kernel_stats.csv gpurun_out/kernel_stats_$tag.csv 2>/dev/null
rm -rf gpurun_out/prof_$tag gpurun_out/pmcf_$tag gpurun_out/pmcw_$tag gpurun_out/pmcs_$tag
