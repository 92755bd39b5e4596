#!/bin/bash
# round evidence: GPU tests + smoke, default bench, rocprof trace of the replayed step, PMC families
set -o pipefail
export TMPDIR=/tmp
tag=$1
bash tools/gpu_round.sh $tag || exit 1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$tag.log 2>&1 || exit 1
bash tools/gpu_pmc_families.sh $tag > /dev/null 2>&1 || exit 1
