#!/bin/bash
# checkpoint evidence: the full GPU suite + smoke + default bench + step trace (gpu_round.sh), then PMC families
export TMPDIR=/tmp
tag=${1:-r05p}
bash tools/gpu_evidence.sh $tag || exit 1
tail -3 gpurun_out/tests_$tag.log
cat gpurun_out/smoke_$tag.log | tail -3
head -12 gpurun_out/pmc_families_$tag.txt
