#!/bin/bash
export TMPDIR=/tmp
tag=${1:-r05g}
DV_HIP_LIB=tools/_stamp/libdv_hip_stamp.so timeout -k 10 120 python tools/mqa_stamp.py > gpurun_out/mqa_stamp_$tag.log 2>&1 || { cat gpurun_out/mqa_stamp_$tag.log; exit 1; }
cat gpurun_out/mqa_stamp_$tag.log
bash tools/gpu_evidence.sh $tag
