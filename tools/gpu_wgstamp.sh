#!/bin/bash
# conv / wgrad phase stamps (diagnostic build: make -C dalle2-video_amd/csrc stamp, copied to tools/_stamp/ so it travels)
export TMPDIR=/tmp
tag=${1:-wgstamp}
mkdir -p gpurun_out
DV_HIP_LIB=tools/_stamp/libdv_hip_stamp.so timeout -k 10 150 python tools/wgrad_stamp.py > gpurun_out/${tag}.log 2>&1 || { cat gpurun_out/${tag}.log; exit 1; }
cat gpurun_out/${tag}.log
