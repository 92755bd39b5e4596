#!/bin/bash
# stripe conv with the window DMA interleaved among the MFMAs: stamps, parity, same-box A/B vs the previous build
export TMPDIR=/tmp
DV_HIP_LIB=tools/_stamp/libdv_hip_stamp.so timeout -k 10 150 python tools/wgrad_stamp.py > gpurun_out/r05n_stamps.log 2>&1 || { cat gpurun_out/r05n_stamps.log; exit 1; }
grep -A1 stripe gpurun_out/r05n_stamps.log
bash tools/gpu_ab_lib.sh r05n
