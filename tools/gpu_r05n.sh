#!/bin/bash
# conv kernel A/B: parity + same-box A/B vs tools/_ab (gpu_ab_lib.sh), then the phase stamps
export TMPDIR=/tmp
tag=${1:-r05n}
bash tools/gpu_ab_lib.sh $tag || exit 1
DV_HIP_LIB=tools/_stamp/libdv_hip_stamp.so timeout -k 10 150 python tools/wgrad_stamp.py > gpurun_out/${tag}_stamps.log 2>&1 || { cat gpurun_out/${tag}_stamps.log; exit 1; }
grep -A1 stripe gpurun_out/${tag}_stamps.log
