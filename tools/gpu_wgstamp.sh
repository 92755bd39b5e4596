#!/bin/bash
# window-wgrad phase stamps (diagnostic build) for DV_WG_ISS 0 / 2 + a kernel trace of the A/B bench
export TMPDIR=/tmp
tag=${1:-wgstamp}
mkdir -p gpurun_out
for v in 2 0; do
  echo "== DV_WG_ISS=$v" >> gpurun_out/${tag}.log
  DV_WG_ISS=$v DV_HIP_LIB=tools/_stamp/libdv_hip_stamp.so timeout -k 10 120 python tools/wgrad_stamp.py >> gpurun_out/${tag}.log 2>&1 || exit 1
done
DV_WG_ISS=2 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${tag}_prof -o run -- python3 tools/wgrad_ab.py > gpurun_out/${tag}_prof.log 2>&1 || exit 1
cat gpurun_out/${tag}.log
