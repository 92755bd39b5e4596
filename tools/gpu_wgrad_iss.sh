#!/bin/bash
# window wgrad DMA-issue placement A/B (DV_WG_ISS 0..3): conv parity per variant, then timing
export TMPDIR=/tmp
tag=${1:-wgiss}
mkdir -p gpurun_out
for v in 1 2 3; do
  DV_WG_ISS=$v timeout -k 10 300 python -u -m pytest tests/test_conv_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${tag}_tests$v.log 2>&1 || { tail -20 gpurun_out/${tag}_tests$v.log; exit 1; }
  tail -1 gpurun_out/${tag}_tests$v.log
done
for rep in 1 2; do
  for v in 0 1 2 3; do
    DV_WG_ISS=$v timeout -k 10 120 python tools/wgrad_ab.py 2>/dev/null | sed "s/^/ISS=$v /" >> gpurun_out/${tag}.log || exit 1
  done
done
grep total gpurun_out/${tag}.log
