#!/bin/bash
# 8x8 window conv as 128-channel 8-wave tiles with the chunk loop split over two
# workgroups (DV_FRAME_W8KS=1 + DV_FRAME_KSPLIT=1 / 2): conv parity, per-launch
# times at the Cfg2 shapes for default / KSPLIT only / KSPLIT + W8KS (alternating)
set -o pipefail
export TMPDIR=/tmp
tag=${1:-w8ks}
mkdir -p gpurun_out
out=gpurun_out/${tag}.log
: > $out
DV_FRAME_KSPLIT=2 DV_FRAME_W8KS=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_conv_gpu.py >> $out 2>&1 || exit 1
DV_FRAME_KSPLIT=1 DV_FRAME_W8KS=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_conv_gpu.py -k "fwd_bwd or ks" >> $out 2>&1 || exit 1
for rep in 1 2; do
  timeout -k 10 200 python -u tools/frame_ab.py base >> $out 2>&1 || exit 1
  DV_FRAME_KSPLIT=2 timeout -k 10 200 python -u tools/frame_ab.py ks2 >> $out 2>&1 || exit 1
  DV_FRAME_KSPLIT=2 DV_FRAME_W8KS=1 timeout -k 10 200 python -u tools/frame_ab.py ks2w8 >> $out 2>&1 || exit 1
  DV_FRAME_KSPLIT=1 DV_FRAME_W8KS=1 timeout -k 10 200 python -u tools/frame_ab.py ks1w8 >> $out 2>&1 || exit 1
done
