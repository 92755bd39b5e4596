#!/bin/bash
# per-launch times for the 8x8 K-split variants (tools/frame_ab.py registers
# the hand-off scratch): default / KSPLIT=2 / KSPLIT=2 + W8KS / KSPLIT=1 + W8KS
set -o pipefail
export TMPDIR=/tmp
tag=${1:-w8kst}
mkdir -p gpurun_out
out=gpurun_out/${tag}.log
: > $out
for rep in 1 2; do
  timeout -k 10 200 python -u tools/frame_ab.py base >> $out 2>&1 || exit 1
  DV_FRAME_KSPLIT=2 timeout -k 10 200 python -u tools/frame_ab.py ks2 >> $out 2>&1 || exit 1
  DV_FRAME_KSPLIT=2 DV_FRAME_W8KS=1 timeout -k 10 200 python -u tools/frame_ab.py ks2w8 >> $out 2>&1 || exit 1
  DV_FRAME_KSPLIT=1 DV_FRAME_W8KS=1 timeout -k 10 200 python -u tools/frame_ab.py ks1w8 >> $out 2>&1 || exit 1
done
