#!/bin/bash
# conv parity tests + same-box A/B of the window wgrad (DV_WG_OLD=0) against the stripe one (=1)
export TMPDIR=/tmp
tag=${1:-wgab}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_conv_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1; rc=$?
tail -3 gpurun_out/${tag}_tests.log
[ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in 0 1; do
    DV_WG_OLD=$v timeout -k 10 120 python tools/wgrad_ab.py >> gpurun_out/${tag}.log 2>&1 || exit 1
  done
done
grep total gpurun_out/${tag}.log
