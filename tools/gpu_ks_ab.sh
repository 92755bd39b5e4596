#!/bin/bash
# window-conv K-split: conv parity (both settings) + same-box step A/B; MQA tests
set -o pipefail
export TMPDIR=/tmp
tag=${1:-ks}
mkdir -p gpurun_out
out=gpurun_out/${tag}.log
: > $out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ops_gpu.py -k "mqa" >> $out 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_conv_gpu.py >> $out 2>&1 || exit 1
DV_FRAME_KS256=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_conv_gpu.py -k "fwd_bwd" >> $out 2>&1 || exit 1
timeout -k 10 600 bash tools/ab_env.sh DV_FRAME_KSPLIT "0 1" ${tag}_ksplit >> $out 2>&1 || exit 1
timeout -k 10 600 bash tools/ab_env.sh DV_FRAME_KS256 "0 1" ${tag}_ks256 >> $out 2>&1 || exit 1
