#!/bin/bash
# round-4 first GPU pass: DP (native RCCL comm), attention A/B, attention tests, config-5 parity
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_dp_trainer_gpu.py > gpurun_out/dp_r04a.log 2>&1 || exit 1
echo "== new" > gpurun_out/attn_r04a.log
timeout -k 10 120 python -u tools/attnbench.py >> gpurun_out/attn_r04a.log 2>&1 || exit 1
echo "== r03" >> gpurun_out/attn_r04a.log
DV_HIP_LIB=$PWD/dalle2-video_amd/csrc/build/ab/libdv_hip_r03.so timeout -k 10 120 python -u tools/attnbench.py >> gpurun_out/attn_r04a.log 2>&1 || exit 1
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_ops_gpu.py -k "mqa" > gpurun_out/ops_mqa_r04a.log 2>&1 || exit 1
DV_PARITY_LOG=gpurun_out/cfg5_parity.jsonl timeout -k 10 500 python -u -m pytest -x -v -s --timeout 400 --timeout-method thread tests/test_cfg5_gpu.py > gpurun_out/cfg5_r04a.log 2>&1 || exit 1
