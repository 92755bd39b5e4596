#!/bin/bash
# MX-fp8 PV mid attention: parity (fp8 tests + the existing MQA tests), the same-process A/B, a kernel trace
export TMPDIR=/tmp
tag=${1:-mqa8}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_mqa_fp8_gpu.py tests/test_ops_gpu.py -k "mqa or fp8" -x -v -s --timeout 300 \
  --timeout-method thread > gpurun_out/tests_$tag.log 2>&1
rc=$?
grep -E "passed|failed|rel" gpurun_out/tests_$tag.log | tail -12
[ $rc = 0 ] || exit 1
timeout -k 10 300 python tools/mqa8_ab.py 2>&1 | tee gpurun_out/ab_$tag.txt || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$tag -o run --output-format csv -- python3 tools/mqa8_ab.py > gpurun_out/prof_$tag.log 2>&1 && \
grep -E "mqa|Name" gpurun_out/prof_$tag/run_kernel_stats.csv | cut -c1-200
