#!/bin/bash
# conv1x1 residual prefetch without the compiler's DMA drains: conv parity + step trace
export TMPDIR=/tmp
tag=${1:-r05j}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_conv_gpu.py tests/test_skipgrad_gpu.py tests/test_cfg2_gpu.py -x -q --timeout 300 \
  --timeout-method thread > gpurun_out/tests_$tag.log 2>&1
rc=$?
tail -4 gpurun_out/tests_$tag.log
[ $rc = 0 ] || exit 1
timeout -k 10 300 python bench.py --no-sampling --no-cpu-baseline --no-fp32 > gpurun_out/bench_$tag.log 2> gpurun_out/bench_$tag.err && \
tail -1 gpurun_out/bench_$tag.log | cut -c1-200 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$tag -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-roofline --no-sampling --no-fp32 > gpurun_out/prof_$tag.log 2>&1 && \
python tools/prof_summary.py gpurun_out/prof_$tag/run_kernel_trace.csv 60 3 > gpurun_out/summary_$tag.txt && head -16 gpurun_out/summary_$tag.txt
