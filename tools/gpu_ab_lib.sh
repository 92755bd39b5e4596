#!/bin/bash
# same-box A/B of two builds of libdv_hip (tools/_ab/libdv_hip_base.so vs the in-tree one):
# conv parity on the new build first, then alternating full-step benches
export TMPDIR=/tmp
tag=${1:-ab}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_conv_gpu.py tests/test_skipgrad_gpu.py tests/test_cfg2_gpu.py -x -q --timeout 300 \
  --timeout-method thread > gpurun_out/tests_$tag.log 2>&1
rc=$?
tail -3 gpurun_out/tests_$tag.log
[ $rc = 0 ] || exit 1
B="--steps 30 --warmup 5 --no-sampling --no-cpu-baseline --no-fp32 --no-roofline"
J="import json,sys; d=json.loads([l for l in sys.stdin if l.startswith('{')][-1]); print(sys.argv[1], d['value'], d['ms_per_step'])"
for rep in 1 2 3; do
  DV_HIP_LIB=tools/_ab/libdv_hip_base.so timeout -k 10 300 python bench.py $B 2>/dev/null | python -c "$J" base || exit 1
  timeout -k 10 300 python bench.py $B 2>/dev/null | python -c "$J" new || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$tag -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-roofline --no-sampling --no-fp32 > gpurun_out/prof_$tag.log 2>&1 && \
python tools/prof_summary.py gpurun_out/prof_$tag/run_kernel_trace.csv 60 3 > gpurun_out/summary_$tag.txt && head -8 gpurun_out/summary_$tag.txt
