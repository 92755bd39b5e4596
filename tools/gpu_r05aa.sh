#!/bin/bash
# stripe conv at W = 128: conv + config-5 parity, then config-5 sampling base vs new library (same box)
export TMPDIR=/tmp
tag=${1:-r05aa}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_conv_gpu.py tests/test_cfg5_gpu.py -x -q --timeout 600 \
  --timeout-method thread > gpurun_out/tests_$tag.log 2>&1
rc=$?
tail -3 gpurun_out/tests_$tag.log
[ $rc = 0 ] || exit 1
B="--steps 5 --warmup 5 --no-cpu-baseline --no-fp32 --no-roofline"
J="import json,sys; d=json.loads([l for l in sys.stdin if l.startswith('{')][-1]); s=d['sampling']; print(sys.argv[1], 'c5 bf16', s['config5_bf16']['value'], 'c5 fp8', s['config5_fp8']['value'], 'bs4', s['bs4']['value'], 'train', d['value'])"
for rep in 1 2; do
  DV_HIP_LIB=tools/_ab/libdv_hip_base.so timeout -k 10 400 python bench.py $B 2>/dev/null | python -c "$J" base || exit 1
  timeout -k 10 400 python bench.py $B 2>/dev/null | python -c "$J" new || exit 1
done
