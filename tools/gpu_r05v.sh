#!/bin/bash
# config 5 with the fp8 PV attention: end-to-end parity, then the bench's sampling legs
export TMPDIR=/tmp
tag=${1:-r05v}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_cfg5_gpu.py tests/test_sample_gpu.py tests/test_mqa_fp8_gpu.py -x -v --timeout 600 \
  --timeout-method thread > gpurun_out/tests_$tag.log 2>&1
rc=$?
grep -E "passed|failed|PASS|FAIL" gpurun_out/tests_$tag.log | tail -30
[ $rc = 0 ] || exit 1
timeout -k 10 600 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-fp32 > gpurun_out/bench_$tag.log 2>&1 || exit 1
tail -1 gpurun_out/bench_$tag.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); s=d.get('sampling',{}); print(json.dumps({k: s.get(k) for k in ('config5_bf16','config5_fp8')}, indent=1)[:3000])"
