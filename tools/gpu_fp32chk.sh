#!/bin/bash
# fp32 leg regression check: which part of the roofline leg slows the fp32 leg after it
export TMPDIR=/tmp
B="--steps 10 --warmup 3 --no-sampling --no-cpu-baseline"
J="import json,sys; d=json.load(sys.stdin); print(sys.argv[1], d['value'], d['fp32']['value'])"
timeout -k 10 300 python bench.py $B 2>/dev/null | tail -1 | python -c "$J" roof || exit 1
DV_BENCH_NOREPLAY=1 timeout -k 10 300 python bench.py $B 2>/dev/null | tail -1 | python -c "$J" noreplay || exit 1
DV_BENCH_GC=1 timeout -k 10 300 python bench.py $B 2>/dev/null | tail -1 | python -c "$J" gc || exit 1
timeout -k 10 300 python bench.py $B --no-roofline 2>/dev/null | tail -1 | python -c "$J" noroof || exit 1
