#!/bin/bash
# one GPU iteration: selected GPU tests, a short bench (train leg only), and the
# rocprofv3 kernel trace of a graph-replayed bench summarised per step.
#   bash tools/gpu_iter.sh <tag> [pytest targets...]
set -o pipefail
export TMPDIR=/tmp
tag=$1; shift
mkdir -p gpurun_out
export DV_PARITY_LOG=gpurun_out/parity_$tag.jsonl
if [ $# -gt 0 ]; then
  timeout -k 10 600 python -u -m pytest "$@" -x -q --timeout 300 --timeout-method thread > gpurun_out/tests_$tag.log 2>&1 || { tail -30 gpurun_out/tests_$tag.log; exit 1; }
  tail -2 gpurun_out/tests_$tag.log
fi
timeout -k 10 300 python bench.py --no-cpu-baseline --no-sampling --no-fp32 --no-config3 > gpurun_out/bench_$tag.log 2> gpurun_out/bench_$tag.err || { tail -20 gpurun_out/bench_$tag.err; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/bench_$tag.log').read().splitlines()[-1]);print('value',d['value'],'ms',d['ms_per_step'],'frac',d['roofline']['frac'],d['roofline']['kernel'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$tag -o run --output-format csv -- python3 bench.py --steps 5 --warmup 5 --no-cpu-baseline --no-roofline --no-sampling --no-fp32 --no-config3 > gpurun_out/prof_$tag.log 2>&1 || { tail -20 gpurun_out/prof_$tag.log; exit 1; }
python tools/prof_summary.py gpurun_out/prof_$tag/run_kernel_trace.csv 60 3 > gpurun_out/summary_$tag.txt && head -24 gpurun_out/summary_$tag.txt
