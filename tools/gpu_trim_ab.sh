#!/bin/bash
# stripe wgrad at W = 64 with the trimmed window image, 3-deep ring (DV_WG_TRIM=1):
# conv parity with it on, rocprof family sums per arm and the same-box step A/B
set -o pipefail
export TMPDIR=/tmp
tag=${1:-trim}
mkdir -p gpurun_out
out=gpurun_out/${tag}.log
: > $out
DV_WG_TRIM=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_conv_gpu.py >> $out 2>&1 || exit 1
B="python3 bench.py --steps 5 --warmup 3 --no-cpu-baseline --no-roofline --no-sampling --no-fp32"
for rep in 1 2; do
  for v in 0 1; do
    DV_WG_TRIM=$v timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${tag}_${v}_$rep -o run -- $B > gpurun_out/prof_${tag}_${v}_$rep.log 2>&1 || exit 1
    echo "== DV_WG_TRIM=$v rep $rep" >> $out
    python3 tools/step_families.py gpurun_out/prof_${tag}_${v}_$rep/run_kernel_trace.csv 4 >> $out 2>&1 || exit 1
    grep -h "wgrad_stripe" gpurun_out/prof_${tag}_${v}_$rep/run_kernel_stats.csv | cut -d, -f1-4 >> $out
  done
done
timeout -k 10 900 bash tools/ab_env.sh DV_WG_TRIM "0 1" ${tag}_step >> $out 2>&1 || exit 1
