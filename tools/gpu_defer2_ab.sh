#!/bin/bash
# window conv with the last two taps deferred behind the barrier (DV_FRAME_DEFER2=1): parity with
# it on, per-launch times at the Cfg2 shapes (alternating), rocprof family sums
# and the same-box step A/B
set -o pipefail
export TMPDIR=/tmp
tag=${1:-defer2}
mkdir -p gpurun_out
# both arms from one library (DV_HIP_LIB, if set: a build beside the in-tree one)
[ -n "$DV_HIP_LIB" ] && export DV_HIP_LIB
out=gpurun_out/${tag}.log
: > $out
DV_FRAME_DEFER2=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_conv_gpu.py >> $out 2>&1 || exit 1
for rep in 1 2; do
  for v in 0 1; do
    DV_FRAME_DEFER2=$v timeout -k 10 200 python -u tools/frame_ab.py defer2=$v >> $out 2>&1 || exit 1
  done
done
B="python3 bench.py --steps 5 --warmup 3 --no-cpu-baseline --no-roofline --no-sampling --no-fp32"
for v in 0 1; do
  DV_FRAME_DEFER2=$v timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${tag}_$v -o run -- $B > gpurun_out/prof_${tag}_$v.log 2>&1 || exit 1
  echo "== DV_FRAME_DEFER2=$v" >> $out
  python3 tools/step_families.py gpurun_out/prof_${tag}_$v/run_kernel_trace.csv 12 >> $out 2>&1 || exit 1
done
timeout -k 10 900 bash tools/ab_env.sh DV_FRAME_DEFER2 "0 1" ${tag}_step >> $out 2>&1 || exit 1
