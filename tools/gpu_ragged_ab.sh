#!/bin/bash
# ragged-grid tiles: DV_FRAME_CO32R (32-channel window-conv tiles where 64-channel
# ones end in a half-empty round) and DV_GLDS_BN64R (64-channel glds tiles for
# cout = 192): conv parity with both on, same-box step A/B, rocprof family sums
set -o pipefail
export TMPDIR=/tmp
tag=${1:-ragged}
mkdir -p gpurun_out
out=gpurun_out/${tag}.log
: > $out
DV_FRAME_CO32R=1 DV_GLDS_BN64R=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_conv_gpu.py -k "fwd_bwd" >> $out 2>&1 || exit 1
B="python3 bench.py --steps 5 --warmup 3 --no-cpu-baseline --no-roofline --no-sampling --no-fp32"
for v in 0 1; do
  DV_FRAME_CO32R=$v DV_GLDS_BN64R=$v timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${tag}_$v -o run -- $B > gpurun_out/prof_${tag}_$v.log 2>&1 || exit 1
  echo "== knobs=$v" >> $out
  python3 tools/step_families.py gpurun_out/prof_${tag}_$v/run_kernel_trace.csv 12 >> $out 2>&1 || exit 1
done
timeout -k 10 900 bash tools/ab_env.sh DV_FRAME_CO32R "0 1" ${tag}_co32r >> $out 2>&1 || exit 1
timeout -k 10 900 bash tools/ab_env.sh DV_GLDS_BN64R "0 1" ${tag}_bn64r >> $out 2>&1 || exit 1
