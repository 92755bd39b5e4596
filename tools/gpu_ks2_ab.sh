#!/bin/bash
# window-conv K split with the XCD-local hand-off (DV_FRAME_KSPLIT=2): conv
# parity + XCD check, same-box step A/B vs off, per-kernel rocprof of both
set -o pipefail
export TMPDIR=/tmp
tag=${1:-ks2}
mkdir -p gpurun_out
out=gpurun_out/${tag}.log
: > $out
DV_FRAME_KSPLIT=2 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_conv_gpu.py -k "fwd_bwd" >> $out 2>&1 || exit 1
DV_FRAME_KSPLIT=2 DV_FRAME_KS256=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_conv_gpu.py -k "fwd_bwd" >> $out 2>&1 || exit 1
timeout -k 10 600 bash tools/ab_env.sh DV_FRAME_KSPLIT "0 2" ${tag}_ksplit >> $out 2>&1 || exit 1
DV_FRAME_KSPLIT=2 timeout -k 10 600 bash tools/ab_env.sh DV_FRAME_KS256 "0 1" ${tag}_ks256 >> $out 2>&1 || exit 1
B="python3 bench.py --steps 5 --warmup 3 --no-cpu-baseline --no-roofline --no-sampling --no-fp32"
for v in 0 2; do
  DV_FRAME_KSPLIT=$v timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${tag}_$v -o run -- $B > gpurun_out/prof_${tag}_$v.log 2>&1 || exit 1
  echo "== DV_FRAME_KSPLIT=$v" >> $out
  python3 - gpurun_out/prof_${tag}_$v/run_kernel_stats.csv >> $out <<'PY' || exit 1
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "frame" in r["Name"]:
        print("   ", r["Name"][:90], r["Calls"], round(float(r["TotalDurationNs"]) / 1e3, 1), "us total",
              round(float(r["AverageNs"]) / 1e3, 2), "us avg")
PY
done
