#!/bin/bash
# cross-attention 8-wave channel split (DV_XA_CS8): parity, same-box step A/B,
# per-kernel rocprof of both settings
set -o pipefail
export TMPDIR=/tmp
tag=${1:-xa}
mkdir -p gpurun_out
out=gpurun_out/${tag}.log
: > $out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ops_gpu.py -k "cross_attention" >> $out 2>&1 || exit 1
timeout -k 10 600 bash tools/ab_env.sh DV_XA_CS8 "0 1" ${tag}_cs8 >> $out 2>&1 || exit 1
B="python3 bench.py --steps 5 --warmup 3 --no-cpu-baseline --no-roofline --no-sampling --no-fp32"
for v in 0 1; do
  DV_XA_CS8=$v timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${tag}_$v -o run -- $B > gpurun_out/prof_${tag}_$v.log 2>&1 || exit 1
  echo "== DV_XA_CS8=$v" >> $out
  python3 - gpurun_out/prof_${tag}_$v/run_kernel_stats.csv >> $out <<'PY' || exit 1
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "xattn" in r["Name"]:
        print("   ", r["Name"][:90], r["Calls"], round(float(r["TotalDurationNs"]) / 1e3, 1), "us total",
              round(float(r["AverageNs"]) / 1e3, 2), "us avg")
PY
done
