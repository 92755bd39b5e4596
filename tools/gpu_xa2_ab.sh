#!/bin/bash
# cross-attention loads out of the store phases: xa0 = before, xa1 = g2 in LDS
# + colsum preloaded, new = xa1 + the backward's Vt^T / Kt^T images and colsum
# staged in LDS per clip-uniform workgroup.  Parity, phase stamps (new),
# same-box step A/B of the three, per-kernel rocprof of each
set -o pipefail
export TMPDIR=/tmp
tag=${1:-xa2}
mkdir -p gpurun_out
out=gpurun_out/${tag}.log
: > $out
NEW=$PWD/dalle2-video_amd/dalle2_video/libdv_hip.so
OLD=$PWD/dalle2-video_amd/csrc/build/ab/libdv_hip_xa0.so
XA1=$PWD/dalle2-video_amd/csrc/build/ab/libdv_hip_xa1.so
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ops_gpu.py -k "cross_attention" >> $out 2>&1 || exit 1
DV_HIP_LIB=$PWD/dalle2-video_amd/csrc/build_stamp/libdv_hip_stamp.so timeout -k 10 200 python -u tools/xattn_stamp.py >> $out 2>&1 || exit 1
timeout -k 10 600 bash tools/ab_env.sh DV_HIP_LIB "$OLD $XA1 $NEW" ${tag}_lib >> $out 2>&1 || exit 1
B="python3 bench.py --steps 5 --warmup 3 --no-cpu-baseline --no-roofline --no-sampling --no-fp32"
for v in old xa1 new; do
  L=$OLD; [ $v = new ] && L=$NEW; [ $v = xa1 ] && L=$XA1
  DV_HIP_LIB=$L timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${tag}_$v -o run -- $B > gpurun_out/prof_${tag}_$v.log 2>&1 || exit 1
  echo "== $v" >> $out
  python3 - gpurun_out/prof_${tag}_$v/run_kernel_stats.csv >> $out <<'PY' || exit 1
import csv, sys
t = 0.0
for r in csv.DictReader(open(sys.argv[1])):
    if "xattn" in r["Name"]:
        t += float(r["TotalDurationNs"])
        print("   ", r["Name"][:90], r["Calls"], round(float(r["TotalDurationNs"]) / 1e3, 1), "us total",
              round(float(r["AverageNs"]) / 1e3, 2), "us avg")
print("    xattn total", round(t / 1e3, 1), "us")
PY
done
