#!/bin/bash
# attention A/B on one box: new lib (pair / single-tile steps, whole-LDS and
# streamed at Cfg2) vs the r03 build, + rocprof kernel stats of each variant
set -o pipefail
export TMPDIR=/tmp
tag=${1:-attn}
mkdir -p gpurun_out
out=gpurun_out/${tag}.log
: > $out
run() {  # name env...
  local name=$1; shift
  echo "== $name" >> $out
  env "$@" timeout -k 10 120 python -u tools/attnbench.py >> $out 2>&1 || return 1
  env "$@" timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${tag}_$name -o run -- python3 tools/attnbench.py > gpurun_out/prof_${tag}_$name.log 2>&1 || return 1
  python3 - gpurun_out/prof_${tag}_$name/run_kernel_stats.csv >> $out <<'PY' || return 1
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "mqa" in r["Name"] or "finish" in r["Name"]:
        print("   ", r["Name"][:70], r["Calls"], round(float(r["AverageNs"]) / 1e3, 2), "us")
PY
}
run pair DV_MQA_PAIR=1 || exit 1
run single DV_MQA_PAIR=0 || exit 1
run pair_stream DV_MQA_PAIR=1 DV_MQA_STREAM=1 || exit 1
run r03 DV_HIP_LIB=$PWD/dalle2-video_amd/csrc/build/ab/libdv_hip_r03.so || exit 1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ops_gpu.py -k "mqa" >> $out 2>&1 || exit 1
DV_MQA_PAIR=0 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ops_gpu.py -k "mqa" >> $out 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_conv_gpu.py >> $out 2>&1 || exit 1
timeout -k 10 900 bash tools/ab_env.sh DV_FRAME_KSPLIT "0 1" ${tag}_ksplit >> $out 2>&1 || exit 1
DV_FRAME_KS256=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_conv_gpu.py >> $out 2>&1 || exit 1
timeout -k 10 900 bash tools/ab_env.sh DV_FRAME_KS256 "0 1" ${tag}_ks256 >> $out 2>&1 || exit 1
