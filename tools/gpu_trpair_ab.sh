#!/bin/bash
# MQA bounded forward: paired V^T reads with immediate offsets (product build) vs
# separate reads (build/ab/libdv_hip_tr0.so): parity + attnbench + rocprof
set -o pipefail
export TMPDIR=/tmp
tag=${1:-msum}
mkdir -p gpurun_out
out=gpurun_out/${tag}.log
: > $out
OLD=$PWD/dalle2-video_amd/csrc/build/ab/libdv_hip_tr0.so
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ops_gpu.py -k "mqa" >> $out 2>&1 || exit 1
run() {  # name env...
  local name=$1; shift
  echo "== $name" >> $out
  env "$@" timeout -k 10 120 python -u tools/attnbench.py >> $out 2>&1 || return 1
  env "$@" timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${tag}_$name -o run -- python3 tools/attnbench.py > gpurun_out/prof_${tag}_$name.log 2>&1 || return 1
  python3 - gpurun_out/prof_${tag}_$name/run_kernel_stats.csv >> $out <<'PY' || return 1
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "mqa_fwd" in r["Name"]:
        print("   ", r["Name"][:70], r["Calls"], round(float(r["AverageNs"]) / 1e3, 2), "us")
PY
}
run pairtr DV_MQA_FIXED=1 || exit 1
run before DV_HIP_LIB=$OLD || exit 1
run pairtr2 DV_MQA_FIXED=1 || exit 1
