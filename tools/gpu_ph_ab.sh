#!/bin/bash
# phased K / V prologue of the forward and dq (DV_MQA_PH) and two query tiles
# per dk/dv step (DV_MQA_TPS=2): MQA parity with each, attnbench + rocprof
# kernel stats per variant (same box), alternating
set -o pipefail
export TMPDIR=/tmp
tag=${1:-ph}
mkdir -p gpurun_out
out=gpurun_out/${tag}.log
: > $out
for e in "DV_MQA_PH=1 DV_MQA_TPS=2" "DV_MQA_PH=0 DV_MQA_TPS=1"; do
  env $e timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ops_gpu.py -k "mqa" >> $out 2>&1 || exit 1
done
run() {  # name env...
  local name=$1; shift
  echo "== $name" >> $out
  env "$@" timeout -k 10 120 python -u tools/attnbench.py >> $out 2>&1 || return 1
  env "$@" timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${tag}_$name -o run -- python3 tools/attnbench.py > gpurun_out/prof_${tag}_$name.log 2>&1 || return 1
  python3 - gpurun_out/prof_${tag}_$name/run_kernel_trace.csv >> $out <<'PY' || return 1
import csv, sys, collections
d = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Kernel_Name"]
    if "mqa" in n:
        key = (n[:60], r["Grid_Size_X"], r["Grid_Size_Y"], r["Grid_Size_Z"])
        d[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in sorted(d.items()):
    v.sort()
    print(f"    {k[0]:60s} grid {k[1]}x{k[2]}x{k[3]} n={len(v)} median {v[len(v) // 2]:.2f} us")
PY
}
for rep in 1 2; do
  run base_$rep DV_MQA_PH=0 DV_MQA_TPS=1 || exit 1
  run ph_$rep DV_MQA_PH=1 DV_MQA_TPS=1 || exit 1
  run tps2_$rep DV_MQA_PH=0 DV_MQA_TPS=2 || exit 1
  run both_$rep DV_MQA_PH=1 DV_MQA_TPS=2 || exit 1
done
