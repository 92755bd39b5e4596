#!/bin/bash
# pixel-shuffle pass: per-launch times of one replayed step under several
# row-grid caps (DV_SHUF_ROWS, an experiment-only knob of this build)
export TMPDIR=/tmp
tag=${1:-shuf}
mkdir -p gpurun_out
DV_SHUF_ROWS=5 timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py tests/test_skipgrad_gpu.py -q -m gpu \
  --timeout 120 --timeout-method thread > gpurun_out/tests_$tag.log 2>&1
rc=$?
tail -2 gpurun_out/tests_$tag.log
[ $rc = 0 ] || exit 1
P="--steps 5 --warmup 2 --no-cpu-baseline --no-roofline --no-sampling --no-fp32"
for rep in 1 2; do
for cap in base 65535 1024 512 256; do
  if [ $cap = base ]; then export DV_HIP_LIB=tools/_ab/libdv_hip_base.so; else unset DV_HIP_LIB; fi
  export DV_SHUF_ROWS=$cap
  d=gpurun_out/${tag}_$cap
  timeout -k 10 300 rocprofv3 --kernel-trace -d $d -o run --output-format csv -- python3 bench.py $P > $d.log 2>&1 || exit 1
  python - $d/run_kernel_trace.csv $cap <<'EOF'
import csv, sys
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
ends = [i for i, r in enumerate(rows) if "adamw" in r["Kernel_Name"]]
se = [i for j, i in enumerate(ends) if j + 1 == len(ends) or ends[j + 1] - i > 8]
t = []
for lo, hi in zip(se[-4:-1], se[-3:]):
    t.append([(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
              for r in rows[lo + 1:hi + 1] if "shuffle_kernel" in r["Kernel_Name"]])
per = [sum(x) / len(x) for x in zip(*t)]
print(f"cap {sys.argv[2]:>5}: sum {sum(per):6.1f} us/step  " + " ".join(f"{v:5.1f}" for v in per))
EOF
done
done
