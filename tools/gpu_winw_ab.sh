#!/bin/bash
# same-box A/B of the window-form 3x3 conv's width set (ops._WINDOW_W, env
# DV_WINDOW_W): the default 8,16 against 8,16,32 and 8,16,32,64, alternating
# full-step benches, then one replayed-step kernel trace per setting
export TMPDIR=/tmp
tag=${1:-winw}
mkdir -p gpurun_out
B="--steps 30 --warmup 5 --no-sampling --no-cpu-baseline --no-fp32 --no-roofline"
J="import json,sys; d=json.loads([l for l in sys.stdin if l.startswith('{')][-1]); print(sys.argv[1], d['value'], d['ms_per_step'])"
for rep in 1 2; do
  for ww in 8,16 8,16,32 8,16,32,64; do
    DV_WINDOW_W=$ww timeout -k 10 300 python bench.py $B 2>/dev/null | python -c "$J" "W=$ww" || exit 1
  done
done
P="--steps 5 --warmup 2 --no-cpu-baseline --no-roofline --no-sampling --no-fp32"
for ww in 8,16 8,16,32 8,16,32,64; do
  export DV_WINDOW_W=$ww
  d=gpurun_out/${tag}_${ww//,/_}
  timeout -k 10 300 rocprofv3 --kernel-trace -d $d -o run --output-format csv -- python3 bench.py $P > $d.log 2>&1 || exit 1
  python tools/prof_summary.py $d/run_kernel_trace.csv 400 3 > $d.txt
  echo "W=$ww"; grep -E "conv_fwd" $d.txt | head -8
done
