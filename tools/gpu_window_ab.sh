#!/bin/bash
# same-box A/B: which frame widths run the window-form conv (DV_WINDOW_W), full training step
export TMPDIR=/tmp
B="--steps 30 --warmup 5 --no-sampling --no-cpu-baseline --no-fp32 --no-roofline"
J="import json,sys; d=json.loads([l for l in sys.stdin if l.startswith('{')][-1]); print(sys.argv[1], d['value'], d['ms_per_step'])"
for rep in 1 2; do
for ww in 8,16 8,16,32 8,16,32,64; do
  DV_WINDOW_W=$ww timeout -k 10 300 python bench.py $B 2>/dev/null | python -c "$J" "W=$ww" || exit 1
done
done
