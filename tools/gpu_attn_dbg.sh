#!/bin/bash
export TMPDIR=/tmp
mkdir -p gpurun_out
out=gpurun_out/attn_dbg.log
: > $out
for v in "DV_MQA_PAIR=0" "DV_MQA_PAIR=1" "DV_MQA_PAIR=1 DV_MQA_STREAM=1" "DV_MQA_PAIR=0 DV_MQA_STREAM=1"; do
  echo "== $v" >> $out
  env $v timeout -k 10 120 python -u tools/attnbench.py --short >> $out 2>&1 || exit 1
done
