#!/bin/bash
# round-5 check: full GPU suite on the cleaned library, the window wgrad A/B
# (DV_WG_ISS 0 / 2, the stripe kernel DV_WG_OLD=1), and the step A/B
export TMPDIR=/tmp
tag=${1:-r05e}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 || { tail -30 gpurun_out/${tag}_tests.log; exit 1; }
tail -2 gpurun_out/${tag}_tests.log
for rep in 1 2; do
  for v in 0 2; do
    DV_WG_ISS=$v timeout -k 10 120 python tools/wgrad_ab.py 2>/dev/null | sed "s/^/ISS=$v /" >> gpurun_out/${tag}_wg.log || exit 1
  done
done
DV_WG_OLD=1 timeout -k 10 120 python tools/wgrad_ab.py 2>/dev/null | sed "s/^/OLD /" >> gpurun_out/${tag}_wg.log || exit 1
grep total gpurun_out/${tag}_wg.log
bash tools/ab_env.sh DV_WG_ISS "0 2" ${tag}_step
