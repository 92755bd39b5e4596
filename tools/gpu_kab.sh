#!/bin/bash
# same-box per-kernel A/B of two builds of libdv_hip (tools/_ab/libdv_hip_base.so
# vs the in-tree one): conv parity on the new build, then base / new / base /
# new replayed steps under rocprofv3 --kernel-trace, and the per-launch mean of
# every kernel whose name matches $2 in each trace.
#   bash tools/gpu_kab.sh <tag> <kernel-name regex>
export TMPDIR=/tmp
tag=${1:-kab}
pat=${2:-conv}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_conv_gpu.py -x -q --timeout 300 --timeout-method thread \
  > gpurun_out/tests_$tag.log 2>&1
rc=$?
tail -3 gpurun_out/tests_$tag.log
[ $rc = 0 ] || exit 1
B="--steps 5 --warmup 2 --no-cpu-baseline --no-roofline --no-sampling --no-fp32"
for rep in 1 2; do
  for v in base new; do
    if [ $v = base ]; then export DV_HIP_LIB=tools/_ab/libdv_hip_base.so; else unset DV_HIP_LIB; fi
    timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/kab_${tag}_$v$rep -o run \
      --output-format csv -- python3 bench.py $B > gpurun_out/kab_${tag}_$v$rep.log 2>&1 || exit 1
    python tools/prof_summary.py gpurun_out/kab_${tag}_$v$rep/run_kernel_trace.csv 400 3 \
      | python -c "import re,sys; [print('$v$rep', l.rstrip()) for l in sys.stdin if re.search(sys.argv[1], l)]" "$pat"
  done
done
