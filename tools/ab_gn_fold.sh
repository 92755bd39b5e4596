# GroupNorm fold A/B on one box: parity tests, then the default bench (config 2
# leg only) alternating fold on / off, then a rocprof step summary with the fold.
#   bash tools/ab_gn_fold.sh <tag>
export TMPDIR=/tmp
tag=$1
mkdir -p gpurun_out
timeout -k 10 100 python tools/gn_fold_probe.py > gpurun_out/probe_$tag.log 2>&1 && cat gpurun_out/probe_$tag.log | tail -1 && timeout -k 10 700 python -u -m pytest tests/test_gn_fold_gpu.py tests/test_conv_gpu.py tests/test_cfg2_trainer_gpu.py tests/test_gn_coop_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/tests_$tag.log 2>&1 || { tail -40 gpurun_out/tests_$tag.log; exit 1; }
tail -2 gpurun_out/tests_$tag.log
B="--no-cpu-baseline --no-sampling --no-fp32 --no-config3"
for i in 1 2; do
  timeout -k 10 300 python bench.py $B > gpurun_out/ab_on${i}_$tag.log 2>&1 || { tail -20 gpurun_out/ab_on${i}_$tag.log; exit 1; }
  timeout -k 10 300 python tools/bench_gn_fold_off.py $B > gpurun_out/ab_off${i}_$tag.log 2>&1 || { tail -20 gpurun_out/ab_off${i}_$tag.log; exit 1; }
  echo "on: $(tail -1 gpurun_out/ab_on${i}_$tag.log | cut -c1-200)"
  echo "off: $(tail -1 gpurun_out/ab_off${i}_$tag.log | cut -c1-200)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$tag -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-roofline --no-sampling --no-fp32 --no-config3 > gpurun_out/prof_$tag.log 2>&1 && \
python tools/prof_summary.py gpurun_out/prof_$tag/run_kernel_trace.csv 60 3 > gpurun_out/summary_$tag.txt && head -24 gpurun_out/summary_$tag.txt
rm -rf gpurun_out/prof_$tag
