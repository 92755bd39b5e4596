# Same-box A/B of an ops switch: the given GPU tests, then the default bench
# (config 2 leg only) alternating the switch's default / off state, then a
# rocprof step summary of the default.
#   bash tools/ab_switch.sh <tag> <SWITCH=VALUE> [test files...]
export TMPDIR=/tmp
tag=$1; sw=$2; shift 2
mkdir -p gpurun_out
if [ $# -gt 0 ]; then
  timeout -k 10 900 python -u -m pytest "$@" -x -q --timeout 300 --timeout-method thread > gpurun_out/tests_$tag.log 2>&1 || { tail -40 gpurun_out/tests_$tag.log; exit 1; }
  tail -2 gpurun_out/tests_$tag.log
fi
B="--no-cpu-baseline --no-sampling --no-fp32 --no-config3"
for i in 1 2 3; do
  timeout -k 10 300 python bench.py $B > gpurun_out/ab_on${i}_$tag.log 2>&1 || { tail -20 gpurun_out/ab_on${i}_$tag.log; exit 1; }
  timeout -k 10 300 python tools/bench_switch.py $sw $B > gpurun_out/ab_off${i}_$tag.log 2>&1 || { tail -20 gpurun_out/ab_off${i}_$tag.log; exit 1; }
  echo "default: $(tail -1 gpurun_out/ab_on${i}_$tag.log | cut -c1-120)"
  echo "$sw: $(tail -1 gpurun_out/ab_off${i}_$tag.log | cut -c1-120)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$tag -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-roofline --no-sampling --no-fp32 --no-config3 > gpurun_out/prof_$tag.log 2>&1 && \
python tools/prof_summary.py gpurun_out/prof_$tag/run_kernel_trace.csv 60 3 > gpurun_out/summary_$tag.txt && head -30 gpurun_out/summary_$tag.txt
rm -rf gpurun_out/prof_$tag
