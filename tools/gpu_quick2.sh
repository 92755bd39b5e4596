# quick GPU iteration: all GPU tests, training bench (no extra legs), rocprof of the graph bench
export TMPDIR=/tmp
tag=$1
mkdir -p gpurun_out
export DV_PARITY_LOG=gpurun_out/parity_$tag.jsonl
rm -f $DV_PARITY_LOG
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/tests_$tag.log 2>&1; rc=$?
tail -15 gpurun_out/tests_$tag.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline --no-sampling --no-fp32 > gpurun_out/bench_$tag.log 2> gpurun_out/bench_$tag.err && tail -3 gpurun_out/bench_$tag.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$tag -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-roofline --no-sampling --no-fp32 > gpurun_out/prof_$tag.log 2>&1 && \
python tools/step_families.py gpurun_out/prof_$tag/run_kernel_trace.csv 30 > gpurun_out/families_$tag.txt && cat gpurun_out/families_$tag.txt
