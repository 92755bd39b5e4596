# GPU check: tests, default bench (with cpu_baseline), rocprof kernel stats of the graph bench
export TMPDIR=/tmp
tag=$1
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tests_$tag.log 2>&1 && tail -3 gpurun_out/tests_$tag.log && \
timeout -k 10 300 python bench.py > gpurun_out/bench_$tag.log 2>&1 && tail -1 gpurun_out/bench_$tag.log | cut -c1-400 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$tag -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-roofline > gpurun_out/prof_$tag.log 2>&1 && \
python tools/prof_summary.py gpurun_out/prof_$tag/run_kernel_stats.csv 7 60 > gpurun_out/summary_$tag.txt
