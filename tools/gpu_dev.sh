# quick GPU iteration: gpu tests, bench (no cpu baseline), rocprof kernel stats
export TMPDIR=/tmp
tag=$1
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tests_$tag.log 2>&1 && tail -3 gpurun_out/tests_$tag.log && \
timeout -k 10 120 python tools/kbench.py > gpurun_out/kb_$tag.log 2>&1 && timeout -k 10 60 python tools/redbench.py > gpurun_out/rb_$tag.log 2>&1 && timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_$tag.log 2>&1 && tail -1 gpurun_out/bench_$tag.log | cut -c1-300 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$tag -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-roofline > gpurun_out/prof_$tag.log 2>&1 && \
python tools/prof_summary.py gpurun_out/prof_$tag/run_kernel_stats.csv 7 40 > gpurun_out/summary_$tag.txt
