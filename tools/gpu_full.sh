# full GPU check used during development: tests, bench (graphs), eager bench, rocprof
export TMPDIR=/tmp
timeout -k 10 400 python -m pytest tests -m gpu -q -x 2>&1 | tail -3 && \
timeout -k 10 240 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_$1.log 2>&1 && tail -1 gpurun_out/bench_$1.log | cut -c1-300 && \
timeout -k 10 240 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-roofline --no-graphs 2>&1 | tail -1 | cut -c1-160 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$1 -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-roofline > gpurun_out/prof_$1.log 2>&1
