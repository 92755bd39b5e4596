# GPU tests, quick bench, kernel trace of a short graph bench (per-step breakdown via tools/step_families.py)
export TMPDIR=/tmp
tag=$1
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tests_$tag.log 2>&1 && tail -2 gpurun_out/tests_$tag.log && \
timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline > gpurun_out/bench_$tag.log 2>&1 && tail -1 gpurun_out/bench_$tag.log | cut -c1-230 && \
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tr_$tag -o run -- python3 bench.py --steps 3 --warmup 2 --no-cpu-baseline --no-roofline > gpurun_out/tr_$tag.log 2>&1
