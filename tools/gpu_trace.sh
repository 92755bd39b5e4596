# kernel trace of the graph bench + per-category step breakdown (last step)
export TMPDIR=/tmp
tag=$1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$tag -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-roofline > gpurun_out/prof_$tag.log 2>&1 && \
python3 tools/step_breakdown.py gpurun_out/prof_$tag/run_kernel_trace.csv
