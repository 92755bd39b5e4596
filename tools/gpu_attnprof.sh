export TMPDIR=/tmp
tag=$1
timeout -k 10 120 python tools/attnbench.py > gpurun_out/ab_$tag.log 2>&1 && cat gpurun_out/ab_$tag.log | grep mqa && \
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/aprof_$tag -o run --output-format csv -- python3 tools/attnbench.py > gpurun_out/aprof_$tag.log 2>&1 && \
python tools/prof_summary.py gpurun_out/aprof_$tag/run_kernel_stats.csv 43 12
