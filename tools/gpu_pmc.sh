# HBM traffic per kernel: two separate rocprofv3 PMC passes over the (eager) bench
export TMPDIR=/tmp
tag=$1
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmcf_$tag -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-roofline --no-graphs --no-sampling --no-fp32 > gpurun_out/pmcf_$tag.log 2>&1 && \
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmcw_$tag -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-roofline --no-graphs --no-sampling --no-fp32 > gpurun_out/pmcw_$tag.log 2>&1 && \
ls gpurun_out/pmcf_$tag gpurun_out/pmcw_$tag
