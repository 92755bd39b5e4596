# one iteration: GPU tests, the GroupNorm probe, the default bench (no CPU baseline)
export TMPDIR=/tmp
tag=$1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/tests_$tag.log 2>&1 && tail -2 gpurun_out/tests_$tag.log && \
(cd tools && timeout -k 10 120 python gn_bw.py > ../gpurun_out/gn_bw_$tag.log 2>&1) && cat gpurun_out/gn_bw_$tag.log | grep nb= && \
timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline --no-sampling --no-fp32 > gpurun_out/bench_$tag.log 2>&1 && tail -1 gpurun_out/bench_$tag.log | cut -c1-200
