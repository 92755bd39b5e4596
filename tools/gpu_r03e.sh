export TMPDIR=/tmp DV_PARITY_LOG=gpurun_out/parity_r03e.jsonl; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_mx8_gpu.py tests/test_trainer_gpu.py > gpurun_out/tests_r03e.log 2>&1; tail -3 gpurun_out/tests_r03e.log
DV_DEFER_STREAM=0 timeout -k 10 200 python bench.py --steps 20 --no-fp32 --no-cpu-baseline --no-sampling --no-roofline > gpurun_out/bench_r03e_s0.log 2>/dev/null; cut -c1-120 gpurun_out/bench_r03e_s0.log
DV_DEFER_STREAM=1 timeout -k 10 200 python bench.py --steps 20 --no-fp32 --no-cpu-baseline --no-sampling --no-roofline > gpurun_out/bench_r03e_s1.log 2>/dev/null; cut -c1-120 gpurun_out/bench_r03e_s1.log
timeout -k 10 400 python bench.py --steps 10 --no-fp32 --no-cpu-baseline > gpurun_out/bench_r03e.log 2> gpurun_out/bench_r03e.err; tail -5 gpurun_out/bench_r03e.err
