export TMPDIR=/tmp DV_PARITY_LOG=gpurun_out/parity_r03c.jsonl; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_mx8_gpu.py > gpurun_out/tests_r03c.log 2>&1; tail -15 gpurun_out/tests_r03c.log
cat gpurun_out/parity_r03c.jsonl
