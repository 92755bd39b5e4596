export TMPDIR=/tmp DV_PARITY_LOG=gpurun_out/parity_r03f.jsonl; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread tests -m gpu -x > gpurun_out/tests_r03f.log 2>&1; tail -5 gpurun_out/tests_r03f.log; grep -E "FAIL|Error" gpurun_out/tests_r03f.log | head -20
