export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_cfg2_gpu.py tests/test_conv_gpu.py > gpurun_out/dbg.log 2>&1; tail -3 gpurun_out/dbg.log
