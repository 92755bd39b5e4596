# window-conv iteration: conv parity tests, then the kbench forward cases with and without it
export TMPDIR=/tmp
tag=$1
timeout -k 10 300 python -u -m pytest tests/test_conv_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/conv_$tag.log 2>&1; rc=$?; tail -4 gpurun_out/conv_$tag.log; [ $rc -eq 0 ] && \
timeout -k 10 120 python tools/kbench.py fwd > gpurun_out/kb8_$tag.log 2>&1 && grep "conv" gpurun_out/kb8_$tag.log && \
DV_NO_WINDOW=1 timeout -k 10 120 python tools/kbench.py fwd > gpurun_out/kb8n_$tag.log 2>&1 && grep "conv" gpurun_out/kb8n_$tag.log
