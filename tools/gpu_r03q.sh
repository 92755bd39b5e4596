# glds: tap mask without divisions (ks 1 / 3), c7 vs c3
# per-shape forward times (kbench fwd) and step A/B vs c3
export TMPDIR=/tmp DV_PARITY_LOG=gpurun_out/parity_r03q.jsonl; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -q -x --timeout 300 --timeout-method thread tests/test_conv_gpu.py tests/test_cfg2_gpu.py tests/test_unet_gpu.py tests/test_cascade_gpu.py > gpurun_out/tests_r03q.log 2>&1 || { tail -30 gpurun_out/tests_r03q.log; exit 1; }
tail -2 gpurun_out/tests_r03q.log
for v in c3 c7; do echo "== $v" >> gpurun_out/kbench_r03q.txt; DV_HIP_LIB=tools/_ab/libdv_hip_$v.so timeout -k 10 180 python tools/kbench.py fwd >> gpurun_out/kbench_r03q.txt 2>/dev/null || exit 1; done
cat gpurun_out/kbench_r03q.txt
bash tools/ab_env.sh DV_HIP_LIB "tools/_ab/libdv_hip_c3.so tools/_ab/libdv_hip_c7.so" ab_r03q
