# glds implicit GEMM with per-row DMA state (tap mask + uniform tap offset, weight K offset in soffset): parity,
# per-shape forward times (kbench fwd) and step A/B vs c3
export TMPDIR=/tmp DV_PARITY_LOG=gpurun_out/parity_r03p.jsonl; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -q -x --timeout 300 --timeout-method thread tests/test_conv_gpu.py tests/test_cfg2_gpu.py tests/test_unet_gpu.py tests/test_cascade_gpu.py > gpurun_out/tests_r03p.log 2>&1 || { tail -30 gpurun_out/tests_r03p.log; exit 1; }
tail -2 gpurun_out/tests_r03p.log
for v in c3 c6; do echo "== $v" >> gpurun_out/kbench_r03p.txt; DV_HIP_LIB=tools/_ab/libdv_hip_$v.so timeout -k 10 180 python tools/kbench.py fwd >> gpurun_out/kbench_r03p.txt 2>/dev/null || exit 1; done
cat gpurun_out/kbench_r03p.txt
bash tools/ab_env.sh DV_HIP_LIB "tools/_ab/libdv_hip_c3.so tools/_ab/libdv_hip_c6.so" ab_r03p
