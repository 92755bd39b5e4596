# implicit-GEMM (glds) conv: fragments of k-step s+1 read before the MFMAs of k-step s (g1) vs head (g0): parity, per-kernel, step A/B
export TMPDIR=/tmp DV_PARITY_LOG=gpurun_out/parity_r03w.jsonl; mkdir -p gpurun_out
DV_HIP_LIB=tools/_ab/libdv_hip_g1.so timeout -k 10 600 python -u -m pytest -q -x --timeout 300 --timeout-method thread tests/test_conv_gpu.py tests/test_cfg2_gpu.py > gpurun_out/tests_r03w.log 2>&1 || { tail -30 gpurun_out/tests_r03w.log; exit 1; }
tail -2 gpurun_out/tests_r03w.log
bash tools/ab_kernels.sh DV_HIP_LIB "tools/_ab/libdv_hip_g0.so tools/_ab/libdv_hip_g1.so" glds > gpurun_out/abk_r03w.txt 2>&1 || exit 1
cat gpurun_out/abk_r03w.txt
bash tools/ab_env.sh DV_HIP_LIB "tools/_ab/libdv_hip_g0.so tools/_ab/libdv_hip_g1.so" ab_r03w
