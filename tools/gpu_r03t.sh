# row-window wgrad epilogue: one-pass halves sum, bf16 tiles transposed by all four waves in one round,
# 16-B partial stores (c8) vs c7: parity, phase stamps, step A/B
export TMPDIR=/tmp DV_PARITY_LOG=gpurun_out/parity_r03t.jsonl; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -q -x --timeout 300 --timeout-method thread tests/test_conv_gpu.py tests/test_cfg2_gpu.py tests/test_trainer_gpu.py tests/test_cfg2_trainer_gpu.py > gpurun_out/tests_r03t.log 2>&1 || { tail -30 gpurun_out/tests_r03t.log; exit 1; }
tail -2 gpurun_out/tests_r03t.log
DV_HIP_LIB=dalle2-video_amd/csrc/build_stamp/libdv_hip_stamp.so timeout -k 10 120 python tools/wgrad_stamp.py > gpurun_out/stamp_r03t.txt 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/stamp_r03t.txt
bash tools/ab_env.sh DV_HIP_LIB "tools/_ab/libdv_hip_c7.so tools/_ab/libdv_hip_c8.so" ab_r03t
