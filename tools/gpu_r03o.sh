# row-window wgrad with one barrier per stage, DMA at the stage top (c5) vs two barriers (c3)
export TMPDIR=/tmp DV_PARITY_LOG=gpurun_out/parity_r03o.jsonl; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -q -x --timeout 300 --timeout-method thread tests/test_conv_gpu.py tests/test_cfg2_gpu.py tests/test_unet_gpu.py > gpurun_out/tests_r03o.log 2>&1 || { tail -30 gpurun_out/tests_r03o.log; exit 1; }
tail -2 gpurun_out/tests_r03o.log
DV_HIP_LIB=dalle2-video_amd/csrc/build_stamp/libdv_hip_stamp.so timeout -k 10 120 python tools/wgrad_stamp.py > gpurun_out/stamp_r03o.txt 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/stamp_r03o.txt
bash tools/ab_env.sh DV_HIP_LIB "tools/_ab/libdv_hip_c3.so tools/_ab/libdv_hip_c5.so" ab_r03o
