# window conv peeled loop (c3) + row-window wgrad single-barrier stages with the DMA in the MFMA shadow (c4):
# parity of the product build (= c4), phase stamps, per-launch window conv, step A/B c1 / c3 / c4
export TMPDIR=/tmp DV_PARITY_LOG=gpurun_out/parity_r03n.jsonl; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -q -x --timeout 300 --timeout-method thread tests/test_conv_gpu.py tests/test_cfg2_gpu.py tests/test_unet_gpu.py > gpurun_out/tests_r03n.log 2>&1 || { tail -30 gpurun_out/tests_r03n.log; exit 1; }
tail -2 gpurun_out/tests_r03n.log
DV_HIP_LIB=dalle2-video_amd/csrc/build_stamp/libdv_hip_stamp.so timeout -k 10 120 python tools/wgrad_stamp.py > gpurun_out/stamp_r03n.txt 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/stamp_r03n.txt
for v in c1 c3; do DV_HIP_LIB=tools/_ab/libdv_hip_$v.so timeout -k 10 120 python tools/frame_ab.py $v >> gpurun_out/frame_ab_r03n.txt 2>/dev/null || exit 1; done
grep -v amdgpu gpurun_out/frame_ab_r03n.txt
bash tools/ab_env.sh DV_HIP_LIB "tools/_ab/libdv_hip_c1.so tools/_ab/libdv_hip_c3.so tools/_ab/libdv_hip_c4.so" ab_r03n
