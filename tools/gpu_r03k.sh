# row-window wgrad prefetch: parity (conv + Cfg2), phase stamps, same-box step A/B vs the HEAD build
export TMPDIR=/tmp DV_PARITY_LOG=gpurun_out/parity_r03k.jsonl; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -q -x --timeout 300 --timeout-method thread tests/test_conv_gpu.py tests/test_cfg2_gpu.py > gpurun_out/tests_r03k.log 2>&1 || { tail -30 gpurun_out/tests_r03k.log; exit 1; }
tail -2 gpurun_out/tests_r03k.log
DV_HIP_LIB=dalle2-video_amd/csrc/build_stamp/libdv_hip_stamp.so timeout -k 10 120 python tools/wgrad_stamp.py > gpurun_out/stamp_r03k.txt 2>&1 || exit 1
cat gpurun_out/stamp_r03k.txt | grep -v amdgpu.ids
bash tools/ab_env.sh DV_HIP_LIB "dalle2-video_amd/dalle2_video/libdv_hip.so tools/_ab/libdv_hip_base.so" ab_r03k
