# window conv: chunk loop peeled (no per-piece branch), split input templated; parity + per-launch + step A/B vs the masked-wave build
export TMPDIR=/tmp DV_PARITY_LOG=gpurun_out/parity_r03m.jsonl; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -q -x --timeout 300 --timeout-method thread tests/test_conv_gpu.py tests/test_cfg2_gpu.py tests/test_unet_gpu.py > gpurun_out/tests_r03m.log 2>&1 || { tail -30 gpurun_out/tests_r03m.log; exit 1; }
tail -2 gpurun_out/tests_r03m.log
for v in c1 c3; do DV_HIP_LIB=tools/_ab/libdv_hip_$v.so timeout -k 10 120 python tools/frame_ab.py $v >> gpurun_out/frame_ab_r03m.txt 2>/dev/null || exit 1; done
grep -v amdgpu gpurun_out/frame_ab_r03m.txt
bash tools/ab_env.sh DV_HIP_LIB "tools/_ab/libdv_hip_c1.so tools/_ab/libdv_hip_c3.so" ab_r03m
