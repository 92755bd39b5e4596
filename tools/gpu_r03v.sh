# window conv: 8-wave 128-channel tiles for the two-round 16x16 grids (DV_FRAME_W8): parity, per-launch, step A/B
export TMPDIR=/tmp DV_PARITY_LOG=gpurun_out/parity_r03v.jsonl; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -q -x --timeout 300 --timeout-method thread tests/test_conv_gpu.py tests/test_cfg2_gpu.py tests/test_unet_gpu.py > gpurun_out/tests_r03v.log 2>&1 || { tail -30 gpurun_out/tests_r03v.log; exit 1; }
tail -2 gpurun_out/tests_r03v.log
for v in 0 1; do DV_FRAME_W8=$v timeout -k 10 120 python tools/frame_ab.py w8_$v >> gpurun_out/frame_ab_r03v.txt 2>/dev/null || exit 1; done
grep -v amdgpu gpurun_out/frame_ab_r03v.txt
bash tools/ab_env.sh DV_FRAME_W8 "0 1" ab_r03v
