export TMPDIR=/tmp DV_PARITY_LOG=gpurun_out/parity_r03h.jsonl; mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_mx8_gpu.py > gpurun_out/tests_r03h.log 2>&1; tail -3 gpurun_out/tests_r03h.log; grep -E "^E " gpurun_out/tests_r03h.log | head
bash tools/gpu_frame_ab.sh > gpurun_out/frame_ab.log 2>&1; cat gpurun_out/frame_ab.log | grep -v amdgpu.ids
DV_FP8=1 DV_FP8_ALL=1 timeout -k 10 120 python tools/cfg5_profile.py > gpurun_out/cfg5_fp8all.log 2>&1; tail -22 gpurun_out/cfg5_fp8all.log
