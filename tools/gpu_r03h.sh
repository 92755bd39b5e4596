# round-3 A/B evidence: MX-fp8 kernels (tests, per-shape times vs bf16 at the
# config-5 shape), window-conv variants, bf16 vs f32 split-K partials
export TMPDIR=/tmp DV_PARITY_LOG=gpurun_out/parity_r03h.jsonl; mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -q --timeout 200 --timeout-method thread tests/test_mx8_gpu.py "tests/test_conv_gpu.py::test_stripe_wgrad_bf16_partials" "tests/test_trainer_gpu.py::test_deferred_wgrad_sum_matches_per_conv_sum" > gpurun_out/tests_r03h.log 2>&1; tail -3 gpurun_out/tests_r03h.log; grep -E "^E " gpurun_out/tests_r03h.log | head
grep -q " failed\|error" gpurun_out/tests_r03h.log && exit 1
bash tools/gpu_frame_ab.sh > gpurun_out/frame_ab.log 2>&1 || exit 1; grep -v amdgpu.ids gpurun_out/frame_ab.log
DV_FP8=0 timeout -k 10 150 python tools/cfg5_profile.py > gpurun_out/cfg5_bf16.log 2>&1 || exit 1; tail -3 gpurun_out/cfg5_bf16.log
DV_FP8=1 timeout -k 10 150 python tools/cfg5_profile.py > gpurun_out/cfg5_fp8.log 2>&1 || exit 1; tail -3 gpurun_out/cfg5_fp8.log
DV_FP8=1 DV_FP8_ALL=1 timeout -k 10 150 python tools/cfg5_profile.py > gpurun_out/cfg5_fp8all.log 2>&1 || exit 1; tail -3 gpurun_out/cfg5_fp8all.log
bash tools/ab_env.sh DV_WG_F32PART "0 1" ab_part || exit 1
