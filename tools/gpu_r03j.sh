# window conv 32-channel tiles (tests + per-launch A/B), the full bench, and
# same-box step A/B of the window widths / wgrad split floor
export TMPDIR=/tmp DV_PARITY_LOG=gpurun_out/parity_r03j.jsonl; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -q -x --timeout 300 --timeout-method thread tests/test_conv_gpu.py tests/test_cfg2_gpu.py tests/test_mx8_gpu.py > gpurun_out/tests_r03j.log 2>&1; tail -3 gpurun_out/tests_r03j.log; grep -E "^E " gpurun_out/tests_r03j.log | head
grep -q " failed\|error" gpurun_out/tests_r03j.log && exit 1
bash tools/gpu_frame_ab.sh > gpurun_out/frame_ab2.log 2>&1 || exit 1; grep -v amdgpu.ids gpurun_out/frame_ab2.log
timeout -k 10 500 python bench.py > gpurun_out/bench_r03j.log 2> gpurun_out/bench_r03j.err || exit 1
tail -1 gpurun_out/bench_r03j.log | python -c "import json,sys; d=json.load(sys.stdin); s=d['sampling']; print(d['value'], d['roofline']['frac'], s['config5_bf16']['value'], s['config5_bf16']['loops_s'], s['config5_fp8']['value'], s['config5_fp8']['loops_s'], s['config5_fp8']['roofline'])"
bash tools/ab_env.sh DV_WINDOW_W "8,16 8,16,32" ab_window || exit 1
bash tools/ab_env.sh DV_WG_MINST "1 2 4" ab_minst || exit 1
