# batched weight repack over one flat tile space (DV_PACK_FLAT): parity, per-kernel, step A/B
export TMPDIR=/tmp DV_PARITY_LOG=gpurun_out/parity_r03x.jsonl; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -q -x --timeout 300 --timeout-method thread tests/test_conv_gpu.py tests/test_cfg2_trainer_gpu.py tests/test_trainer_gpu.py > gpurun_out/tests_r03x.log 2>&1 || { tail -30 gpurun_out/tests_r03x.log; exit 1; }
tail -2 gpurun_out/tests_r03x.log
bash tools/ab_kernels.sh DV_PACK_FLAT "0 1" pack > gpurun_out/abk_r03x.txt 2>&1 || exit 1
cat gpurun_out/abk_r03x.txt
bash tools/ab_env.sh DV_PACK_FLAT "0 1" ab_r03x
