# fused GroupNorm -> MX-fp8 quantisation: tests, config-5 forward with / without
# the fusion at both fp8 coverages, and the training step after the frame defaults
export TMPDIR=/tmp DV_PARITY_LOG=gpurun_out/parity_r03i.jsonl; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -q -x --timeout 300 --timeout-method thread tests/test_mx8_gpu.py tests/test_conv_gpu.py > gpurun_out/tests_r03i.log 2>&1; tail -3 gpurun_out/tests_r03i.log; grep -E "^E " gpurun_out/tests_r03i.log | head
grep -q " failed\|error" gpurun_out/tests_r03i.log && exit 1
for cfg in "1 0" "1 1" "0 1" "0 0"; do set -- $cfg
  DV_FP8=1 DV_FP8_FUSE=$1 DV_FP8_ALL=$2 timeout -k 10 150 python tools/cfg5_profile.py > gpurun_out/cfg5_f$1a$2.log 2>&1 || exit 1
  echo "fuse=$1 all=$2: $(tail -1 gpurun_out/cfg5_f$1a$2.log)"
done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-roofline --no-fp32 > gpurun_out/bench_r03i.log 2>&1 || exit 1
tail -1 gpurun_out/bench_r03i.log | python -c "import json,sys; d=json.load(sys.stdin); print(d['value'], json.dumps(d['sampling'].get('config5_fp8'))[:300], d['sampling']['config5_bf16']['value'])"
