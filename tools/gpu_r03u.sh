# MX-fp8 convs without per-piece branches / 64-bit divisions (c9) vs c8: fp8 parity, config-5 forward (graph replay) A/B
export TMPDIR=/tmp DV_PARITY_LOG=gpurun_out/parity_r03u.jsonl; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -q -x --timeout 300 --timeout-method thread tests/test_mx8_gpu.py > gpurun_out/tests_r03u.log 2>&1 || { tail -30 gpurun_out/tests_r03u.log; exit 1; }
tail -2 gpurun_out/tests_r03u.log
for rep in 1 2; do for v in c8 c9; do echo "== $v fp8 rep$rep" >> gpurun_out/cfg5_r03u.txt; DV_FP8=1 DV_HIP_LIB=tools/_ab/libdv_hip_$v.so timeout -k 10 180 python tools/cfg5_profile.py >> gpurun_out/cfg5_r03u.txt 2>/dev/null || exit 1; done; done
grep -E "==|graph|replay|timed" gpurun_out/cfg5_r03u.txt
