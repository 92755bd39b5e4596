export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 120 python tools/cfg5_profile.py > gpurun_out/cfg5_bf16.log 2>&1; tail -12 gpurun_out/cfg5_bf16.log
DV_FP8=1 timeout -k 10 120 python tools/cfg5_profile.py > gpurun_out/cfg5_fp8.log 2>&1; tail -30 gpurun_out/cfg5_fp8.log
