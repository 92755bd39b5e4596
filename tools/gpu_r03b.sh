export TMPDIR=/tmp DV_PARITY_LOG=gpurun_out/parity_r03b.jsonl; mkdir -p gpurun_out
timeout -k 5 60 tools/probes/mx8_probe > gpurun_out/mx8_probe.log 2>&1; cat gpurun_out/mx8_probe.log
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_cfg2_trainer_gpu.py tests/test_cfg3_unet2_gpu.py tests/test_dp_trainer_gpu.py > gpurun_out/tests_r03b.log 2>&1; tail -8 gpurun_out/tests_r03b.log
timeout -k 10 120 python tools/cfg5_profile.py > gpurun_out/cfg5_prof.log 2>&1; tail -30 gpurun_out/cfg5_prof.log
