export TMPDIR=/tmp
tag=$1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_cfg5_gpu.py tests/test_conv_gpu.py tests/test_sample_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/tests_$tag.log 2>&1 || { tail -30 gpurun_out/tests_$tag.log; exit 1; }
tail -1 gpurun_out/tests_$tag.log
B="--steps 5 --warmup 3 --no-cpu-baseline --no-fp32 --no-config3 --no-roofline"
ex='import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); s=d["sampling"]; print("train", d["value"], "bs4", s["bs4"]["value"], "bs1", s["bs1"]["value"], "c5 bf16", s["config5_bf16"]["value"], "c5 fp8", s["config5_fp8"]["value"], "cascade", s["cascade"]["value"])'
for i in 1 2; do
  timeout -k 10 400 python bench.py $B > gpurun_out/ab128on${i}_$tag.log 2>&1 || { tail -20 gpurun_out/ab128on${i}_$tag.log; exit 1; }
  echo "on : $(python3 -c "$ex" gpurun_out/ab128on${i}_$tag.log)"
  timeout -k 10 400 python tools/bench_gn_stats128_off.py $B > gpurun_out/ab128off${i}_$tag.log 2>&1 || { tail -20 gpurun_out/ab128off${i}_$tag.log; exit 1; }
  echo "off: $(python3 -c "$ex" gpurun_out/ab128off${i}_$tag.log)"
done
