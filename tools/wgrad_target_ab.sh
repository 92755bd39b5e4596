export TMPDIR=/tmp
for v in 512 2048 4096; do
  DV_WGRAD_TARGET=$v timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/wt_$v -o run -- python3 bench.py --steps 3 --warmup 2 --no-cpu-baseline --no-roofline > gpurun_out/wt_$v.log 2>&1 || exit 1
done
