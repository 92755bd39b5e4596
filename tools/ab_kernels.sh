# same-box per-kernel A/B: rocprofv3 kernel stats of the graph bench under VAR=v for each v
# bash tools/ab_kernels.sh VAR "v1 v2" filter
export TMPDIR=/tmp
var=$1; vals=$2; flt=$3
mkdir -p gpurun_out
for v in $vals; do
  t=$(basename "$v" .so)
  env $var=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/abk_$t -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-roofline --no-sampling --no-fp32 > gpurun_out/abk_$t.log 2>&1 || exit 1
  echo "== $var=$v: $(grep 'train:' gpurun_out/abk_$t.log | tail -1)"
  python tools/trace_shapes.py gpurun_out/abk_$t/run_kernel_trace.csv 7 $flt | head -14
done
