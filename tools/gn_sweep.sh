# GPU tests, GroupNorm gnbench under rocprofv3 kernel trace, then a quick bench
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gn_tests.log 2>&1 && tail -2 gpurun_out/gn_tests.log && \
cd tools && \
run() {
  tag=$1; shift
  env "$@" timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d ../gpurun_out/gns_$tag -o run -- python3 gnbench.py > ../gpurun_out/gns_$tag.log 2>&1
}
run A DV_GN_UR0=8 && \
cd .. && timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline > gpurun_out/bench_q.log 2>&1 && tail -1 gpurun_out/bench_q.log | cut -c1-300
