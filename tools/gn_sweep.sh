# GroupNorm launch-shape sweep: gnbench under rocprofv3 kernel trace per config, then a quick bench
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "gn or group or norm or block or resnet" > gpurun_out/gn_tests.log 2>&1 && tail -2 gpurun_out/gn_tests.log && \
cd tools && \
run() {
  tag=$1; shift
  env "$@" timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d ../gpurun_out/gns_$tag -o run -- python3 gnbench.py > ../gpurun_out/gns_$tag.log 2>&1
}
run A DV_GN_UR0=8 && \
run D DV_GN_UA0=2 DV_GN_TA0=1024 DV_GN_UA1=2 DV_GN_TA1=768 DV_GN_UR1=2 DV_GN_TR1=768 && \
run E DV_GN_UR0=4 DV_GN_TR0=1536 DV_GN_UA0=2 DV_GN_TA0=1024 DV_GN_UA1=2 DV_GN_TA1=768 DV_GN_UR1=2 DV_GN_TR1=1536 && \
cd .. && timeout -k 10 300 python bench.py --no-cpu-baseline --no-roofline > gpurun_out/bench_q.log 2>&1 && tail -1 gpurun_out/bench_q.log | cut -c1-300
