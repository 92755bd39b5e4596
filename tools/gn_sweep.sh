# GroupNorm launch-shape sweep: gnbench under rocprofv3 kernel trace per DV_GN_* config
export TMPDIR=/tmp
cd tools
run() {
  tag=$1; shift
  env "$@" timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d ../gpurun_out/gns_$tag -o run -- python3 gnbench.py > ../gpurun_out/gns_$tag.log 2>&1
}
run A DV_GN_UR0=8 && \
run B DV_GN_UA0=2 DV_GN_TA0=2048 DV_GN_UR1=2 DV_GN_TR1=1536 && \
run C DV_GN_TA0=2048 DV_GN_TR0=1536 DV_GN_TR1=1536 DV_GN_TA1=1536 && \
run D DV_GN_UR1=2 DV_GN_TR1=768 DV_GN_UA0=2 DV_GN_TA0=1024 && \
run E DV_GN_UR0=4 DV_GN_TR0=768 DV_GN_UR1=8 DV_GN_TR1=512
