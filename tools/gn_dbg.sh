export TMPDIR=/tmp
cd tools
run() {
  tag=$1; shift
  env "$@" timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d ../gpurun_out/gns_$tag -o run -- python3 gnbench.py > ../gpurun_out/gns_$tag.log 2>&1
}
run d0 DV_GN_DBG=0 && run d1 DV_GN_DBG=1 && run d2 DV_GN_DBG=2 && run d4 DV_GN_DBG=4 && run d8 DV_GN_DBG=8 && run d15 DV_GN_DBG=15
