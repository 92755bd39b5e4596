# per-kernel GroupNorm durations at the Cfg2 shapes (kernel trace of tools/gn_bw.py); env passes through
export TMPDIR=/tmp
mkdir -p gpurun_out
t=${1:-x}
cd tools && timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d ../gpurun_out/gntr$t -o run -- python3 gn_bw.py > ../gpurun_out/gntr$t.log 2>&1 && cd .. && \
python tools/trace_by_grid.py gpurun_out/gntr$t/run_kernel_trace.csv gn_reduce | sed 's/(anonymous namespace):://g' | cut -c1-150
