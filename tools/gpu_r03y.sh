# round-3 evidence run of the final tree: PMC passes first (their traffic JSON is what bench.py's roofline reads),
# then tests + bench + rocprof (tools/gpu_round.sh), then the phase stamps of the diagnostic build
export TMPDIR=/tmp; mkdir -p gpurun_out
bash tools/gpu_pmc_families.sh r03y || exit 1
cp gpurun_out/pmc_traffic_r03y.json profiles/pmc_traffic_r03y.json || exit 1
bash tools/gpu_round.sh r03y || exit 1
DV_HIP_LIB=dalle2-video_amd/csrc/build_stamp/libdv_hip_stamp.so timeout -k 10 120 python tools/wgrad_stamp.py > gpurun_out/stamp_r03y.txt 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/stamp_r03y.txt
