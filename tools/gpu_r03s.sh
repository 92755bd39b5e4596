# round-3 evidence run of the tree (tests + bench + rocprof + phase stamps + PMC), plus the mid-attention
# forward with K/V streamed at Cfg2 (DV_MQA_STREAM) A/B
export TMPDIR=/tmp; mkdir -p gpurun_out
bash tools/gpu_round.sh r03s || exit 1
DV_HIP_LIB=dalle2-video_amd/csrc/build_stamp/libdv_hip_stamp.so timeout -k 10 120 python tools/wgrad_stamp.py > gpurun_out/stamp_r03s.txt 2>&1 || exit 1
for v in 0 1; do DV_MQA_STREAM=$v timeout -k 10 120 python tools/attnbench.py >> gpurun_out/attn_r03s.txt 2>/dev/null || exit 1; done
cat gpurun_out/attn_r03s.txt
bash tools/gpu_pmc_families.sh r03s
