# A/B: frame kernel wave index masked (DMA piece types fold), wgrad prefetch depth 6
export TMPDIR=/tmp; mkdir -p gpurun_out
for v in base c1 c2; do DV_HIP_LIB=tools/_ab/libdv_hip_$v.so timeout -k 10 120 python tools/frame_ab.py $v >> gpurun_out/frame_ab_r03l.txt 2>/dev/null || exit 1; done
grep -v amdgpu gpurun_out/frame_ab_r03l.txt
bash tools/ab_env.sh DV_HIP_LIB "tools/_ab/libdv_hip_base.so tools/_ab/libdv_hip_c1.so tools/_ab/libdv_hip_c2.so" ab_r03l
