# glds ring depth for the many-tile grids (DV_GLDS_RING): per-shape forward + step A/B; GN statistics epilogue everywhere (DV_GN_STATS_ALL)
export TMPDIR=/tmp; mkdir -p gpurun_out
for v in auto deep mid; do echo "== $v" >> gpurun_out/kbench_r03r.txt; DV_GLDS_RING=$([ $v = auto ] && echo "" || echo $v) timeout -k 10 180 python tools/kbench.py fwd >> gpurun_out/kbench_r03r.txt 2>/dev/null || exit 1; done
cat gpurun_out/kbench_r03r.txt
bash tools/ab_env.sh DV_GLDS_RING "x deep mid" ab_r03r_ring
bash tools/ab_env.sh DV_GN_STATS_ALL "0 1" ab_r03r_gnstats
