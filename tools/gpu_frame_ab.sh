# per-launch A/B of the window conv at the Cfg2 8x8 / 16x16 shapes: 32-channel
# tiles for the grids that leave CUs idle (DV_FRAME_CO32=1, default) vs 64 only
export TMPDIR=/tmp
for v in 1 0; do DV_FRAME_CO32=$v timeout -k 10 120 python tools/frame_ab.py co32_$v || exit 1; done
