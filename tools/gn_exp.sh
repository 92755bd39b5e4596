# GroupNorm apply A/B: register prologue per direction (DV_GN_DIRECT bits: 1 fwd, 2 bwd)
export TMPDIR=/tmp
cd tools
for d in 0 1 3; do
  echo "DIRECT=$d"; DV_GN_DIRECT=$d timeout -k 10 100 python gn_bw.py 2>/dev/null | cut -c1-150 || exit 1
done
