# forward GroupNorm apply launch shape: workgroup target x rows in flight (gnbench fwd times)
export TMPDIR=/tmp
for ta in 256 512 1024 2048 4096; do
  for ua in 2 4 8; do
    echo "TA0=$ta UA0=$ua $(DV_GN_TA0=$ta DV_GN_UA0=$ua timeout -k 10 60 python tools/gnbench.py 2>/dev/null | head -3 | awk '{print $6, $7}' | tr '\n' ' ')" || exit 1
  done
done
