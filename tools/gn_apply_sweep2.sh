# forward GroupNorm apply launch shape after the register prologue (graph-timed probe, apply column)
export TMPDIR=/tmp
cd tools
for cfg in "256 4" "512 4" "768 4"; do
  set -- $cfg
  echo "TA0=$1 UA0=$2"; DV_GN_TA0=$1 DV_GN_UA0=$2 timeout -k 10 100 python gn_bw.py 2>/dev/null | awk -F'|' '{print $1 "|" $2}' || exit 1
done
