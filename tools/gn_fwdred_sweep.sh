# forward GroupNorm reduce launch shape (graph-timed probe, fwd reduce+apply column)
export TMPDIR=/tmp
cd tools
for cfg in "768 8" "384 8" "1536 8" "768 4"; do
  set -- $cfg
  echo "TR0=$1 UR0=$2"; DV_GN_TR0=$1 DV_GN_UR0=$2 timeout -k 10 100 python gn_bw.py 2>/dev/null | sed 's/.*C=/C=/' | awk -F'|' '{print $1 "|" $5}' || exit 1
done
