# backward GroupNorm (reduce + apply) launch targets (graph-timed probe, bwd column)
export TMPDIR=/tmp
cd tools
for cfg in "768 768" "384 768" "768 384" "384 384" "1536 1536"; do
  set -- $cfg
  echo "TR1=$1 TA1=$2"; DV_GN_TR1=$1 DV_GN_TA1=$2 timeout -k 10 100 python gn_bw.py 2>/dev/null | awk -F'|' '{print $1 "|" $4}' || exit 1
done
