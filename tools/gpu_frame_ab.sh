# A/B of the window conv's fragment prefetch distance / deferred last tap
export TMPDIR=/tmp
for v in "2 0" "3 0" "2 1" "3 1"; do set -- $v; DV_FRAME_PF=$1 DV_FRAME_DEFER=$2 timeout -k 10 120 python tools/frame_ab.py pf$1d$2 || exit 1; done
