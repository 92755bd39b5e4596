# unet2 forward (graph replay) under the xe forward tile knobs and GroupNorm apply knobs
mkdir -p gpurun_out
run() {  # tag, env assignments...
  local tag=$1; shift
  env "$@" timeout -k 10 200 python tools/unet2_profile.py > gpurun_out/xs_$tag.log 2>&1 || exit 1
  echo "$tag: $(grep -E "'fwd', 1048576, 8, (72|144|16|1350)" gpurun_out/xs_$tag.log | awk '{printf "%s/%s ", $1, $3}') | $(tail -1 gpurun_out/xs_$tag.log)"
}
run base DV_XE_R=8
run r4 DV_XE_R=4
run r16 DV_XE_R=16
run wb128 DV_XE_WB=128
run r4wb256 DV_XE_R=4 DV_XE_WB=256
run ua8 DV_GN_UA0=8
run ta512 DV_GN_TA0=512
run ta2048 DV_GN_TA0=2048
run ur4 DV_GN_UR0=4
run tr1536 DV_GN_TR0=1536
