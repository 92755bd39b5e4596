# same-box A/B of a GroupNorm launch knob over the whole training step
export TMPDIR=/tmp
for v in "$@"; do
  DV_GN_MINB=$v timeout -k 10 200 python bench.py --no-cpu-baseline --no-sampling --no-fp32 --no-roofline --steps 40 2>&1 >/dev/null | grep train: | sed "s/^/minb=$v /"
done
