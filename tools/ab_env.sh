# same-box A/B of an env knob on the training step: bash tools/ab_env.sh VAR "v1 v2 ..." [tag]
export TMPDIR=/tmp
var=$1; vals=$2; tag=${3:-ab}
mkdir -p gpurun_out
for rep in 1 2; do
  for v in $vals; do
    r=$(env $var=$v timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-roofline --no-sampling --no-fp32 2>/dev/null | tail -1 | python -c "import json,sys; print(json.load(sys.stdin)['value'])") || exit 1
    echo "$var=$v rep$rep: $r steps/s" | tee -a gpurun_out/$tag.log
  done
done
