export TMPDIR=/tmp; mkdir -p gpurun_out
B="--no-cpu-baseline --no-sampling --no-fp32 --no-config3 --no-roofline"
run() { timeout -k 10 300 python -c "
import os, runpy, sys
sys.path.insert(0, 'dalle2-video_amd')
from dalle2_video import ops
ops.WGRAD_DEFER.FLUSH_BYTES = int(sys.argv[1])
sys.argv = ['bench.py'] + sys.argv[2:]
runpy.run_path('bench.py', run_name='__main__')
" $1 $B 2>/dev/null | tail -1 | python -c "import json,sys; print('flush', sys.argv[1], json.loads(sys.stdin.read())['value'])" $1; }
for i in 1 2; do run 0 && run 134217728 && run 268435456 || exit 1; done
