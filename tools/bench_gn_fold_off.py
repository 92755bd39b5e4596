"""bench.py with the Block3D -> Block3D GroupNorm fold switched off
(ops.GN_FOLD = False): the same-box A/B of tools/ab_gn_fold.sh.
  python tools/bench_gn_fold_off.py [bench.py args]"""
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dalle2-video_amd"))
from dalle2_video import ops  # noqa: E402

ops.GN_FOLD = False
sys.argv = [os.path.join(ROOT, "bench.py")] + sys.argv[1:]
runpy.run_path(sys.argv[0], run_name="__main__")
