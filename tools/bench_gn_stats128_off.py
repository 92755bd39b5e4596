"""bench.py without the GroupNorm statistics epilogue on the W = 128 stripe conv
(config 5's 128^2 stage: the GroupNorm reduces z itself): the A/B of that route.
  python tools/bench_gn_stats128_off.py [bench.py args]"""
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dalle2-video_amd"))
from dalle2_video import ops  # noqa: E402

ops.GN_STATS_KERNELS = tuple(k for k in ops.GN_STATS_KERNELS if k != "conv_fwd_stripe_kernel<128>")
sys.argv = [os.path.join(ROOT, "bench.py")] + sys.argv[1:]
runpy.run_path(sys.argv[0], run_name="__main__")
