"""Micro-bench of the memory-bound 1x1 convs of the Cfg2 up path (res_conv
128 -> 64 forward, and its dgrad 64 -> 128 accumulated into dX), for tile A/B
(DV_GLDS_SMALLK=0/1)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dalle2-video_amd"))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import torch  # noqa: E402

from dalle2_video import ops  # noqa: E402
from dalle2_video._lib import call, ptr, stream, dt  # noqa: E402
from kbench import timeit  # noqa: E402


def case(cin, cout, acc):
    nf, h, w = 64, 64, 64
    x = torch.randn(nf, h, w, cin, device="cuda", dtype=torch.bfloat16)
    wt = torch.randn(cout, cin, 1, 1, 1, device="cuda") / cin ** 0.5
    wp = ops.pack_conv_weight(wt, torch.bfloat16, cin, 0)
    y = torch.randn(nf, h, w, cout, device="cuda", dtype=torch.bfloat16)
    res = y if acc else None
    fn = lambda: call("dv_conv_fwd", dt(x), ptr(x), cin, cin, None, 0, ptr(wp), None, ptr(res),
                      cout if acc else 0, ptr(y), cout, nf, h, w, cin, cout, 1, 0, None, 0, 0, stream())
    ms = timeit(fn, iters=50)
    m = nf * h * w
    nbytes = 2 * m * (cin + cout * (2 if acc else 1))
    print(f"1x1 {cin}->{cout} acc={acc}: {ms * 1e3:7.1f} us  {nbytes / ms / 1e9:6.2f} TB/s "
          f"(SMALLK={os.environ.get('DV_GLDS_SMALLK', '0')})")


if __name__ == "__main__":
    case(128, 64, False)
    case(64, 128, True)
    case(256, 128, False)
    case(128, 256, True)
