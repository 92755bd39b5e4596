"""Micro-benchmark: forward conv with / without the GroupNorm statistics
epilogue (dv_conv_fwd gn_sums) at the Cfg2 shapes, and the separate reduce it
replaces (dv_gn_fwd with / without sums_replicas)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dalle2-video_amd"))
import torch  # noqa: E402

from dalle2_video import ops  # noqa: E402
from dalle2_video._lib import call, ptr, stream, dt  # noqa: E402
from kbench import timeit  # noqa: E402


def case(nb, T, h, w, cin, cout, R_list=(0, 8, 64), x1c=0):
    nf = nb * T
    dtype = torch.bfloat16
    x = torch.randn(nf, h, w, cin - x1c, device="cuda", dtype=dtype)
    x1 = torch.randn(nf, h, w, x1c, device="cuda", dtype=dtype) if x1c else None
    wt = torch.randn(cout, cin, 1, 3, 3, device="cuda") / (cin * 9) ** 0.5
    b = torch.randn(cout, device="cuda")
    y = torch.empty(nf, h, w, cout, device="cuda", dtype=dtype)
    P = T * h * w
    sums = torch.zeros(64 * nb * cout * 2, device="cuda")
    c0 = cin - x1c
    win = ops.window_ok(x, x1, cin, c0, cout, c0, x1c or c0, cout, 0, 3, h, w, nf, P)
    wp = ops.pack_conv_weight(wt, dtype, cin, 2 if win else 0)
    out = []
    for R in R_list:
        gs = ptr(sums) if R else None
        if win:
            fn = lambda: call("dv_conv_fwd8", dt(x), ptr(x), c0, c0, ptr(x1), x1c, ptr(wp), ptr(b), None, 0, None, 0,
                              ptr(y), cout, nf, h, w, cin, cout, 0, gs, P, R, stream())
        else:
            fn = lambda: call("dv_conv_fwd", dt(x), ptr(x), c0, c0, ptr(x1), x1c, ptr(wp), ptr(b), None, 0, None, 0,
                              ptr(y), cout, nf, h, w, cin, cout, 3, 0, gs, P, R, stream())
        out.append(timeit(fn) * 1e3)
    # the separate GroupNorm reduce + apply vs apply only
    g = torch.ones(cout, device="cuda")
    be = torch.zeros(cout, device="cuda")
    yo = torch.empty_like(y)
    mean = torch.empty(nb * 8, device="cuda")
    rstd = torch.empty_like(mean)
    nxt = torch.zeros(8 * nb * cout * 2, device="cuda")
    gn = []
    for ready in (0, 8):
        fn = lambda: call("dv_gn_fwd", dt(y), ptr(y), cout, ptr(yo), cout, None, 0, nb, P, cout, 8,
                          ops.ctypes_float(1e-5), ptr(g), ptr(be), None, 1, ptr(mean), ptr(rstd),
                          ptr(sums), ptr(nxt), nxt.numel(), ready, stream())
        gn.append(timeit(fn) * 1e3)
    print(f"{nf}x{h}x{w} {cin}->{cout} ({'window' if win else 'dv_conv_fwd'}): conv "
          + " ".join(f"R={R}:{t:7.1f}us" for R, t in zip(R_list, out))
          + f" | gn reduce+apply {gn[0]:6.1f} us, apply only {gn[1]:6.1f} us", flush=True)


if __name__ == "__main__":
    case(4, 16, 64, 64, 64, 64)              # stage-0 block convs (stripe)
    case(4, 16, 64, 64, 128, 64, x1c=64)     # up3 block1 (glds 256x64, dual source)
    case(4, 16, 32, 32, 192, 128, x1c=64)    # up2
    case(4, 16, 16, 16, 384, 256, x1c=128)   # up1 (window 16)
    case(4, 16, 8, 8, 512, 512)              # mid (window 8)
