"""Per-launch time of the window-form 3x3 conv (conv_fwd_frame_kernel) at the
Cfg2 8x8 / 16x16 shapes — run once per library build (DV_HIP_LIB selects one;
tools/frame_pmc.sh runs it under the PMC passes):  python tools/frame_ab.py [tag]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dalle2-video_amd"))
import torch  # noqa: E402

from dalle2_video import ops  # noqa: E402
from dalle2_video._lib import call, dt, ptr, stream  # noqa: E402

SHAPES = [(64, 8, 8, 512, 512), (64, 8, 8, 256, 256), (64, 8, 8, 768, 512), (64, 8, 8, 512, 256),
          (64, 16, 16, 256, 256), (64, 16, 16, 384, 256)]


def bench(nf, h, w, cin, cout, iters=50):
    g = torch.Generator(device="cuda").manual_seed(1)
    x = torch.randn(nf, h, w, cin, device="cuda", generator=g).bfloat16()
    wt = torch.randn(cout, cin, 1, 3, 3, device="cuda", generator=g) / (9 * cin) ** 0.5
    b = torch.randn(cout, device="cuda", generator=g)
    y = torch.empty(nf, h, w, cout, device="cuda", dtype=torch.bfloat16)
    wp = ops.pack_conv_weight(wt, torch.bfloat16, cin, 2, cache=False)
    f = lambda: call("dv_conv_fwd8", dt(x), ptr(x), cin, cin, None, 0, ptr(wp), ptr(b), None, 0, None, 0, ptr(y), cout,
                     nf, h, w, cin, cout, 0, None, 0, 0, stream())
    for _ in range(5):
        f()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(iters)]
    for s, e in ev:
        torch.cuda._sleep(200_000)
        s.record()
        f()
        e.record()
    torch.cuda.synchronize()
    t = sorted(s.elapsed_time(e) for s, e in ev)[iters // 2] * 1e3
    ref = torch.nn.functional.conv2d(x.float().permute(0, 3, 1, 2), wt[:, :, 0], b, padding=1).permute(0, 2, 3, 1)
    err = ((y.float() - ref).norm() / ref.norm()).item()
    return t, 2.0 * nf * h * w * cin * cout * 9 / (t * 1e-6) / 1e12, err


tag = sys.argv[1] if len(sys.argv) > 1 else ""
for shp in SHAPES:
    t, tf, err = bench(*shp)
    print(f"{tag:10s} {str(shp):26s} {t:7.2f} us  {tf:6.1f} TF/s  {tf / 2516.6:.3f}  err {err:.1e}", flush=True)
