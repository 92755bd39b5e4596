"""bf16 conv forward of every Cfg2 3x3 shape vs torch's own f32 conv on the GPU
(rel-err, max |y|).   python tools/conv_shape_check.py"""
import os
import sys

import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "dalle2-video_amd"), ROOT]
from dalle2_video import ops  # noqa: E402

SHAPES = [  # nf, h, w, c0, c1, cout
    (64, 16, 16, 128, 0, 256), (64, 16, 16, 256, 0, 256), (64, 16, 16, 256, 256, 256),
    (64, 16, 16, 256, 128, 256), (64, 8, 8, 256, 0, 512), (64, 8, 8, 512, 0, 512),
    (64, 8, 8, 512, 512, 512), (64, 8, 8, 512, 256, 512), (64, 8, 8, 256, 0, 256),
    (64, 16, 16, 512, 0, 256), (64, 32, 32, 128, 0, 128), (64, 32, 32, 64, 0, 128),
    (64, 16, 16, 64, 0, 128), (16, 16, 16, 128, 0, 256), (64, 16, 16, 160, 0, 256),
]
torch.manual_seed(0)
for nf, h, w, c0, c1, cout in SHAPES:
    x0 = torch.randn(nf, h, w, c0, device="cuda").bfloat16()
    x1 = torch.randn(nf, h, w, c1, device="cuda").bfloat16() if c1 else None
    wt = (torch.randn(cout, c0 + c1, 1, 3, 3, device="cuda") / (9 * (c0 + c1)) ** 0.5)
    b = torch.randn(cout, device="cuda") * 0.1
    with torch.no_grad():
        y = ops.conv(x0, wt, b, x1=x1) if c1 else ops.conv(x0, wt, b)
        xx = x0 if x1 is None else torch.cat([x0, x1], -1)
        ref = F.conv2d(xx.float().permute(0, 3, 1, 2), wt[:, :, 0].float(), b, padding=1).permute(0, 2, 3, 1)
    torch.cuda.synchronize()
    err = ((y.float() - ref).norm() / ref.norm()).item()
    print(f"{(nf, h, w, c0, c1, cout)!s:34} rel {err:.2e}  max|y| {y.float().abs().max().item():.3e}",
          flush=True)
