import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dalle2-video_amd"))
import torch
import torch.nn.functional as F
from dalle2_video import ops
torch.set_printoptions(linewidth=200, precision=3)
for dtype in (torch.float32, torch.bfloat16):
    for (nf, h, w, cin, cout, k) in [(1, 8, 8, 64, 64, 1), (2, 8, 8, 64, 64, 3), (1,8,8,8,8,1)]:
        x = torch.randn(nf, h, w, cin)
        wt = torch.randn(cout, cin, 1, k, k) / (cin * k * k) ** 0.5
        if k == 1 and cin == cout:
            wt = torch.eye(cout).reshape(cout, cin, 1, 1, 1)
        xr = x.to(dtype).float(); wr = wt.to(dtype).float()
        yr = F.conv2d(xr.permute(0, 3, 1, 2), wr[:, :, 0], padding=k // 2).permute(0, 2, 3, 1)
        y = ops.conv(x.to("cuda", dtype), wt.cuda()).float().cpu()
        err = (y - yr).abs()
        print(dtype, (nf, h, w, cin, cout, k), "max err", err.max().item(), "rel", (err.norm() / yr.norm()).item())
        if err.max() > 1e-2:
            bad = (err > 1e-2).nonzero()
            print(" first bad idx", bad[:8].tolist())
            print(" y  ", y.reshape(-1, cout)[:2, :16])
            print(" ref", yr.reshape(-1, cout)[:2, :16])
