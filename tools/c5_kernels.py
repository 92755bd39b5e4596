"""Config-5 shape (unet1 sampling forward, 2 x 3 x 32 x 128^2, no_grad, bf16
autocast): the live kernel timer's per-kernel totals of one forward, bf16 vs
the MX-fp8 mode (Unet3D.fp8).  `python tools/c5_kernels.py [bf16|fp8]` runs one
mode only (for a rocprofv3 kernel trace of every launch).
"""
import sys, os
sys.path.insert(0, "dalle2-video_amd")
import torch
from dalle2_video.dalle2_video import Unet3D
from dalle2_video.utils import deterministic_fill_
from dalle2_video import ops
dev = "cuda"
u = Unet3D(64, video_embed_dim=512, channels=3, dim_mults=(1, 2, 4, 8)).to(dev)
deterministic_fill_(u)
res = {}
modes = {"bf16": (False,), "fp8": (True,)}.get(sys.argv[1] if len(sys.argv) > 1 else "", (False, True))
for fp8 in modes:
    u.fp8 = fp8
    ops.TIMER = ops.KernelTimer()
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16), ops.private_pack_cache():
        xin = torch.randn(2, 3, 32, 128, 128, device=dev)
        tin = torch.full((2,), 500, device=dev, dtype=torch.long)
        u(xin, tin)
        ops.TIMER.records.clear()
        u(xin, tin)
    res[fp8] = ops.TIMER.summary(); ops.TIMER = None
for fp8, s in res.items():
    tot = sum(v["ms"] for v in s.values())
    print(f"== fp8={fp8} timed total {tot:.3f} ms")
    for k, v in sorted(s.items(), key=lambda kv: -kv[1]["ms"])[:14]:
        print(f"   {v['ms']:7.3f} ms  n={v['count']:3d}  {k}")
