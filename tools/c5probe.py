"""Config-5 shape eager unet forward (bf16 autocast, no_grad) with the live
kernel timer: prints the mid attention's operand dtypes and which MQA path ran
(bf16 streamed / fp8 PV) with its time:  python tools/c5probe.py"""
import sys, os
sys.path.insert(0, "dalle2-video_amd")
import torch
from dalle2_video.dalle2_video import Unet3D
from dalle2_video.utils import deterministic_fill_
from dalle2_video import ops
dev = "cuda"
u = Unet3D(64, video_embed_dim=512, channels=3, dim_mults=(1, 2, 4, 8)).to(dev)
deterministic_fill_(u)
orig = ops.MQAFn.forward
def fwd(ctx, q, kv, null_kv, B, N, H, scale, gm=True):
    print("mqa q", q.dtype, tuple(q.shape), "kv", kv.dtype, "B N H", B, N, H, flush=True)
    return orig(ctx, q, kv, null_kv, B, N, H, scale, gm)
ops.MQAFn.forward = staticmethod(fwd)
for fp8 in (False, True):
    u.fp8 = fp8
    ops.TIMER = ops.KernelTimer()
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16), ops.private_pack_cache():
        xin = torch.randn(2, 3, 32, 128, 128, device=dev)
        tin = torch.full((2,), 500, device=dev, dtype=torch.long)
        u(xin, tin)
        ops.TIMER.records.clear()
        u(xin, tin)
    s = ops.TIMER.summary(); ops.TIMER = None
    for k, v in s.items():
        if k.startswith("attn"): print(fp8, k, v, flush=True)
