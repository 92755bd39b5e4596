"""Step-by-step Unet3D forward with a sync after every module (fault localisation)."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "dalle2-video_amd"))
import torch
from dalle2_video import dalle2_video as D
def log(*a):
    torch.cuda.synchronize(); print(*a, flush=True)
u = D.Unet3D(64, video_embed_dim=512, channels=3, dim_mults=(1, 2, 4, 8)).cuda()
x = torch.randn(1, 3, 8, 32, 32, device="cuda"); t = torch.tensor([537], device="cuda")
from dalle2_video import ops
xc = ops.to_cl(x, torch.float32); log("to_cl", xc.shape)
h = u.init_conv.forward_cl(xc); log("init", h.shape)
tt, c, mc = u._conditioning(t, 1, x.device, 0.0, 0.0); log("cond", tt.shape, c.shape)
for i, (_, ib, blocks, attn, post) in enumerate(u.downs):
    h = ib.forward_cl(h, tt, c, 1); log("down", i, "init", h.shape)
    for blk in blocks:
        h = blk.forward_cl(h, tt, c, 1); log("down", i, "blk", h.shape)
    h = post.forward_cl(h); log("down", i, "post", h.shape)
h = u.mid_block1.forward_cl(h, tt, mc, 1); log("mid1")
h = u.mid_attn.forward_cl(h, 1); log("mid_attn")
t0 = time.time()
y = u(x, t); log("full forward", y.shape, time.time() - t0)
with torch.autocast("cuda", dtype=torch.bfloat16):
    y = u(x, t); log("bf16 forward", y.shape)
