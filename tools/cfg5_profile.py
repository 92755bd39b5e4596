"""Unet1 forward at a sampling shape -- default the BASELINE config-5 shape (32 frames
x 128 x 128, bs 2, bf16; argv: bs frames size [fp8]) -- per-shape conv times
(KernelTimer) and the whole forward by HIP-graph replay; a 4th argument `fp8`
runs the MX-fp8 sampling mode (Unet3D.fp8)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dalle2-video_amd"))
import torch  # noqa: E402

from dalle2_video import dalle2_video as D, ops  # noqa: E402
from dalle2_video.utils import deterministic_fill_  # noqa: E402

un = D.Unet3D(64, video_embed_dim=512, channels=3, dim_mults=(1, 2, 4, 8))
deterministic_fill_(un)
un = un.cuda()
un.fp8 = len(sys.argv) > 4 and sys.argv[4] == "fp8"
bs, fr, sz = (int(v) for v in (sys.argv[1:4] if len(sys.argv) > 3 else (2, 32, 128)))
x = torch.randn(bs, 3, fr, sz, sz, device="cuda")
emb = torch.randn(bs, 512, device="cuda")
t = torch.full((bs,), 100, device="cuda", dtype=torch.long)
with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16), ops.private_pack_cache():
    for _ in range(2):
        un(x, t, video_embed=emb)
    torch.cuda.synchronize()
    ops.TIMER = ops.KernelTimer()
    un(x, t, video_embed=emb)
    summ = ops.TIMER.summary(by_shape=True)
    ops.TIMER = None
    tot = sum(v["ms"] for v in summ.values())
    print(f"timed launches: {tot:.3f} ms")
    for (k, shp), v in sorted(summ.items(), key=lambda kv: -kv[1]["ms"])[:25]:
        print(f"{v['ms']*1e3:8.1f} us {v['count']:3d}  {k:40s} {shp}")
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        un(x, t, video_embed=emb)
        ops.gn_graph_boundary(x.device)
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
print(f"unet1 forward bs={bs} {fr}x{sz}x{sz} (graph replay): {e0.elapsed_time(e1) / 10:.3f} ms")
