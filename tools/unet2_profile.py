"""Per-kernel time of one cascade-SR unet2 forward (BASELINE config 4: dim 8,
mults 1..16, lowres conditioning, 16x256x256, bs 1), bf16, KernelTimer."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dalle2-video_amd"))
import torch  # noqa: E402

from dalle2_video import dalle2_video as D, ops  # noqa: E402
from dalle2_video.utils import deterministic_fill_  # noqa: E402

u1 = D.Unet3D(64, video_embed_dim=512, channels=3, dim_mults=(1, 2, 4, 8))
u2 = D.Unet3D(8, video_embed_dim=512, channels=3, dim_mults=(1, 2, 4, 8, 16))
dec = D.VideoDecoder(unet=(u1, u2), frame_sizes=(64, 256), frame_numbers=(16, 16), timesteps=250,
                     learned_variance=False)
deterministic_fill_(dec.unets[1])
un = dec.unets[1].cuda()
x = torch.randn(1, 3, 16, 256, 256, device="cuda")
low = torch.randn(1, 3, 16, 256, 256, device="cuda")
t = torch.full((1,), 100, device="cuda", dtype=torch.long)
with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
    for _ in range(2):
        un(x, t, lowres_cond_video=low)
    torch.cuda.synchronize()
    ops.TIMER = ops.KernelTimer()
    un(x, t, lowres_cond_video=low)
    summ = ops.TIMER.summary(by_shape=True)
    ops.TIMER = None
tot = sum(v["ms"] for v in summ.values())
print(f"timed launches: {tot:.3f} ms")
for (k, shp), v in sorted(summ.items(), key=lambda kv: -kv[1]["ms"])[:25]:
    print(f"{v['ms']*1e3:8.1f} us {v['count']:3d}  {k:40s} {shp}")

# GPU time of the whole forward (every kernel, incl. GroupNorm / attention):
# replays of one captured HIP graph, under a private (static) pack cache
with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16), ops.private_pack_cache():
    for _ in range(2):
        un(x, t, lowres_cond_video=low)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        un(x, t, lowres_cond_video=low)
        ops.gn_graph_boundary(x.device)
    g.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
knobs = " ".join(f"{k}={v}" for k, v in sorted(os.environ.items()) if k.startswith("DV_"))
print(f"unet2 forward (graph replay): {e0.elapsed_time(e1) / 20:.3f} ms  [{knobs}]")
