"""Per-mode cost of the conv-weight packer (dv_pack_conv_weight) on the Cfg2
unet's largest weights, and the batched repack of every Cfg2 image
(PackCache.refresh), by HIP events over 20 launches each:
  python tools/pack_bench.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dalle2-video_amd"))
import torch  # noqa: E402

from dalle2_video import ops  # noqa: E402


def timed(f, n=20):
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        f()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / n * 1e3


for co, ci, k in [(512, 512, 3), (512, 768, 3), (64, 64, 3), (512, 768, 1)]:
    w = torch.randn(co, ci, 1, k, k, device="cuda")
    for mode in (0, 1, 2, 3):
        pad = ((ci if mode % 2 == 0 else co) + 15) // 16 * 16
        us = timed(lambda: ops.pack_conv_weight(w, torch.bfloat16, pad, mode, cache=False))
        gbs = w.numel() * 6 / us / 1e3
        print(f"({co},{ci},{k}) mode {mode}: {us:7.1f} us  {gbs:6.0f} GB/s (4 B read + 2 B write per element)", flush=True)

# every Cfg2 conv weight, both images (bf16, modes as the convs request them)
from dalle2_video.dalle2_video import Unet3D  # noqa: E402
u = Unet3D(dim=64, video_embed_dim=512, channels=3, dim_mults=(1, 2, 4, 8), cond_on_text_encodings=False).cuda()
cache = ops.PackCache()
cache.enabled = True
n = el = 0
for p in u.parameters():
    if p.dim() != 5 or p.shape[-1] > 3:
        continue
    co, ci, k = p.shape[0], p.shape[1], p.shape[-1]
    for mode in (2, 3) if k == 3 and ci % 16 == 0 and co % 16 == 0 else (0, 1):
        pad = ((ci if mode % 2 == 0 else co) + 15) // 16 * 16
        cache.lookup(p, p.data, torch.bfloat16, co, ci, k, pad, mode)
        n += 1
        el += p.numel()
us = timed(cache.refresh)
print(f"batched repack: {n} images, {el / 1e6:.1f} M elements: {us:.1f} us ({el * 6 / us / 1e3:.0f} GB/s)", flush=True)
