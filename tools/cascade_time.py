"""Config-4 cascade timing split: whole sample() cold and warm, and the pure
denoise-loop time per stage (graph replays) for comparison."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dalle2-video_amd"))
import torch  # noqa: E402

from dalle2_video import dalle2_video as D  # noqa: E402
from dalle2_video.utils import deterministic_fill_  # noqa: E402

u1 = D.Unet3D(64, video_embed_dim=512, channels=3, dim_mults=(1, 2, 4, 8))
u2 = D.Unet3D(8, video_embed_dim=512, channels=3, dim_mults=(1, 2, 4, 8, 16))
dec = D.VideoDecoder(unet=(u1, u2), frame_sizes=(64, 256), frame_numbers=(16, 16), timesteps=250,
                     learned_variance=False)
for un in dec.unets:
    deterministic_fill_(un)
dec = dec.cuda()
emb = torch.randn(1, 512, device="cuda")
orig = D.VideoDecoder.p_sample_loop_ddpm


def timed_loop(self, *a, **k):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    out = orig(self, *a, **k)
    torch.cuda.synchronize()
    print(f"   p_sample_loop_ddpm {a[1]}: {time.perf_counter() - t0:.3f} s", flush=True)
    return out


D.VideoDecoder.p_sample_loop_ddpm = timed_loop
with torch.autocast("cuda", dtype=torch.bfloat16):
    for rep in range(2):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        vid = dec.sample(video_embed=emb)
        torch.cuda.synchronize()
        print(f"sample() run {rep}: {time.perf_counter() - t0:.3f} s", flush=True)
