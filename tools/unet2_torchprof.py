"""torch-side ops of one cascade unet2 forward (copies / fills / elementwise
that are not HIP-extension launches), from torch.profiler."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dalle2-video_amd"))
import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402

from dalle2_video import dalle2_video as D  # noqa: E402
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
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], with_stack=True) as prof:
        un(x, t, lowres_cond_video=low)
        torch.cuda.synchronize()
print(prof.key_averages(group_by_stack_n=6).table(sort_by="self_cuda_time_total", row_limit=25,
                                                    max_name_column_width=60))
