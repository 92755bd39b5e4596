"""Config 3's unet2 training step alone (for a rocprofv3 kernel trace:
tools/prof_summary.py delimits the steps by their AdamW launches):
VideoDecoderTrainer(use_graphs, amp) on the two-unet decoder, unet_number=2
(128^2, low-res conditioned, blur p = 0.5), 4x3x16x224^2 synthetic clips.

  python tools/unet2_train.py [steps]
"""
import os
import random
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dalle2-video_amd"))
import torch  # noqa: E402

from dalle2_video.dalle2_video import Unet3D, VideoDecoder  # noqa: E402
from dalle2_video.trainer import VideoDecoderTrainer  # noqa: E402
from dalle2_video.utils import deterministic_fill_  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
random.seed(0)
u1 = Unet3D(64, video_embed_dim=512, channels=3, dim_mults=(1, 2, 4, 8), cond_on_text_encodings=False)
u2 = Unet3D(8, video_embed_dim=512, channels=3, dim_mults=(1, 2, 4, 8, 16), cond_on_text_encodings=False)
dec = VideoDecoder(unet=(u1, u2), frame_sizes=(64, 128), frame_numbers=(16, 16), timesteps=1000,
                   learned_variance=False)
for u in dec.unets:
    deterministic_fill_(u)
dec = dec.cuda()
tr = VideoDecoderTrainer(dec, lr=3e-4, wd=1e-2, use_ema=False, amp=True, use_graphs=True)
video = torch.rand(4, 3, 16, 224, 224, device="cuda")
for _ in range(8):
    tr(video=video, unet_number=2)
    tr.update(2)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(steps):
    tr(video=video, unet_number=2)
    tr.update(2)
torch.cuda.synchronize()
print(f"unet2 train step {(time.perf_counter() - t0) / steps * 1e3:.3f} ms, graphs {len(tr._graphs)}")
