"""Debug HIP-graph replay vs eager: per-parameter gradient differences."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "dalle2-video_amd"))
import torch  # noqa: E402

from dalle2_video import dalle2_video as D  # noqa: E402
from dalle2_video.trainer import VideoDecoderTrainer  # noqa: E402
from dalle2_video.utils import deterministic_fill_  # noqa: E402

u = D.Unet3D(16, video_embed_dim=512, channels=3, dim_mults=(1, 2, 4, 8))
dec = D.VideoDecoder(u, frame_sizes=(32,), frame_numbers=(4,), timesteps=1000, learned_variance=False)
deterministic_fill_(dec.unets[0])
dec = dec.cuda()
tr = VideoDecoderTrainer(dec, lr=3e-4, use_ema=False, use_graphs=True)
g = torch.Generator(device="cuda").manual_seed(3)
video = torch.rand(2, 3, 4, 32, 32, device="cuda", generator=g)
torch.cuda.manual_seed(1)
tr(video=video, unet_number=1)
tr.update(1)
opt = tr.optim0
G = opt.flat_grad
names = {id(p): n for n, p in dec.named_parameters()}
res = {}
seq = [("A", 7), ("B", 8)] + [(f"R{i}", 7 + (i % 2)) for i in range(10)]
flat = {}
for tag, seed in seq:
    opt.zero_grad()
    torch.cuda.manual_seed(seed)
    loss = tr(video=video, unet_number=1)
    torch.cuda.synchronize()
    grads = {}
    for n, p in dec.named_parameters():
        if p.grad is not None:
            inside = G.data_ptr() <= p.grad.data_ptr() < G.data_ptr() + G.numel() * 4
            grads[n] = (p.grad.detach().clone(), inside)
    res[tag] = (loss, grads)
    flat[tag] = G.clone()
    ref = flat["A"] if seed == 7 else flat.get("B", G)
    print(tag, "loss", loss, "flat norm", G.norm().item(), "max|G|", G.abs().max().item(),
          "rel vs eager", ((G - ref).norm() / ref.norm()).item())
for e, gph in (("A", "R0"), ("B", "R1"), ("A", "R2"), ("B", "R3")):
    bad = []
    for n, (ge, ie) in res[e][1].items():
        gg, ig = res[gph][1][n]
        err = ((ge - gg).norm() / ge.norm().clamp_min(1e-30)).item()
        if err > 1e-4 or ie != ig:
            bad.append((err, n, ie, ig))
    bad.sort(reverse=True)
    print(e, gph, "bad params:", len(bad))
    for b in bad[:15]:
        print("   ", b)
