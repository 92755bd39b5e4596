"""Find the first Unet3D submodule whose bf16 output holds a NaN / Inf at Cfg2
(forward hooks, synchronised).   python tools/nan_probe.py"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "dalle2-video_amd"), ROOT]
from dalle2_video import dalle2_video as D  # noqa: E402
from oracle import dv_ref as R  # noqa: E402


def build(mod):
    u = mod.Unet3D(64, video_embed_dim=512, channels=3, dim_mults=(1, 2, 4, 8),
                   cond_on_text_encodings=False)
    return u.cast_model_parameters(lowres_cond=False, lowres_noise_cond=False, channels=3,
                                   channels_out=3, cond_on_image_embeds=True,
                                   cond_on_text_encodings=False)


ou = R.deterministic_fill_(build(R))
u = build(D)
u.load_state_dict(ou.state_dict(), strict=True)
u = u.cuda()
u.compute_dtype = torch.bfloat16
bad = []


def hook(name):
    def f(mod, inp, out):
        outs = out if isinstance(out, (tuple, list)) else (out,)
        for o in outs:
            if torch.is_tensor(o) and o.is_floating_point():
                torch.cuda.synchronize()
                if not torch.isfinite(o).all():
                    bad.append((name, type(mod).__name__, tuple(o.shape)))
    return f


from dalle2_video import ops  # noqa: E402
import inspect  # noqa: E402


def wrap(name, fn):
    def w(*a, **k):
        out = fn(*a, **k)
        outs = out if isinstance(out, (tuple, list)) else (out,)
        for o in outs:
            if torch.is_tensor(o) and o.is_floating_point() and o.is_cuda:
                torch.cuda.synchronize()
                if not torch.isfinite(o).all() or o.float().abs().max() > 1e3:
                    shp = [(tuple(t.shape), t.stride()[-2] if t.dim() > 1 else 0, float(t.float().abs().max()), str(t.dtype)) for t in a if torch.is_tensor(t)]
                    nn_ = (~torch.isfinite(o)).float()
                    where = nn_.reshape(o.shape[0], -1).sum(1).nonzero().flatten()[:8].tolist()
                    chans = nn_.reshape(-1, o.shape[-1]).sum(0).nonzero().flatten()[:16].tolist()
                    bad.append((name, tuple(o.shape), shp, "frames", where, "chans", chans,
                                "count", int(nn_.sum())))
        return out
    return w


for n in dir(ops):
    f = getattr(ops, n)
    if inspect.isfunction(f) and f.__module__ == ops.__name__ and not n.startswith("_"):
        setattr(ops, n, wrap(n, f))
    elif inspect.isclass(f) and issubclass(f, torch.autograd.Function):
        f.apply = wrap(n, f.apply)
for n, m in u.named_modules():
    m.register_forward_hook(hook(n))
g = torch.Generator().manual_seed(1234)
x = torch.rand(4, 3, 16, 64, 64, generator=g).cuda() * 2 - 1
with torch.no_grad():
    y = u(x, torch.tensor([0, 537, 999, 250]).cuda(), video_embed=None)
torch.cuda.synchronize()
print("output finite:", bool(torch.isfinite(y).all()))
for b in bad[:15]:
    print("non-finite:", b)
