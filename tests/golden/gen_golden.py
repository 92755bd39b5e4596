"""Generate the golden fixtures under tests/golden/ (run in the build container).

The reference cannot be imported as a package here (termcolor, x_clip,
coca_pytorch and dalle2-pytorch 1.14.2 are absent — ordinary import errors,
SURVEY §8c).  Its torch-only 3-D classes, however, execute verbatim: this
script AST-extracts `Downsample3D`, `PixelShuffleUpsample3D`,
`temporal_apply`, `Block3D`, `ResnetBlock3D`, `CrossEmbedLayer3D` and `Unet3D`
from `/root/reference/dalle2_video/dalle2_video.py` AT RUN TIME, executes them
with the oracle's restated dalle2-pytorch leaves, checks the oracle against
them, and writes small .npz fixtures (data only — no reference source is
stored in the repo).

Fixtures
  g1_blocks.npz    reference Block3D / ResnetBlock3D / CrossEmbedLayer3D /
                   Downsample3D / PixelShuffleUpsample3D outputs (independent)
  g2_unet_cfg1.npz reference Unet3D wiring + restated leaves, Cfg1 input
                   (1,3,8,32,32), time=[537] (semi-independent)
  g3_sched.npz     NoiseScheduler tables, cosine + linear (closed form)
  g4_plosses.npz   p_losses value + a 3-step training trace on a small unet
Usage: python tests/golden/gen_golden.py [--check]   (--check: compare only)
"""
from __future__ import annotations

import ast
import os
import sys
from functools import partial
from typing import Any, Callable, Dict, List, Optional, Tuple, Union

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F
from einops import pack, rearrange, repeat, unpack
from einops.layers.torch import Rearrange

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
from oracle import dv_ref as R  # noqa: E402

REF_FILE = "/root/reference/dalle2_video/dalle2_video.py"
WANTED = {"Downsample3D", "NearestUpsample3D", "PixelShuffleUpsample3D", "temporal_apply",
          "Block3D", "ResnetBlock3D", "CrossEmbedLayer3D", "Unet3D"}


def load_reference_classes():
    src = open(REF_FILE).read()
    tree = ast.parse(src)
    body = [n for n in tree.body
            if isinstance(n, (ast.FunctionDef, ast.ClassDef)) and n.name in WANTED]
    assert {n.name for n in body} == WANTED, "reference layout changed"
    mod = ast.Module(body=body, type_ignores=[])

    class _NeverResnetBlock:  # the 2-D dalle2 ResnetBlock (Q5 isinstance check)
        pass

    ns: Dict[str, Any] = dict(
        torch=torch, nn=nn, F=F, rearrange=rearrange, repeat=repeat, pack=pack, unpack=unpack,
        Rearrange=Rearrange, partial=partial, Any=Any, Callable=Callable, Optional=Optional,
        Tuple=Tuple, List=List, Dict=Dict, Union=Union,
        exists=R.exists, default=R.default, cast_tuple=R.cast_tuple, first=R.first,
        maybe=R.maybe, identity=R.identity, zero_init_=R.zero_init_,
        prob_mask_like=R.prob_mask_like, LayerNorm=R.LayerNorm,
        SinusoidalPosEmb=R.SinusoidalPosEmb, Residual=R.Residual,
        RearrangeToSequence=R.RearrangeToSequence, Attention=R.Attention,
        CrossAttention=R.CrossAttention, UpsampleCombiner=R.UpsampleCombiner,
        ResnetBlock=_NeverResnetBlock, make_checkpointable=None, LinearAttention=None,
    )
    exec(compile(mod, REF_FILE, "exec"), ns)
    return ns


def rel(a, b):
    a, b = a.double(), b.double()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def same_weights(dst: nn.Module, src: nn.Module):
    dst.load_state_dict(src.state_dict(), strict=True)


def build_unet(cls, dim, mults, lowres):
    u = cls(dim, video_embed_dim=512, channels=3, dim_mults=mults, cond_on_text_encodings=False)
    return u.cast_model_parameters(lowres_cond=lowres, lowres_noise_cond=False, channels=3,
                                   channels_out=3, cond_on_image_embeds=not lowres,
                                   cond_on_text_encodings=False)


def gen(check_only=False):
    torch.manual_seed(0)
    ref = load_reference_classes()
    out = {}

    # ---------------- G1: component blocks (independent) ----------------
    g1 = {}
    gen_ = torch.Generator().manual_seed(1234)
    x = torch.randn(1, 32, 4, 16, 16, generator=gen_)
    x3 = torch.rand(1, 3, 4, 16, 16, generator=gen_)
    temb = torch.randn(1, 128, generator=gen_)
    cond = torch.randn(1, 2, 32, generator=gen_)
    g1.update(x=x, x3=x3, temb=temb, cond=cond)
    cases = {
        "block": (lambda ns: ns["Block3D"](32, 48), lambda m: m(x)),
        "block_ss": (lambda ns: ns["Block3D"](32, 48),
                     lambda m: m(x, scale_shift=(0.1 * temb[:, :48, None, None, None],
                                                 0.1 * temb[:, 48:96, None, None, None]))),
        "resnet": (lambda ns: ns["ResnetBlock3D"](32, 64, time_cond_dim=128),
                   lambda m: m(x, temb)),
        "resnet_xattn": (lambda ns: ns["ResnetBlock3D"](32, 64, cond_dim=32, time_cond_dim=128),
                         lambda m: m(x, temb, cond)),
        "crossembed": (lambda ns: ns["CrossEmbedLayer3D"](3, dim_out=32, kernel_sizes=(3, 7, 15),
                                                          stride=1), lambda m: m(x3)),
        "downsample": (lambda ns: ns["Downsample3D"](32, 64), lambda m: m(x)),
        "pixelshuffle": (lambda ns: ns["PixelShuffleUpsample3D"](32, 16), lambda m: m(x)),
    }
    oracle_ns = dict(Block3D=R.Block3D, ResnetBlock3D=R.ResnetBlock3D,
                     CrossEmbedLayer3D=R.CrossEmbedLayer3D, Downsample3D=R.Downsample3D,
                     PixelShuffleUpsample3D=R.PixelShuffleUpsample3D)
    for name, (mk, run) in cases.items():
        m_ref = R.deterministic_fill_(mk(ref))
        m_or = mk(oracle_ns)
        same_weights(m_or, m_ref)
        with torch.no_grad():
            y_ref, y_or = run(m_ref), run(m_or)
        e = rel(y_or, y_ref)
        print(f"G1 {name:14s} oracle vs reference rel-err {e:.2e}")
        assert e < 1e-6, name
        g1[f"y_{name}"] = y_ref
    out["g1_blocks"] = g1

    # ---------------- G2: Unet3D forward at Cfg1 ----------------
    u_ref = R.deterministic_fill_(build_unet(ref["Unet3D"], 64, (1, 2, 4, 8), False))
    assert u_ref.cond_on_video_embeds is False and u_ref.to_video_hiddens is None  # Q3
    u_or = build_unet(R.Unet3D, 64, (1, 2, 4, 8), False)
    assert list(u_or.state_dict().keys()) == list(u_ref.state_dict().keys())
    same_weights(u_or, u_ref)
    gen_ = torch.Generator().manual_seed(1234)
    x = torch.randn(1, 3, 8, 32, 32, generator=gen_)
    times = torch.tensor([537])
    with torch.no_grad():
        y_ref = u_ref(x, times, video_embed=torch.randn(1, 512, generator=gen_))
        y_or, inter = u_or(x, times, return_intermediates=True)
    e = rel(y_or, y_ref)
    print(f"G2 unet1 cfg1 oracle vs reference rel-err {e:.2e}  |y|={y_ref.abs().mean():.4f}")
    assert e < 1e-6
    g2 = dict(x=x, times=times, y=y_ref)
    for k, v in inter.items():
        g2[f"sum_{k}"] = v.double().sum().reshape(1)
        g2[f"abssum_{k}"] = v.double().abs().sum().reshape(1)
        g2[f"head_{k}"] = v.flatten()[:256].clone()
    # unet2 (cascade SR unet: lowres_cond, 6 input channels) — small input
    u2_ref = R.deterministic_fill_(build_unet(ref["Unet3D"], 8, (1, 2, 4, 8, 16), True))
    u2_or = build_unet(R.Unet3D, 8, (1, 2, 4, 8, 16), True)
    same_weights(u2_or, u2_ref)
    x2 = torch.randn(1, 3, 4, 32, 32, generator=gen_)
    lo = torch.randn(1, 3, 4, 32, 32, generator=gen_)
    t2 = torch.tensor([11])
    with torch.no_grad():
        y2_ref = u2_ref(x2, t2, video_embed=None, lowres_cond_video=lo)
        y2_or = u2_or(x2, t2, lowres_cond_video=lo)
    e2 = rel(y2_or, y2_ref)
    print(f"G2 unet2 oracle vs reference rel-err {e2:.2e}")
    assert e2 < 1e-6
    g2.update(x2=x2, lowres2=lo, times2=t2, y2=y2_ref)
    out["g2_unet_cfg1"] = g2

    # ---------------- G3: scheduler tables ----------------
    g3 = {}
    for sch in ("cosine", "linear"):
        s = R.NoiseScheduler(beta_schedule=sch, timesteps=1000, loss_type="l2")
        for b in R.NoiseScheduler.BUFFERS:
            g3[f"{sch}_{b}"] = getattr(s, b)
    out["g3_sched"] = g3

    # ---------------- G4: p_losses + 3-step training trace ----------------
    sched = R.NoiseScheduler(beta_schedule="cosine", timesteps=1000, loss_type="l2")
    u4 = R.deterministic_fill_(build_unet(R.Unet3D, 16, (1, 2, 4, 8), False))
    gen_ = torch.Generator().manual_seed(1234)
    xs = torch.rand(2, 3, 4, 32, 32, generator=gen_)
    times = torch.tensor([537, 3])
    noise = torch.randn(xs.shape, generator=gen_)
    loss0 = R.p_losses(u4, sched, xs, times, noise, video_cond_drop_prob=0.0,
                       text_cond_drop_prob=0.0)
    opt = R.get_optimizer(u4.parameters(), lr=3e-4, wd=1e-2)
    losses = []
    for step in range(3):
        losses.append(R.train_step(u4, sched, opt, xs, times, noise,
                                   video_cond_drop_prob=0.0, text_cond_drop_prob=0.0))
    psum = sum(p.double().sum() for p in u4.parameters())
    g4 = dict(x=xs, times=times, noise=noise, loss0=loss0.detach().reshape(1),
              losses=torch.tensor(losses), param_sum=psum.reshape(1),
              to_out_w=u4.to_out.weight.detach().flatten())
    print(f"G4 loss0={loss0.item():.6f} trace={losses} param_sum={psum.item():.6f}")
    out["g4_plosses"] = g4

    for name, d in out.items():
        path = os.path.join(HERE, f"{name}.npz")
        arrs = {k: (v.detach().numpy() if torch.is_tensor(v) else np.asarray(v))
                for k, v in d.items()}
        if check_only:
            old = np.load(path)
            for k, v in arrs.items():
                assert np.allclose(old[k], v, rtol=1e-5, atol=1e-6), (name, k)
            print(f"checked {path}")
        else:
            np.savez_compressed(path, **arrs)
            print(f"wrote {path} ({os.path.getsize(path) / 1024:.0f} KiB)")


if __name__ == "__main__":
    gen(check_only="--check" in sys.argv)
