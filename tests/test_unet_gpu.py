"""End-to-end parity of the HIP Unet3D against the golden fixtures (G2, pinned
to the reference's own wiring) and the CPU oracle (gradients).

Tolerances (norm-wise relative error):
  f32 mode forward   <= 1e-4   (north-star parity bar)
  f32 mode grads     <= 1e-3   (per parameter tensor, atomics reorder sums)
  bf16 mode forward  <= 5e-2
"""
import os

import numpy as np
import pytest
import torch

from oracle import dv_ref as R

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


def rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def build(mod, dim, mults, lowres):
    u = mod.Unet3D(dim, video_embed_dim=512, channels=3, dim_mults=mults, cond_on_text_encodings=False)
    return u.cast_model_parameters(lowres_cond=lowres, lowres_noise_cond=False, channels=3,
                                   channels_out=3, cond_on_image_embeds=not lowres,
                                   cond_on_text_encodings=False)


def hip_copy_of(oracle_unet, dim, mults, lowres):
    from dalle2_video import dalle2_video as D

    u = build(D, dim, mults, lowres)
    assert list(u.state_dict().keys()) == list(oracle_unet.state_dict().keys())
    u.load_state_dict(oracle_unet.state_dict(), strict=True)
    return u.cuda()


def test_state_dict_and_cast_quirk():
    from dalle2_video import dalle2_video as D

    u = build(D, 64, (1, 2, 4, 8), False)
    assert u.cond_on_video_embeds is False and u.to_video_hiddens is None
    sd = u.state_dict()
    assert len(sd) == 439
    assert sum(p.numel() for p in u.parameters()) == 49_967_171
    assert "mid_attn.fn.fn.to_kv.weight" in sd and "downs.1.2.0.cross_attn.to_q.weight" in sd
    u2 = build(D, 8, (1, 2, 4, 8, 16), True)
    assert len(u2.state_dict()) == 539 and tuple(u2.to_out.weight.shape) == (3, 11, 1, 1, 1)


def test_unet1_forward_matches_golden_f32():
    g = np.load(os.path.join(GOLD, "g2_unet_cfg1.npz"))
    ou = R.deterministic_fill_(build(R, 64, (1, 2, 4, 8), False))
    u = hip_copy_of(ou, 64, (1, 2, 4, 8), False)
    x = torch.from_numpy(g["x"]).cuda()
    t = torch.from_numpy(g["times"]).cuda()
    with torch.no_grad():
        y = u(x, t, video_embed=torch.randn(1, 512, device="cuda"))
    e = rel(y, torch.from_numpy(g["y"]))
    print(f"unet1 cfg1 f32 rel-err vs golden {e:.3e}")
    assert e <= 1e-4


def test_unet2_forward_matches_golden_f32():
    g = np.load(os.path.join(GOLD, "g2_unet_cfg1.npz"))
    ou = R.deterministic_fill_(build(R, 8, (1, 2, 4, 8, 16), True))
    u = hip_copy_of(ou, 8, (1, 2, 4, 8, 16), True)
    with torch.no_grad():
        y = u(torch.from_numpy(g["x2"]).cuda(), torch.from_numpy(g["times2"]).cuda(),
              video_embed=None, lowres_cond_video=torch.from_numpy(g["lowres2"]).cuda())
    e = rel(y, torch.from_numpy(g["y2"]))
    print(f"unet2 f32 rel-err vs golden {e:.3e}")
    assert e <= 1e-4


def test_unet1_forward_bf16():
    g = np.load(os.path.join(GOLD, "g2_unet_cfg1.npz"))
    ou = R.deterministic_fill_(build(R, 64, (1, 2, 4, 8), False))
    u = hip_copy_of(ou, 64, (1, 2, 4, 8), False)
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
        y = u(torch.from_numpy(g["x"]).cuda(), torch.from_numpy(g["times"]).cuda(), video_embed=None)
    e = rel(y, torch.from_numpy(g["y"]))
    print(f"unet1 cfg1 bf16 rel-err vs golden {e:.3e}")
    assert e <= 5e-2


@pytest.mark.parametrize("dtype,ftol,gtol", [(torch.float32, 1e-4, 1e-3), (torch.bfloat16, 5e-2, 1.5e-1)])
def test_p_losses_forward_backward_vs_oracle(dtype, ftol, gtol):
    """Training step arithmetic: q_sample -> unet -> l2 loss -> backward, with
    injected times/noise; every parameter gradient compared to CPU autograd."""
    from dalle2_video import dalle2_video as D

    sched_o = R.NoiseScheduler(beta_schedule="cosine", timesteps=1000, loss_type="l2")
    ou = R.deterministic_fill_(build(R, 16, (1, 2, 4, 8), False))
    u = hip_copy_of(ou, 16, (1, 2, 4, 8), False)
    u.compute_dtype = dtype
    gen = torch.Generator().manual_seed(1234)
    xs = torch.rand(2, 3, 4, 32, 32, generator=gen)
    times = torch.tensor([537, 3])
    noise = torch.randn(xs.shape, generator=gen)
    loss_o = R.p_losses(ou, sched_o, xs, times, noise, video_cond_drop_prob=0.0, text_cond_drop_prob=0.0)
    loss_o.backward()
    dec = D.VideoDecoder(u, frame_sizes=(32,), frame_numbers=(4,), timesteps=1000,
                         learned_variance=False).cuda()
    loss = dec.p_losses(u, xs.cuda(), times.cuda(), video_embed=None,
                        noise_scheduler=dec.noise_schedulers[0], noise=noise.cuda())
    assert abs(loss.item() - loss_o.item()) / loss_o.item() < ftol
    loss.backward()
    worst, worst_name = 0.0, ""
    for (n, po), (n2, p) in zip(ou.named_parameters(), u.named_parameters()):
        assert n == n2
        if po.grad is None:
            assert p.grad is None or p.grad.abs().max() == 0, n
            continue
        e = rel(p.grad, po.grad)
        if e > worst:
            worst, worst_name = e, n
    print(f"{dtype}: loss {loss.item():.6f} vs {loss_o.item():.6f}; worst grad {worst_name} {worst:.3e}")
    assert worst < gtol, worst_name
