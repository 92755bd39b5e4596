"""BASELINE config 3's second training stage: the SR unet (unet2 — dim 8, mults
1/2/4/8/16, low-res conditioned, linear schedule) trained after every unet1
step at 4x3x16x128x128 (reference train_decoder.py:135-138 ->
VideoDecoder.forward(unet_number=2), dalle2_video.py:2188-2299: the
LowresVideoConditioner makes the 64² -> 128² conditioning clip with a 50 %
kornia blur, `:1115-1166`, then p_losses `:1908-2006`).

The blur decision is forced on and off (blur_prob 1 / 0) so both branches of
the conditioner run; times and noise are injected.  Each case compares, on
the same weights, the conditioning clip, the Unet3D forward, the p_losses loss
and every parameter gradient with the CPU oracle (oracle/dv_ref.py:
lowres_condition + the reference wiring).  At this size the SR stage's
small-channel kernels run at full M: 8-channel GroupNorms over 262,144-pixel
clips, the direct small-channel convs at 128², the implicit-GEMM dgrad /
wgrad of the cin = 8..16 convs, the C = 128 mid attention over 1,024 tokens.

Tolerances (norm-wise relative error):
  conditioning clip         <= 1e-6 (blur: f32 separable taps; no blur: bit-exact resize)
  f32  forward <= 1e-4, loss <= 1e-5, per-parameter gradient <= 1e-3
  bf16 forward <= 3e-2, loss <= 5e-3, per-parameter gradient <= 1e-1,
       whole flattened gradient <= 3e-2
  Analytically-zero gradients — the conv biases in front of the 8-channel
  GroupNorms (groups = 8: one channel per group, whose mean subtraction
  cancels a per-channel bias exactly): the oracle's value is f32 roundoff, so
  these are checked in absolute terms, ||g|| <= 1e-6 (f32) / 1e-2 (bf16: the
  channel sum of bf16-rounded dz) times the whole gradient's norm.
The observed values are printed and appended to $DV_PARITY_LOG.
"""
import pytest
import torch

from oracle import dv_ref as R

pytestmark = pytest.mark.gpu

B, T, S, S_LO = 4, 16, 128, 64


def rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def _sr(mod):
    u = mod.Unet3D(8, video_embed_dim=512, channels=3, dim_mults=(1, 2, 4, 8, 16), cond_on_text_encodings=False)
    return u.cast_model_parameters(lowres_cond=True, lowres_noise_cond=False, channels=3, channels_out=3,
                                   cond_on_image_embeds=False, cond_on_text_encodings=False)


_ORACLE = {}


def _oracle(blur):
    """CPU oracle at config 3 for one blur setting (computed once per setting)."""
    if blur in _ORACLE:
        return _ORACLE[blur]
    torch.set_num_threads(min(16, torch.get_num_threads() * 2))
    ou = R.deterministic_fill_(_sr(R))
    sched = R.NoiseScheduler(beta_schedule="linear", timesteps=1000, loss_type="l2")
    g = torch.Generator().manual_seed(303)
    video = torch.rand(B, 3, T, S, S, generator=g)
    noise = torch.randn(video.shape, generator=g)
    times = torch.tensor([0, 999, 421, 77])
    lowres = R.lowres_condition(video, target_frame_size=S, downsample_frame_size=S_LO, blur=blur)
    x_noisy = sched.q_sample(R.normalize_neg_one_to_one(video), times, noise)
    lr_n = R.normalize_neg_one_to_one(lowres)
    pred = ou(x_noisy, times, video_embed=None, lowres_cond_video=lr_n, video_cond_drop_prob=0.0,
              text_cond_drop_prob=0.0)
    loss = ((pred - noise) ** 2).mean()
    loss.backward()
    # conv biases in front of a one-channel-per-group GroupNorm (Block3D.project -> norm)
    zero = {n for n in dict(ou.named_parameters()) if n.endswith("project.bias")
            and ou.get_submodule(n[:-len("project.bias")] + "norm").num_groups
            == ou.get_submodule(n[:-len("project.bias")] + "norm").num_channels}
    _ORACLE[blur] = dict(zero=zero, state=ou.state_dict(), video=video, noise=noise, times=times, lowres=lowres,
                         x_noisy=x_noisy, lr_n=lr_n, pred=pred.detach(), loss=loss.item(),
                         grads={n: p.grad.clone() for n, p in ou.named_parameters() if p.grad is not None})
    return _ORACLE[blur]


@pytest.mark.parametrize("blur,dtype", [(True, torch.float32), (True, torch.bfloat16), (False, torch.float32)])
def test_unet2_config3_train_step_vs_oracle(parity_log, blur, dtype):
    from dalle2_video import dalle2_video as D

    o = _oracle(blur)
    base = D.Unet3D(8, video_embed_dim=512, channels=3, dim_mults=(1, 2))
    dec = D.VideoDecoder((base, _sr(D)), frame_sizes=(S_LO, S), frame_numbers=(T, T), timesteps=1000,
                         learned_variance=False)
    dec.unets[1].load_state_dict(o["state"], strict=True)
    dec = dec.cuda()
    u = dec.unets[1]
    cond = dec.lowres_conds[1]
    cond.blur_prob = 1.0 if blur else 0.0  # force the 50 % decision (random.random() < blur_prob)
    video = o["video"].cuda()
    lowres, _ = cond(video, target_frame_size=S, downsample_frame_size=S_LO)
    e_cond = rel(lowres, o["lowres"])
    amp = torch.autocast("cuda", dtype=torch.bfloat16, enabled=dtype == torch.bfloat16)
    with torch.no_grad(), amp:
        y = u(o["x_noisy"].cuda(), o["times"].cuda(), video_embed=None, lowres_cond_video=o["lr_n"].cuda())
    fwd = rel(y.float(), o["pred"])
    with amp:
        loss = dec.p_losses(u, video, o["times"].cuda(), video_embed=None, noise_scheduler=dec.noise_schedulers[1],
                            lowres_cond_video=lowres, noise=o["noise"].cuda())
    lerr = abs(loss.item() - o["loss"]) / abs(o["loss"])
    loss.backward()
    torch.cuda.synchronize()
    worst, worst_name, num, den = 0.0, "", 0.0, 0.0
    gnorm = sum(g.double().pow(2).sum().item() for g in o["grads"].values()) ** 0.5
    zero_worst, zero_names = 0.0, []
    for n, p in u.named_parameters():
        if n not in o["grads"]:
            assert p.grad is None or p.grad.abs().max() == 0, n
            continue
        gr = o["grads"][n].double()
        gh = p.grad.detach().double().cpu()
        num += (gh - gr).pow(2).sum().item()
        den += gr.pow(2).sum().item()
        if n in o["zero"]:  # analytically zero (see the docstring)
            zero_names.append(n)
            zero_worst = max(zero_worst, gh.norm().item() / gnorm)
            continue
        e = rel(gh, gr)
        if e > worst:
            worst, worst_name = e, n
    gall = (num / den) ** 0.5
    parity_log(config="cfg3 unet2 4x3x16x128x128 lowres 64->128", blur=blur, dtype=str(dtype),
               cond_rel=e_cond, fwd_rel=fwd, loss=loss.item(), loss_oracle=o["loss"], loss_rel=lerr,
               grad_worst_rel=worst, grad_worst_param=worst_name, grad_all_rel=gall,
               zero_grads=len(zero_names), zero_grad_worst_abs=zero_worst)
    assert e_cond <= 1e-6, e_cond
    if dtype == torch.float32:
        ftol, ltol, gtol, atol, ztol = 1e-4, 1e-5, 1e-3, 1e-3, 1e-6
    else:
        ftol, ltol, gtol, atol, ztol = 3e-2, 5e-3, 1e-1, 3e-2, 1e-2
    assert zero_worst <= ztol, zero_worst
    assert fwd <= ftol, fwd
    assert lerr <= ltol, lerr
    assert worst <= gtol, (worst_name, worst)
    assert gall <= atol, gall
