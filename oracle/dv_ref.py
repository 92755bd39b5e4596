"""CPU fp32 ORACLE for the Unet3D denoising path — TEST INFRASTRUCTURE ONLY.

This module is a plain PyTorch-CPU restatement of the reference's hot path
(`/root/reference/dalle2_video/dalle2_video.py:19-952` for Unet3D and its 3-D
blocks, `:1531-1664` / `:1908-2006` for p_sample / p_losses) together with the
third-party leaves it star-imports from `dalle2-pytorch==1.14.2`
(`dalle2_video.py:13`, `requirements.txt:1`), which are absent from this image.

Who may use it: only `tests/`, `__graft_entry__.smoke()` and the
`cpu_baseline` leg of `bench.py`, and only as the CHECKER / the timed CPU
baseline.  The product path (`dalle2-video_amd/dalle2_video`) never imports it.

Pinning status
--------------
* The torch-only reference classes (Block3D, ResnetBlock3D, CrossEmbedLayer3D,
  Downsample3D, PixelShuffleUpsample3D and the Unet3D wiring) are checked
  against the reference's OWN source, AST-extracted and executed by
  `tests/golden/gen_golden.py` (fixtures G1/G2): pinned.
* The dalle2-pytorch 1.14.2 leaves (Attention, CrossAttention, LayerNorm,
  SinusoidalPosEmb, NoiseScheduler, get_optimizer) are restated from that
  package's published algorithm.  The reference has no
  tests and the package is not importable here, so these leaves are
  **parity unpinned**; their call sites are cited below.

The module tree and parameter names are identical to the reference so that
`state_dict()` keys match (439 keys / 49,967,171 params for unet1).
"""
from __future__ import annotations

import math
import zlib
from functools import partial

import torch
import torch.nn as nn
import torch.nn.functional as F
from einops import rearrange, repeat, reduce
from einops.layers.torch import Rearrange

# --------------------------------------------------------------------------
# trivial helpers (dalle2-pytorch; used throughout dalle2_video.py)
# --------------------------------------------------------------------------


def exists(v):
    return v is not None


def default(v, d):
    if exists(v):
        return v
    return d() if callable(d) else d


def identity(t, *args, **kwargs):
    return t


def first(arr, d=None):
    return arr[0] if len(arr) > 0 else d


def maybe(fn):
    def inner(x, *args, **kwargs):
        if not exists(x):
            return x
        return fn(x, *args, **kwargs)

    return inner


def cast_tuple(val, length=None, validate=True):
    if isinstance(val, list):
        val = tuple(val)
    out = val if isinstance(val, tuple) else ((val,) * default(length, 1))
    if exists(length) and validate:
        assert len(out) == length
    return out


def zero_init_(m):
    nn.init.zeros_(m.weight)
    if exists(m.bias):
        nn.init.zeros_(m.bias)


def prob_mask_like(shape, prob, device):
    # p==1 / p==0 consume no RNG (App. B); called at dalle2_video.py:772-779
    if prob == 1:
        return torch.ones(shape, device=device, dtype=torch.bool)
    if prob == 0:
        return torch.zeros(shape, device=device, dtype=torch.bool)
    return torch.zeros(shape, device=device).float().uniform_(0, 1) < prob


def normalize_neg_one_to_one(img):
    return img * 2 - 1


def unnormalize_zero_to_one(t):
    return (t + 1) * 0.5


def resize_image_to(image, target_image_size, clamp_range=None, nearest=False):
    # used per frame via temporal_apply at dalle2_video.py:2257
    if image.shape[-1] == target_image_size:
        return image
    if nearest:
        out = F.interpolate(image, target_image_size, mode="nearest")
    else:
        out = F.interpolate(image, target_image_size, mode="bilinear", align_corners=False)
    if exists(clamp_range):
        out = out.clamp(*clamp_range)
    return out


def temporal_apply(fn, x, *args, **kwargs):
    # dalle2_video.py:81-96 — per-frame application along dim 2
    return torch.stack([fn(x[:, :, i], *args, **kwargs) for i in range(x.shape[2])], dim=2)


# --------------------------------------------------------------------------
# kornia gaussian_blur2d (third-party, imported by the reference for
# LowresVideoConditioner.blur_image, dalle2_video.py:1108).  kornia is absent
# from this image: restated from its published algorithm — parity unpinned.
#   gaussian(ks, sigma): x = arange(ks) - ks // 2 (+0.5 if ks even),
#                        g = exp(-x^2 / (2 sigma^2)), g / sum(g)
#   gaussian_blur2d(img, (ks, ks), (s, s)) with border_type="reflect":
#     filter2d_separable = filter2d(kernel_x) then filter2d(kernel_y), each a
#     depthwise cross-correlation after F.pad(..., mode="reflect").
# --------------------------------------------------------------------------


def gaussian_kernel1d(ks, sigma):
    x = torch.arange(ks, dtype=torch.float32) - ks // 2
    if ks % 2 == 0:
        x = x + 0.5
    g = torch.exp(-x.pow(2.0) / (2 * float(sigma) ** 2))
    return g / g.sum()


def gaussian_blur2d(img, kernel_size, sigma):
    """img (b, c, h, w); kernel_size / sigma are (y, x) pairs."""
    b, c, h, w = img.shape
    ky = gaussian_kernel1d(kernel_size[0], sigma[0])
    kx = gaussian_kernel1d(kernel_size[1], sigma[1])
    x = img.reshape(b * c, 1, h, w)
    px = kx.numel() // 2
    x = F.conv2d(F.pad(x, (px, kx.numel() - 1 - px, 0, 0), mode="reflect"), kx.reshape(1, 1, 1, -1))
    py = ky.numel() // 2
    x = F.conv2d(F.pad(x, (0, 0, py, ky.numel() - 1 - py), mode="reflect"), ky.reshape(1, 1, -1, 1))
    return x.reshape(b, c, h, w)


def lowres_condition(video, *, target_frame_size, downsample_frame_size, blur, blur_sigma=0.6,
                     blur_kernel_size=3, clamp_range=(0.0, 1.0), downsample_first=True):
    """LowresVideoConditioner.forward (dalle2_video.py:1115-1166) with the
    50 % blur decision made by the caller (`blur`) and no Imagen noising:
    per-frame nearest down-resize (clamped), optional per-frame kornia blur,
    per-frame nearest resize to the target (clamped)."""
    if downsample_first and exists(downsample_frame_size):
        video = temporal_apply(resize_image_to, video, downsample_frame_size, clamp_range=clamp_range,
                               nearest=True)
    if blur:
        video = temporal_apply(gaussian_blur2d, video, (blur_kernel_size,) * 2, (blur_sigma,) * 2)
    return temporal_apply(resize_image_to, video, target_frame_size, clamp_range=clamp_range,
                          nearest=True)


# --------------------------------------------------------------------------
# third-party leaves (dalle2-pytorch 1.14.2) — parity unpinned
# --------------------------------------------------------------------------


class LayerNorm(nn.Module):
    """Gain-only LayerNorm; eps 1e-5 in fp32 (fp16_eps otherwise)."""

    def __init__(self, dim, eps=1e-5, fp16_eps=1e-3, stable=False):
        super().__init__()
        self.eps, self.fp16_eps, self.stable = eps, fp16_eps, stable
        self.g = nn.Parameter(torch.ones(dim))

    def forward(self, x):
        eps = self.eps if x.dtype == torch.float32 else self.fp16_eps
        if self.stable:
            x = x / x.amax(dim=-1, keepdim=True).detach()
        var = torch.var(x, dim=-1, unbiased=False, keepdim=True)
        mean = torch.mean(x, dim=-1, keepdim=True)
        return (x - mean) * (var + eps).rsqrt() * self.g


class SinusoidalPosEmb(nn.Module):
    """Called at dalle2_video.py:349 (to_time_hiddens) and :395."""

    def __init__(self, dim):
        super().__init__()
        self.dim = dim

    def forward(self, x):
        half = self.dim // 2
        step = math.log(10000) / (half - 1)
        freqs = torch.exp(torch.arange(half, device=x.device, dtype=x.dtype) * -step)
        arg = x[:, None] * freqs[None, :]
        return torch.cat((arg.sin(), arg.cos()), dim=-1).type(x.dtype)


class Residual(nn.Module):
    def __init__(self, fn):
        super().__init__()
        self.fn = fn

    def forward(self, x, **kwargs):
        return self.fn(x, **kwargs) + x


class RearrangeToSequence(nn.Module):
    def __init__(self, fn):
        super().__init__()
        self.fn = fn

    def forward(self, x):
        x = rearrange(x, "b c ... -> b ... c")
        shape = x.shape
        x = x.reshape(shape[0], -1, shape[-1])
        x = self.fn(x)
        x = x.reshape(shape)
        return rearrange(x, "b ... c -> b c ...")


class Attention(nn.Module):
    """Multi-query self attention with a learned null key/value (one shared
    K/V head).  Constructed at dalle2_video.py:424-432, used as mid_attn
    (:551, :921-922).  q is scaled by `scale` and then q,k by sqrt(scale):
    the logit factor is scale**2 = dim_head**-1 when cosine_sim is False."""

    def __init__(self, dim, *, dim_head=64, heads=8, dropout=0.0, causal=False,
                 rotary_emb=None, cosine_sim=True, cosine_sim_scale=16):
        super().__init__()
        self.scale = cosine_sim_scale if cosine_sim else dim_head ** -0.5
        self.cosine_sim = cosine_sim
        self.heads = heads
        inner = dim_head * heads
        self.causal = causal
        self.norm = LayerNorm(dim)
        self.dropout = nn.Dropout(dropout)
        self.null_kv = nn.Parameter(torch.randn(2, dim_head))
        self.to_q = nn.Linear(dim, inner, bias=False)
        self.to_kv = nn.Linear(dim, dim_head * 2, bias=False)
        self.rotary_emb = rotary_emb
        self.to_out = nn.Sequential(nn.Linear(inner, dim, bias=False), LayerNorm(dim))

    def forward(self, x, mask=None, attn_bias=None):
        b = x.shape[0]
        x = self.norm(x)
        q = self.to_q(x)
        k, v = self.to_kv(x).chunk(2, dim=-1)
        q = rearrange(q, "b n (h d) -> b h n d", h=self.heads) * self.scale
        nk, nv = (repeat(t, "d -> b 1 d", b=b) for t in self.null_kv.unbind(dim=-2))
        k = torch.cat((nk, k), dim=-2)
        v = torch.cat((nv, v), dim=-2)
        if self.cosine_sim:
            q, k = F.normalize(q, dim=-1), F.normalize(k, dim=-1)
        q, k = q * math.sqrt(self.scale), k * math.sqrt(self.scale)
        sim = torch.einsum("bhid,bjd->bhij", q, k)
        attn = sim.softmax(dim=-1, dtype=torch.float32).type(sim.dtype)
        attn = self.dropout(attn)
        out = torch.einsum("bhij,bjd->bhid", attn, v)
        out = rearrange(out, "b h n d -> b n (h d)")
        return self.to_out(out)


class CrossAttention(nn.Module):
    """Per-head cross attention against the conditioning tokens with a
    learned null key/value prepended (3 keys at this config).  Constructed
    at dalle2_video.py:159-162, called at :195-201.  Logit factor
    dim_head**-0.5."""

    def __init__(self, dim, *, context_dim=None, dim_head=64, heads=8, dropout=0.0,
                 norm_context=False, cosine_sim=False, cosine_sim_scale=16):
        super().__init__()
        self.cosine_sim = cosine_sim
        self.scale = cosine_sim_scale if cosine_sim else dim_head ** -0.5
        self.heads = heads
        inner = dim_head * heads
        context_dim = default(context_dim, dim)
        self.norm = LayerNorm(dim)
        self.norm_context = LayerNorm(context_dim) if norm_context else nn.Identity()
        self.dropout = nn.Dropout(dropout)
        self.null_kv = nn.Parameter(torch.randn(2, dim_head))
        self.to_q = nn.Linear(dim, inner, bias=False)
        self.to_kv = nn.Linear(context_dim, inner * 2, bias=False)
        self.to_out = nn.Sequential(nn.Linear(inner, dim, bias=False), LayerNorm(dim))

    def forward(self, x, context, mask=None):
        b = x.shape[0]
        x = self.norm(x)
        context = self.norm_context(context)
        q = self.to_q(x)
        k, v = self.to_kv(context).chunk(2, dim=-1)
        q, k, v = (rearrange(t, "b n (h d) -> b h n d", h=self.heads) for t in (q, k, v))
        nk, nv = (repeat(t, "d -> b h 1 d", h=self.heads, b=b) for t in self.null_kv.unbind(dim=-2))
        k = torch.cat((nk, k), dim=-2)
        v = torch.cat((nv, v), dim=-2)
        if self.cosine_sim:
            q, k = F.normalize(q, dim=-1), F.normalize(k, dim=-1)
        q, k = q * math.sqrt(self.scale), k * math.sqrt(self.scale)
        sim = torch.einsum("bhid,bhjd->bhij", q, k)
        attn = sim.softmax(dim=-1, dtype=torch.float32).type(sim.dtype)
        out = torch.einsum("bhij,bhjd->bhid", attn, v)
        out = rearrange(out, "b h n d -> b n (h d)")
        return self.to_out(out)


class UpsampleCombiner(nn.Module):
    """Only the disabled form is reachable (combine_upsample_fmaps=False)."""

    def __init__(self, dim, *, enabled=False, dim_ins=tuple(), dim_outs=tuple()):
        super().__init__()
        assert not enabled, "UpsampleCombiner(enabled=True) is outside the hot path"
        self.enabled = False
        self.dim_out = dim

    def forward(self, x, fmaps=None):
        return x


def cosine_beta_schedule(timesteps, s=0.008):
    steps = timesteps + 1
    x = torch.linspace(0, timesteps, steps, dtype=torch.float64)
    ac = torch.cos(((x / timesteps) + s) / (1 + s) * torch.pi * 0.5) ** 2
    ac = ac / ac[0]
    betas = 1 - (ac[1:] / ac[:-1])
    return torch.clip(betas, 0, 0.999)


def linear_beta_schedule(timesteps):
    scale = 1000 / timesteps
    return torch.linspace(scale * 0.0001, scale * 0.02, timesteps, dtype=torch.float64)


def extract(a, t, x_shape):
    b = t.shape[0]
    return a.gather(-1, t).reshape(b, *((1,) * (len(x_shape) - 1)))


class NoiseScheduler(nn.Module):
    """Gaussian diffusion tables (fp64 → fp32 buffers).  Constructed at
    dalle2_video.py:1388; q_sample at :1956; loss_fn at :1997;
    predict_start_from_noise / q_posterior at :1591-1607."""

    BUFFERS = (
        "betas", "alphas_cumprod", "alphas_cumprod_prev", "sqrt_alphas_cumprod",
        "sqrt_one_minus_alphas_cumprod", "log_one_minus_alphas_cumprod",
        "sqrt_recip_alphas_cumprod", "sqrt_recipm1_alphas_cumprod", "posterior_variance",
        "posterior_log_variance_clipped", "posterior_mean_coef1", "posterior_mean_coef2",
        "p2_loss_weight",
    )

    def __init__(self, *, beta_schedule, timesteps, loss_type, p2_loss_weight_gamma=0.0,
                 p2_loss_weight_k=1):
        super().__init__()
        if beta_schedule == "cosine":
            betas = cosine_beta_schedule(timesteps)
        elif beta_schedule == "linear":
            betas = linear_beta_schedule(timesteps)
        else:
            raise NotImplementedError(beta_schedule)
        alphas = 1.0 - betas
        ac = torch.cumprod(alphas, dim=0)
        ac_prev = F.pad(ac[:-1], (1, 0), value=1.0)
        self.num_timesteps = int(betas.shape[0])
        assert loss_type == "l2", "only the l2 loss is on the hot path"
        self.loss_type = loss_type
        self.loss_fn = F.mse_loss
        reg = lambda n, v: self.register_buffer(n, v.to(torch.float32))
        reg("betas", betas)
        reg("alphas_cumprod", ac)
        reg("alphas_cumprod_prev", ac_prev)
        reg("sqrt_alphas_cumprod", torch.sqrt(ac))
        reg("sqrt_one_minus_alphas_cumprod", torch.sqrt(1.0 - ac))
        reg("log_one_minus_alphas_cumprod", torch.log(1.0 - ac))
        reg("sqrt_recip_alphas_cumprod", torch.sqrt(1.0 / ac))
        reg("sqrt_recipm1_alphas_cumprod", torch.sqrt(1.0 / ac - 1))
        pv = betas * (1.0 - ac_prev) / (1.0 - ac)
        reg("posterior_variance", pv)
        reg("posterior_log_variance_clipped", torch.log(pv.clamp(min=1e-20)))
        reg("posterior_mean_coef1", betas * torch.sqrt(ac_prev) / (1.0 - ac))
        reg("posterior_mean_coef2", (1.0 - ac_prev) * torch.sqrt(alphas) / (1.0 - ac))
        self.has_p2_loss_reweighting = p2_loss_weight_gamma > 0.0
        reg("p2_loss_weight", (p2_loss_weight_k + ac / (1 - ac)) ** -p2_loss_weight_gamma)

    def q_sample(self, x_start, t, noise):
        return (extract(self.sqrt_alphas_cumprod, t, x_start.shape) * x_start
                + extract(self.sqrt_one_minus_alphas_cumprod, t, x_start.shape) * noise)

    def predict_start_from_noise(self, x_t, t, noise):
        return (extract(self.sqrt_recip_alphas_cumprod, t, x_t.shape) * x_t
                - extract(self.sqrt_recipm1_alphas_cumprod, t, x_t.shape) * noise)

    def q_posterior(self, x_start, x_t, t):
        mean = (extract(self.posterior_mean_coef1, t, x_t.shape) * x_start
                + extract(self.posterior_mean_coef2, t, x_t.shape) * x_t)
        return (mean, extract(self.posterior_variance, t, x_t.shape),
                extract(self.posterior_log_variance_clipped, t, x_t.shape))

    def p2_reweigh_loss(self, loss, times):
        if not self.has_p2_loss_reweighting:
            return loss
        return loss * extract(self.p2_loss_weight, times, loss.shape)


# --------------------------------------------------------------------------
# 3-D blocks (restating dalle2_video.py:19-244)
# --------------------------------------------------------------------------


def Downsample3D(dim, dim_out=None):
    # dalle2_video.py:19-26 — space-to-depth (c s1 s2) then 1x1x1 conv
    return nn.Sequential(
        Rearrange("b c t (h s1) (w s2) -> b (c s1 s2) t h w", s1=2, s2=2),
        nn.Conv3d(dim * 4, default(dim_out, dim), 1),
    )


class PixelShuffleUpsample3D(nn.Module):
    # dalle2_video.py:38-78 — conv 1x1 -> SiLU -> per-frame PixelShuffle(2)
    def __init__(self, dim, dim_out=None):
        super().__init__()
        dim_out = default(dim_out, dim)
        self.conv = nn.Conv3d(dim, dim_out * 4, 1)
        self.act = nn.SiLU()
        self.pixel_shuffle = nn.PixelShuffle(upscale_factor=2)
        o, i, t, h, w = self.conv.weight.shape
        w0 = torch.empty(o // 4, i, t, h, w)
        nn.init.kaiming_uniform_(w0)
        self.conv.weight.data.copy_(repeat(w0, "o ... -> (o 4) ..."))
        nn.init.zeros_(self.conv.bias.data)

    def forward(self, x):
        x = self.act(self.conv(x))
        t = x.shape[2]
        x = rearrange(x, "b c t h w -> (b t) c h w")
        x = self.pixel_shuffle(x)
        return rearrange(x, "(b t) c h w -> b c t h w", t=t)


class Block3D(nn.Module):
    # dalle2_video.py:99-133
    def __init__(self, dim, dim_out, groups=8, weight_standardization=False):
        super().__init__()
        self.project = nn.Conv3d(dim, dim_out, kernel_size=(1, 3, 3), padding=(0, 1, 1))
        self.norm = nn.GroupNorm(groups, dim_out)
        self.act = nn.SiLU()

    def forward(self, x, scale_shift=None):
        x = self.norm(self.project(x))
        if exists(scale_shift):
            scale, shift = scale_shift
            x = x * (scale + 1) + shift
        return self.act(x)


class ResnetBlock3D(nn.Module):
    # dalle2_video.py:136-205
    def __init__(self, dim, dim_out, *, cond_dim=None, time_cond_dim=None, groups=8,
                 weight_standardization=False, cosine_sim_cross_attn=False):
        super().__init__()
        self.time_mlp = (nn.Sequential(nn.SiLU(), nn.Linear(time_cond_dim, dim_out * 2))
                         if exists(time_cond_dim) else None)
        self.cross_attn = (CrossAttention(dim=dim_out, context_dim=cond_dim,
                                          cosine_sim=cosine_sim_cross_attn)
                           if exists(cond_dim) else None)
        self.block1 = Block3D(dim, dim_out, groups=groups)
        self.block2 = Block3D(dim_out, dim_out, groups=groups)
        self.res_conv = nn.Conv3d(dim, dim_out, 1) if dim != dim_out else nn.Identity()

    def forward(self, x, time_emb=None, cond=None):
        scale_shift = None
        if exists(self.time_mlp) and exists(time_emb):
            te = self.time_mlp(time_emb)[:, :, None, None, None]
            scale_shift = te.chunk(2, dim=1)
        h = self.block1(x, scale_shift=scale_shift)
        if exists(self.cross_attn):
            assert exists(cond)
            b, c = h.shape[:2]
            spatial = h.shape[2:]
            seq = h.reshape(b, c, -1).transpose(1, 2)
            seq = self.cross_attn(seq, context=cond) + seq
            h = seq.transpose(1, 2).reshape(b, c, *spatial)
        h = self.block2(h)
        return h + self.res_conv(x)


class CrossEmbedLayer3D(nn.Module):
    # dalle2_video.py:208-244 — sorted kernel sizes, channel split dim/2, dim/4, rest
    def __init__(self, dim_in, kernel_sizes, dim_out=None, stride=2):
        super().__init__()
        assert all((k % 2) == (stride % 2) for k in kernel_sizes)
        dim_out = default(dim_out, dim_in)
        ks = sorted(kernel_sizes)
        scales = [int(dim_out / (2 ** i)) for i in range(1, len(ks))]
        scales = [*scales, dim_out - sum(scales)]
        self.convs = nn.ModuleList([
            nn.Conv3d(dim_in, s, (1, k, k), stride=(1, stride, stride),
                      padding=(0, (k - stride) // 2, (k - stride) // 2))
            for k, s in zip(ks, scales)
        ])

    def forward(self, x):
        return torch.cat([conv(x) for conv in self.convs], dim=1)


# --------------------------------------------------------------------------
# Unet3D (restating dalle2_video.py:247-952 on the paths train_decoder.py uses)
# --------------------------------------------------------------------------


class Unet3D(nn.Module):
    def __init__(self, dim, *, video_embed_dim=None, text_embed_dim=None, cond_dim=None,
                 num_image_tokens=4, num_time_tokens=2, out_dim=None, dim_mults=(1, 2, 4, 8),
                 channels=3, channels_out=None, self_attn=False, attn_dim_head=32,
                 attn_heads=16, lowres_cond=False, lowres_noise_cond=False, self_cond=False,
                 sparse_attn=False, cosine_sim_cross_attn=False, cosine_sim_self_attn=False,
                 attend_at_middle=True, cond_on_text_encodings=False, max_text_len=256,
                 cond_on_video_embeds=False, add_video_embeds_to_time=True, init_dim=None,
                 init_conv_ksize=7, resnet_groups=8, resnet_weight_standardization=False,
                 num_resnet_blocks=2, init_cross_embed=True,
                 init_cross_embed_kernel_sizes=(3, 7, 15), cross_embed_downsample=False,
                 cross_embed_downsample_kernel_sizes=(2, 4), memory_efficient=False,
                 scale_skip_connection=False, pixel_shuffle_upsample=True, final_conv_ksize=1,
                 combine_upsample_fmaps=False, checkpoint_during_training=False, **kwargs):
        super().__init__()
        self._locals = dict(locals())
        del self._locals["self"]
        self._locals.pop("__class__", None)
        # only the configuration train_decoder.py builds is restated
        assert not (self_attn or sparse_attn or memory_efficient or cross_embed_downsample
                    or combine_upsample_fmaps or cond_on_text_encodings or self_cond
                    or cond_on_video_embeds or lowres_noise_cond), "outside the hot path"
        assert init_cross_embed and pixel_shuffle_upsample

        self.lowres_cond = lowres_cond
        self.self_cond = self_cond
        self.channels = channels
        self.channels_out = default(channels_out, channels)
        init_channels = channels * (1 + int(lowres_cond) + int(self_cond))
        init_dim = default(init_dim, dim)
        self.init_conv = CrossEmbedLayer3D(init_channels, dim_out=init_dim,
                                           kernel_sizes=init_cross_embed_kernel_sizes, stride=1)
        dims = [init_dim, *(dim * m for m in dim_mults)]
        in_out = list(zip(dims[:-1], dims[1:]))
        n_stages = len(in_out)
        cond_dim = default(cond_dim, dim)
        tcd = dim * 4
        self.to_time_hiddens = nn.Sequential(SinusoidalPosEmb(dim), nn.Linear(dim, tcd), nn.GELU())
        self.to_time_tokens = nn.Sequential(nn.Linear(tcd, cond_dim * num_time_tokens),
                                            Rearrange("b (r d) -> b r d", r=num_time_tokens))
        self.to_time_cond = nn.Sequential(nn.Linear(tcd, tcd))
        self.video_to_tokens = nn.Identity()
        self.to_video_hiddens = None
        self.norm_cond = nn.LayerNorm(cond_dim)
        self.norm_mid_cond = nn.LayerNorm(cond_dim)
        self.text_to_cond = None
        self.text_embed_dim = None
        self.lowres_noise_cond = lowres_noise_cond
        self.to_lowres_noise_cond = None
        self.cond_on_text_encodings = cond_on_text_encodings
        self.cond_on_video_embeds = cond_on_video_embeds
        self.null_video_embed = nn.Parameter(torch.randn(1, num_image_tokens, cond_dim))
        self.null_video_hiddens = nn.Parameter(torch.randn(1, tcd))
        self.max_text_len = max_text_len
        self.null_text_embed = nn.Parameter(torch.randn(1, max_text_len, cond_dim))
        self.skip_connect_scale = 1.0 if not scale_skip_connection else 2 ** -0.5

        attn_kwargs = dict(heads=attn_heads, dim_head=attn_dim_head, cosine_sim=cosine_sim_self_attn)
        groups = cast_tuple(resnet_groups, n_stages)
        n_blocks = cast_tuple(num_resnet_blocks, n_stages)
        rb = partial(ResnetBlock3D, cosine_sim_cross_attn=cosine_sim_cross_attn)
        self.init_resnet_block = None

        self.downs = nn.ModuleList([])
        self.ups = nn.ModuleList([])
        skip_dims = []
        for ind, ((d_in, d_out), g, nb) in enumerate(zip(in_out, groups, n_blocks)):
            is_first, is_last = ind == 0, ind >= n_stages - 1
            lcd = None if is_first else cond_dim
            skip_dims.append(d_in)
            self.downs.append(nn.ModuleList([
                None,
                rb(d_in, d_in, time_cond_dim=tcd, groups=g),
                nn.ModuleList([rb(d_in, d_in, cond_dim=lcd, time_cond_dim=tcd, groups=g)
                               for _ in range(nb)]),
                nn.Identity(),
                Downsample3D(d_in, dim_out=d_out) if not is_last else nn.Conv3d(d_in, d_out, 1),
            ]))
        mid = dims[-1]
        self.mid_block1 = rb(mid, mid, cond_dim=cond_dim, time_cond_dim=tcd, groups=groups[-1])
        self.mid_attn = RearrangeToSequence(Residual(Attention(mid, **attn_kwargs)))
        self.mid_block2 = rb(mid, mid, cond_dim=cond_dim, time_cond_dim=tcd, groups=groups[-1])
        for ind, ((d_in, d_out), g, nb) in enumerate(zip(reversed(in_out), reversed(groups),
                                                         reversed(n_blocks))):
            is_last = ind >= n_stages - 1
            lcd = cond_dim if not is_last else None
            sd = skip_dims.pop()
            self.ups.append(nn.ModuleList([
                rb(d_out + sd, d_out, cond_dim=lcd, time_cond_dim=tcd, groups=g),
                nn.ModuleList([rb(d_out + sd, d_out, cond_dim=lcd, time_cond_dim=tcd, groups=g)
                               for _ in range(nb)]),
                nn.Identity(),
                PixelShuffleUpsample3D(d_out, d_in) if not is_last else nn.Identity(),
            ]))
        self.upsample_combiner = UpsampleCombiner(dim=dim, enabled=False)
        self.final_resnet_block = rb(self.upsample_combiner.dim_out + dim, dim,
                                     time_cond_dim=tcd, groups=groups[0])
        out_dim_in = dim + (channels if lowres_cond else 0)
        self.to_out = nn.Conv3d(out_dim_in, self.channels_out, kernel_size=(1, final_conv_ksize,
                                final_conv_ksize), padding=(0, final_conv_ksize // 2,
                                                            final_conv_ksize // 2))
        zero_init_(self.to_out)
        self.checkpoint_during_training = checkpoint_during_training

    def cast_model_parameters(self, *, lowres_cond, lowres_noise_cond, channels, channels_out,
                              cond_on_image_embeds, cond_on_text_encodings):
        # dalle2_video.py:652-681: `cond_on_image_embeds` is not a Unet3D
        # argument; it lands in **kwargs, so the rebuilt unet keeps
        # cond_on_video_embeds=False.
        if (lowres_cond == self.lowres_cond and channels == self.channels
                and cond_on_image_embeds == self.cond_on_video_embeds
                and cond_on_text_encodings == self.cond_on_text_encodings
                and lowres_noise_cond == self.lowres_noise_cond
                and channels_out == self.channels_out):
            return self
        kw = dict(self._locals)
        extra = kw.pop("kwargs", {})
        kw.update(extra)
        kw.update(lowres_cond=lowres_cond, channels=channels, channels_out=channels_out,
                  cond_on_image_embeds=cond_on_image_embeds,
                  cond_on_text_encodings=cond_on_text_encodings,
                  lowres_noise_cond=lowres_noise_cond)
        return self.__class__(**kw)

    def forward_with_cond_scale(self, *args, cond_scale=1.0, **kwargs):
        logits = self.forward(*args, **kwargs)
        if cond_scale == 1:
            return logits
        null = self.forward(*args, text_cond_drop_prob=1.0, video_cond_drop_prob=1.0, **kwargs)
        return null + (logits - null) * cond_scale

    def forward(self, x, time, *, video_embed=None, lowres_cond_video=None,
                lowres_noise_level=None, text_encodings=None, video_cond_drop_prob=0.0,
                text_cond_drop_prob=0.0, blur_sigma=None, blur_kernel_size=None,
                disable_checkpoint=False, self_cond=None, return_intermediates=False):
        b, device = x.shape[0], x.device
        assert not (self.lowres_cond and not exists(lowres_cond_video))
        if exists(lowres_cond_video):
            x = torch.cat((x, lowres_cond_video), dim=1)
        inter = {}
        x = self.init_conv(x)
        r = x.clone()
        inter["init_conv"] = x
        th = self.to_time_hiddens(time.type_as(x))
        time_tokens = self.to_time_tokens(th)
        t = self.to_time_cond(th)
        # RNG-consuming masks whose results are dead at this config
        prob_mask_like((b,), 1 - video_cond_drop_prob, device=device)
        prob_mask_like((b,), 1 - text_cond_drop_prob, device=device)
        c = self.norm_cond(time_tokens)
        mid_c = self.norm_mid_cond(time_tokens)
        hiddens = []
        for _, init_block, blocks, attn, post in self.downs:
            x = init_block(x, t, c)
            for blk in blocks:
                x = blk(x, t, c)
                hiddens.append(x.contiguous())
            x = attn(x)
            hiddens.append(x.contiguous())
            x = post(x)
        inter["down"] = x
        x = self.mid_block1(x, t, mid_c)
        x = self.mid_attn(x)
        inter["mid_attn"] = x
        x = self.mid_block2(x, t, mid_c)
        skip = lambda f: torch.cat((f, hiddens.pop() * self.skip_connect_scale), dim=1)
        for init_block, blocks, attn, up in self.ups:
            x = init_block(skip(x), t, c)
            for blk in blocks:
                x = blk(skip(x), t, c)
            x = up(attn(x))
        x = torch.cat((x, r), dim=1)
        x = self.final_resnet_block(x, t)
        if exists(lowres_cond_video):
            x = torch.cat((x, lowres_cond_video), dim=1)
        inter["pre_out"] = x
        out = self.to_out(x)
        return (out, inter) if return_intermediates else out


# --------------------------------------------------------------------------
# VideoDecoder training / sampling arithmetic (dalle2_video.py:1531-2006)
# --------------------------------------------------------------------------


def p_losses(unet, sched, x_start, times, noise, video_embed=None, lowres_cond_video=None,
             video_cond_drop_prob=0.1, text_cond_drop_prob=0.5):
    """dalle2_video.py:1908-2006 with learned_variance=False, predict eps."""
    x_start = normalize_neg_one_to_one(x_start)
    lowres_cond_video = maybe(normalize_neg_one_to_one)(lowres_cond_video)
    x_noisy = sched.q_sample(x_start, times, noise)
    pred = unet(x_noisy, times, video_embed=video_embed, lowres_cond_video=lowres_cond_video,
                video_cond_drop_prob=video_cond_drop_prob, text_cond_drop_prob=text_cond_drop_prob)
    loss = F.mse_loss(pred, noise, reduction="none")
    loss = reduce(loss, "b ... -> b (...)", "mean").mean(dim=-1)
    loss = sched.p2_reweigh_loss(loss, times)
    return loss.mean()


def p_sample(unet, sched, x, times, noise, video_embed=None, lowres_cond_video=None,
             cond_scale=1.0, clip_denoised=True):
    """dalle2_video.py:1551-1664 (static threshold, eps prediction)."""
    pred = unet.forward_with_cond_scale(x, times, video_embed=video_embed,
                                        lowres_cond_video=lowres_cond_video, cond_scale=cond_scale)
    x_start = sched.predict_start_from_noise(x, times, pred)
    if clip_denoised:
        x_start = x_start.clamp(-1.0, 1.0)
    mean, _, logvar = sched.q_posterior(x_start, x, times)
    nonzero = (1 - (times == 0).float()).reshape(x.shape[0], *((1,) * (x.ndim - 1)))
    return mean + nonzero * (0.5 * logvar).exp() * noise, x_start


# --------------------------------------------------------------------------
# trainer step (dalle2_video/trainer.py:247-274 + dalle2-pytorch get_optimizer)
# --------------------------------------------------------------------------


def get_optimizer(params, lr=1e-4, wd=1e-2, betas=(0.9, 0.99), eps=1e-8, group_wd_params=True):
    params = list(params)
    if wd == 0:
        return torch.optim.Adam(params, lr=lr, betas=betas, eps=eps)
    if group_wd_params:
        wd_p = [p for p in params if p.ndim >= 2]
        no_wd = [p for p in params if p.ndim < 2]
        params = [{"params": wd_p}, {"params": no_wd, "weight_decay": 0}]
    return torch.optim.AdamW(params, lr=lr, weight_decay=wd, betas=betas, eps=eps)


def train_step(unet, sched, opt, x_start, times, noise, max_grad_norm=0.5, **kw):
    loss = p_losses(unet, sched, x_start, times, noise, **kw)
    loss.backward()
    torch.nn.utils.clip_grad_norm_([p for p in unet.parameters()], max_grad_norm)
    opt.step()
    opt.zero_grad()
    return loss.item()


# --------------------------------------------------------------------------
# deterministic parameter fill — shared rule with the product
# --------------------------------------------------------------------------


def deterministic_fill_(module: nn.Module):
    """Fill every parameter from a generator seeded by crc32(name):
    ndim>=2 -> randn/sqrt(fan_in); 1-D gains -> 1+0.1*randn; biases ->
    0.01*randn.  `to_out` is therefore non-zero."""
    with torch.no_grad():
        for name, p in module.named_parameters():
            g = torch.Generator().manual_seed(zlib.crc32(name.encode()))
            r = torch.randn(p.shape, generator=g, dtype=torch.float64)
            if name.endswith("bias"):
                v = 0.01 * r
            elif p.ndim >= 2:
                fan_in = p[0].numel() if p.ndim > 1 else 1
                v = r / math.sqrt(max(fan_in, 1))
            else:
                v = 1.0 + 0.1 * r
            p.copy_(v.to(p.dtype))
    return module
