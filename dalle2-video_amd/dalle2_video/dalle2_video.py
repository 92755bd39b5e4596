"""MI355X-native Unet3D / VideoDecoder — drop-in for
`dalle2_video/dalle2_video.py` of SeanNobel/DALLE2-video on the Unet3D hot path.

Same constructor / forward / sample signatures and the same module tree, so
`state_dict()` keys match the reference (439 keys for unet1).  Parameters live
in the reference layout (f32 nn.Conv3d / nn.Linear / nn.GroupNorm holders);
every forward runs through the HIP kernels of libdv_hip (`ops`) on
channels-last (batch*frames, H, W, C) activations; the NCTHW layout exists
only at the module boundary.  There is no CPU or torch-compute fallback.

Precision: f32 (the reference's, exact f32 MFMA) unless the call runs under
`torch.autocast("cuda", dtype=torch.bfloat16)` (or `unet.compute_dtype` is
set), in which case activations are bf16 with f32 accumulation/statistics.
"""
from __future__ import annotations

import copy
import math
import random
from contextlib import contextmanager, nullcontext
from functools import partial
from typing import Optional, Tuple, Union

import torch
import torch.nn as nn
import torch.nn.functional as F
from einops.layers.torch import Rearrange

from . import ops
from ._lib import ACT_SILU, DVError

# ---------------------------------------------------------------------------
# helpers (dalle2-pytorch semantics)
# ---------------------------------------------------------------------------


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
        return x if not exists(x) else fn(x, *args, **kwargs)
    return inner


def cast_tuple(val, length=None, validate=True):
    if isinstance(val, list):
        val = tuple(val)
    out = val if isinstance(val, tuple) else ((val,) * default(length, 1))
    if exists(length) and validate:
        assert len(out) == length
    return out


def pad_tuple_to_length(t, length, fillvalue=None):
    rem = length - len(t)
    return t if rem <= 0 else (*t, *((fillvalue,) * rem))


def zero_init_(m):
    nn.init.zeros_(m.weight)
    if exists(m.bias):
        nn.init.zeros_(m.bias)


def normalize_neg_one_to_one(img):
    return img * 2 - 1


def unnormalize_zero_to_one(t):
    return (t + 1) * 0.5


def prob_mask_like(shape, prob, device):
    if prob == 1:
        return torch.ones(shape, device=device, dtype=torch.bool)
    if prob == 0:
        return torch.zeros(shape, device=device, dtype=torch.bool)
    # (the reference fills zeros first; uniform_ overwrites every element, so
    # the draw -- and the generator state after it -- is the same without the fill)
    return torch.empty(shape, device=device).uniform_(0, 1) < prob


def _compute_dtype(module, ref: torch.Tensor):
    forced = getattr(module, "compute_dtype", None)
    if forced is not None:
        return forced
    if ref.is_cuda and torch.is_autocast_enabled("cuda"):
        adt = torch.get_autocast_dtype("cuda")
        if adt in (torch.bfloat16, torch.float16):
            return torch.bfloat16
    return torch.float32


def _ln_eps(dtype):
    # dalle2-pytorch LayerNorm: eps=1e-5 in f32, fp16_eps=1e-3 otherwise
    return 1e-5 if dtype == torch.float32 else 1e-3


def _ss_flat(scale_shift, dim_out):
    if scale_shift is None:
        return None
    scale, shift = scale_shift
    b = scale.shape[0]
    return torch.cat((scale.reshape(b, dim_out), shift.reshape(b, dim_out)), dim=1).float()


# ---------------------------------------------------------------------------
# dalle2-pytorch leaves used by the hot path (parameter holders + HIP forward)
# ---------------------------------------------------------------------------


class LayerNorm(nn.Module):
    """Gain-only LayerNorm (dalle2-pytorch)."""

    def __init__(self, dim, eps=1e-5, fp16_eps=1e-3, stable=False):
        super().__init__()
        assert not stable
        self.eps, self.fp16_eps, self.stable = eps, fp16_eps, stable
        self.g = nn.Parameter(torch.ones(dim))

    def forward(self, x):
        eps = self.eps if x.dtype == torch.float32 else self.fp16_eps
        shp = x.shape
        return ops.layer_norm(x.reshape(-1, shp[-1]), self.g, eps=eps).reshape(shp)


class SinusoidalPosEmb(nn.Module):
    def __init__(self, dim):
        super().__init__()
        self.dim = dim

    def forward(self, x):
        return ops.sinusoidal(x, self.dim)


class Residual(nn.Module):
    def __init__(self, fn):
        super().__init__()
        self.fn = fn

    def forward_cl(self, x, nb):
        return self.fn.forward_cl(x, nb, residual=True)


class RearrangeToSequence(nn.Module):
    def __init__(self, fn):
        super().__init__()
        self.fn = fn

    def forward_cl(self, x, nb):
        # channels-last frames of one batch element are already its (t h w) token sequence
        return self.fn.forward_cl(x, nb)

    def forward(self, x):
        b, c, t = x.shape[:3]
        dt = _compute_dtype(self, x)
        y = self.forward_cl(ops.to_cl(x, dt), b)
        return ops.from_cl(y, b, c, t)


class Attention(nn.Module):
    """Multi-query self attention (dalle2-pytorch Attention), mid block only.
    Parameters: norm.g, null_kv (2, dim_head), to_q, to_kv (one K/V head),
    to_out = [Linear, LayerNorm]."""

    def __init__(self, dim, *, dim_head=64, heads=8, dropout=0.0, causal=False, rotary_emb=None,
                 cosine_sim=True, cosine_sim_scale=16):
        super().__init__()
        assert not causal and rotary_emb is None and not cosine_sim, "outside the hot path"
        self.scale = dim_head ** -0.5
        self.cosine_sim = cosine_sim
        self.heads = heads
        self.dim_head = dim_head
        inner = dim_head * heads
        self.causal = causal
        self.norm = LayerNorm(dim)
        self.dropout = nn.Dropout(dropout)
        self.null_kv = nn.Parameter(torch.randn(2, dim_head))
        self.to_q = nn.Linear(dim, inner, bias=False)
        self.to_kv = nn.Linear(dim, dim_head * 2, bias=False)
        self.rotary_emb = rotary_emb
        self.to_out = nn.Sequential(nn.Linear(inner, dim, bias=False), LayerNorm(dim))

    def forward_cl(self, x, nb, residual=False):
        nf, h, w, c = x.shape
        eps = _ln_eps(x.dtype)
        tokens = x.reshape(-1, c)
        xn = ops.layer_norm(tokens, self.norm.g, eps=eps).reshape(nf, h, w, c)
        q = ops.conv(xn, self.to_q.weight)
        kv = ops.conv(xn, self.to_kv.weight)
        n = (nf // nb) * h * w
        # logit factor: q*scale, then q,k*sqrt(scale)  ->  scale**2 = dim_head**-1
        o = ops.mqa(q.reshape(-1, q.shape[-1]), kv.reshape(-1, kv.shape[-1]), self.null_kv, nb, n,
                    self.heads, self.scale * self.scale)
        o = ops.conv(o.reshape(nf, h, w, -1), self.to_out[0].weight)
        y = ops.layer_norm(o.reshape(-1, c), self.to_out[1].g, res=tokens if residual else None,
                           eps=eps)
        return y.reshape(nf, h, w, c)


class CrossAttention(nn.Module):
    """dalle2-pytorch CrossAttention (8 heads x 64, null k/v), folded on MI355X."""

    def __init__(self, dim, *, context_dim=None, dim_head=64, heads=8, dropout=0.0,
                 norm_context=False, cosine_sim=False, cosine_sim_scale=16):
        super().__init__()
        assert heads == 8 and dim_head == 64 and not norm_context and not cosine_sim, \
            "outside the hot path"
        self.cosine_sim = cosine_sim
        self.scale = dim_head ** -0.5
        self.heads = heads
        inner = dim_head * heads
        context_dim = default(context_dim, dim)
        self.norm = LayerNorm(dim)
        self.norm_context = nn.Identity()
        self.dropout = nn.Dropout(dropout)
        self.null_kv = nn.Parameter(torch.randn(2, dim_head))
        self.to_q = nn.Linear(dim, inner, bias=False)
        self.to_kv = nn.Linear(context_dim, inner * 2, bias=False)
        self.to_out = nn.Sequential(nn.Linear(inner, dim, bias=False), LayerNorm(dim))

    def forward_cl(self, x, context, nb, kv=None, fold=None):
        """Returns cross_attn(x, context) + x (the residual of ResnetBlock3D:197);
        kv / fold: this block's to_kv(context) and folded operands when the Unet
        batched them (one launch for every block)."""
        return ops.cross_attention(x, context, self.norm.g, self.null_kv, self.to_q.weight,
                                   self.to_kv.weight, self.to_out[0].weight, self.to_out[1].g, nb,
                                   _ln_eps(x.dtype), kv=kv, fold=fold)

    def make_fold(self, kv, nb, dtype):
        """Unrun XattnFold of this block for ops.xattn_fold_batched."""
        return ops.XattnFold(dtype, kv, self.norm.g, self.null_kv, self.to_q.weight,
                             self.to_out[0].weight, nb, self.to_out[0].weight.shape[0])


class UpsampleCombiner(nn.Module):
    def __init__(self, dim, *, enabled=False, dim_ins=tuple(), dim_outs=tuple()):
        super().__init__()
        assert not enabled, "UpsampleCombiner(enabled=True) is outside the hot path"
        self.enabled = False
        self.dim_out = dim

    def forward(self, x, fmaps=None):
        return x


# ---------------------------------------------------------------------------
# diffusion schedule (dalle2-pytorch NoiseScheduler; buffers identical)
# ---------------------------------------------------------------------------


def cosine_beta_schedule(timesteps, s=0.008):
    steps = timesteps + 1
    x = torch.linspace(0, timesteps, steps, dtype=torch.float64)
    ac = torch.cos(((x / timesteps) + s) / (1 + s) * torch.pi * 0.5) ** 2
    ac = ac / ac[0]
    return torch.clip(1 - (ac[1:] / ac[:-1]), 0, 0.999)


def linear_beta_schedule(timesteps):
    scale = 1000 / timesteps
    return torch.linspace(scale * 0.0001, scale * 0.02, timesteps, dtype=torch.float64)


def extract(a, t, x_shape):
    b = t.shape[0]
    return a.gather(-1, t).reshape(b, *((1,) * (len(x_shape) - 1)))


class NoiseScheduler(nn.Module):
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
        if loss_type != "l2":
            raise NotImplementedError("only the l2 loss is on the MI355X hot path")
        self.loss_type = loss_type
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

    def sample_random_times(self, batch):
        return torch.randint(0, self.num_timesteps, (batch,), device=self.betas.device,
                             dtype=torch.long)

    def q_sample(self, x_start, t, noise=None):
        noise = default(noise, lambda: torch.randn_like(x_start))
        y = ops.q_sample_cl(x_start, noise, t, self.sqrt_alphas_cumprod,
                            self.sqrt_one_minus_alphas_cumprod, torch.float32, normalize=False)
        return ops.from_cl(y, x_start.shape[0], x_start.shape[1], x_start.shape[2])


class NullVQGanVAE(nn.Module):
    def __init__(self, *, channels):
        super().__init__()
        self.encoded_dim = channels
        self.layers = 0

    def get_encoded_fmap_size(self, size):
        return size

    def copy_for_eval(self):
        return self

    def encode(self, x):
        return x

    def decode(self, x):
        return x


# ---------------------------------------------------------------------------
# 3-D blocks (dalle2_video.py:19-244)
# ---------------------------------------------------------------------------


class _Downsample3D(nn.Sequential):
    def forward_cl(self, x, skip_in=None):
        return ops.conv(ops.space_to_depth(x, skip_in=skip_in), self[1].weight, self[1].bias)

    def forward(self, x):
        b, c, t = x.shape[:3]
        y = self.forward_cl(ops.to_cl(x, _compute_dtype(self, x)))
        return ops.from_cl(y, b, y.shape[-1], t)


def Downsample3D(dim, dim_out=None):
    """space-to-depth (c s1 s2) then a 1x1x1 conv — dalle2_video.py:19-26."""
    return _Downsample3D(Rearrange("b c t (h s1) (w s2) -> b (c s1 s2) t h w", s1=2, s2=2),
                         nn.Conv3d(dim * 4, default(dim_out, dim), 1))


class _Conv1x1(nn.Conv3d):
    def forward_cl(self, x, skip_in=None):
        return ops.conv(x, self.weight, self.bias, skip_in=skip_in)


class PixelShuffleUpsample3D(nn.Module):
    """conv 1x1 -> SiLU -> per-frame PixelShuffle(2), ICNR init (dalle2_video.py:38-78)."""

    def __init__(self, dim, dim_out=None):
        super().__init__()
        dim_out = default(dim_out, dim)
        self.conv = nn.Conv3d(dim, dim_out * 4, 1)
        self.act = nn.SiLU()
        self.pixel_shuffle = nn.PixelShuffle(upscale_factor=2)
        o, i, t, h, w = self.conv.weight.shape
        w0 = torch.empty(o // 4, i, t, h, w)
        nn.init.kaiming_uniform_(w0)
        self.conv.weight.data.copy_(w0.repeat_interleave(4, dim=0))
        nn.init.zeros_(self.conv.bias.data)

    def forward_cl(self, x):
        return ops.silu_pixel_shuffle(ops.conv(x, self.conv.weight, self.conv.bias))

    def forward(self, x):
        b, c, t = x.shape[:3]
        y = self.forward_cl(ops.to_cl(x, _compute_dtype(self, x)))
        return ops.from_cl(y, b, y.shape[-1], t)


class Block3D(nn.Module):
    """conv(1,3,3) -> GroupNorm -> x*(scale+1)+shift -> SiLU (dalle2_video.py:99-133)."""

    def __init__(self, dim, dim_out, groups=8, weight_standardization=False):
        super().__init__()
        assert not weight_standardization
        self.project = nn.Conv3d(dim, dim_out, kernel_size=(1, 3, 3), padding=(0, 1, 1))
        self.norm = nn.GroupNorm(groups, dim_out)
        self.act = nn.SiLU()

    def forward_cl(self, x0, nb, x1=None, scale_shift=None, res=None, sink=None, res_sink=None,
                   skip_in=None, skip_out=None, defer_norm=False):
        # the conv's epilogue accumulates the GroupNorm statistics of z, so the
        # norm is a single apply pass over z -- or none (defer_norm: the output
        # feeds only the next Block3D's conv, which applies the norm while it
        # stages z, ops.group_norm_act(defer=True))
        nf, h, w = x0.shape[:3]
        st = ops.gn_stats(nb, self.project.out_channels, (nf // nb) * h * w, x0.device)
        z = ops.conv(x0, self.project.weight, self.project.bias, x1=x1, sink=sink, gn=st,
                     skip_in=skip_in, skip_out=skip_out)
        return ops.group_norm_act(z, self.norm.weight, self.norm.bias, nb, self.norm.num_groups,
                                  self.norm.eps, scale_shift=scale_shift, res=res, act=ACT_SILU,
                                  stats=st, res_sink=res_sink, defer=defer_norm)

    def forward(self, x, scale_shift=None):
        b, c, t = x.shape[:3]
        dt = _compute_dtype(self, x)
        y = self.forward_cl(ops.to_cl(x, dt), b,
                            scale_shift=_ss_flat(scale_shift, self.project.out_channels))
        return ops.from_cl(y, b, self.project.out_channels, t)


class ResnetBlock3D(nn.Module):
    """time-MLP scale/shift -> block1 -> [cross-attn + residual] -> block2 + res_conv(x)
    (dalle2_video.py:136-205)."""

    def __init__(self, dim, dim_out, *, cond_dim=None, time_cond_dim=None, groups=8,
                 weight_standardization=False, cosine_sim_cross_attn=False):
        super().__init__()
        self.time_mlp = (nn.Sequential(nn.SiLU(), nn.Linear(time_cond_dim, dim_out * 2))
                         if exists(time_cond_dim) else None)
        self.cross_attn = (CrossAttention(dim=dim_out, context_dim=cond_dim,
                                          cosine_sim=cosine_sim_cross_attn)
                           if exists(cond_dim) else None)
        self.block1 = Block3D(dim, dim_out, groups=groups, weight_standardization=weight_standardization)
        self.block2 = Block3D(dim_out, dim_out, groups=groups, weight_standardization=weight_standardization)
        self.res_conv = nn.Conv3d(dim, dim_out, 1) if dim != dim_out else nn.Identity()

    def forward_cl(self, x0, time_emb, cond, nb, x1=None, ss=None, kv=None, fold=None,
                   skip_in=None, skip_out=None):
        """ss / kv: this block's time_mlp(time_emb) / to_kv(cond) when the Unet
        computed them for all blocks in one grouped launch (ops.linear_group).
        skip_in: the ops.SkipGrad of x0 when x0 is a unet skip (block1's conv
        adds its parked up-path gradients); skip_out: that of x1 when x1 is one
        (the up-path dgrad parks dX1 there)."""
        if ss is None and exists(self.time_mlp) and exists(time_emb):
            ss = ops.linear_group(time_emb, [self.time_mlp[1].weight], [self.time_mlp[1].bias],
                                  act_in=ACT_SILU)[0]
        # block1's conv and res_conv read the same input: one shared dX buffer
        # (ops.GradSink) instead of an autograd add of two input gradients
        # res_conv runs first so that its (cheap, 1x1) input-gradient is the
        # one that accumulates into block1's 3x3 dgrad output, not the reverse:
        # autograd runs the later-recorded node's backward first
        identity = isinstance(self.res_conv, nn.Identity)
        if identity:
            if x1 is not None:
                raise DVError("identity residual with a split input")
            # block2's residual add and block1's conv both read x0: the
            # residual gradient (block2's dy) becomes block1's dgrad
            # accumulator (no autograd add of two full tensors)
            sink, res = ops.GradSink(), x0
        else:
            sink = ops.GradSink()
            res = ops.conv(x0, self.res_conv.weight, self.res_conv.bias, x1=x1, sink=sink,
                           skip_out=skip_out)
        # block1's conv is x0's gradient owner either way: the second reader of
        # the shared buffer (identity) or the first (res_conv), so it takes skip_in
        # block1's output feeds block2's conv alone when there is no cross-attention
        h = self.block1.forward_cl(x0, nb, x1=x1, scale_shift=ss, sink=sink, skip_in=skip_in,
                                   skip_out=skip_out, defer_norm=self.cross_attn is None and ops.GN_FOLD)
        if exists(self.cross_attn):
            assert exists(cond)
            h = self.cross_attn.forward_cl(h, cond, nb, kv=kv, fold=fold)
        return self.block2.forward_cl(h, nb, res=res, res_sink=sink if identity else None)

    def forward(self, x, time_emb=None, cond=None):
        b, c, t = x.shape[:3]
        dt = _compute_dtype(self, x)
        te = time_emb.float() if exists(time_emb) else None
        cf = cond.float() if exists(cond) else None
        y = self.forward_cl(ops.to_cl(x, dt), te, cf, b)
        return ops.from_cl(y, b, y.shape[-1], t)


class CrossEmbedLayer3D(nn.Module):
    """Convs (1,k,k) for sorted k with channel split dim/2, dim/4, rest (dalle2_video.py:208-244)."""

    def __init__(self, dim_in, kernel_sizes, dim_out=None, stride=2):
        super().__init__()
        assert all((k % 2) == (stride % 2) for k in kernel_sizes)
        assert stride == 1, "only stride 1 is on the hot path"
        dim_out = default(dim_out, dim_in)
        ks = sorted(kernel_sizes)
        scales = [int(dim_out / (2 ** i)) for i in range(1, len(ks))]
        scales = [*scales, dim_out - sum(scales)]
        self.convs = nn.ModuleList([
            nn.Conv3d(dim_in, s, (1, k, k), stride=(1, stride, stride),
                      padding=(0, (k - stride) // 2, (k - stride) // 2))
            for k, s in zip(ks, scales)
        ])

    def forward_cl(self, x):
        weights = [c.weight for c in self.convs]
        if ops.cross_embed_ok(x, weights):
            # direct kernels: each 16-channel tile runs only its own window
            # (dv_cross_embed_fwd / _wgrad)
            return ops.cross_embed(x, weights, [c.bias for c in self.convs])
        # f32 / other shapes: one conv with the smaller kernels
        # zero-embedded at the centre of the largest window (same 'same'
        # padding arithmetic) writes the channel concatenation directly. The
        # (cout <= 64) MMA tile is then full, and the input is gathered once
        # instead of once per kernel size.
        kmax = max(c.weight.shape[-1] for c in self.convs)
        w = torch.cat([F.pad(c.weight, [(kmax - c.weight.shape[-1]) // 2] * 4) for c in self.convs], dim=0)
        b = torch.cat([c.bias for c in self.convs], dim=0)
        # algorithmic FLOPs are those of the three unpadded convs
        cin = self.convs[0].weight.shape[1]
        algo = sum(c.weight.shape[0] * cin * c.weight.shape[-1] ** 2 for c in self.convs)
        executed = w.shape[0] * x.shape[-1] * kmax * kmax
        return ops.conv(x, w, b, cache=False, algo_scale=algo / executed)

    def forward(self, x):
        b, c, t = x.shape[:3]
        y = self.forward_cl(ops.to_cl(x, _compute_dtype(self, x)))
        return ops.from_cl(y, b, y.shape[-1], t)


def temporal_apply(fn, x, *args, **kwargs):
    return torch.stack([fn(x[:, :, i], *args, **kwargs) for i in range(x.shape[2])], dim=2)


# ---------------------------------------------------------------------------
# Unet3D (dalle2_video.py:247-952)
# ---------------------------------------------------------------------------


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
        unsupported = dict(self_attn=self_attn, sparse_attn=sparse_attn,
                           memory_efficient=memory_efficient,
                           cross_embed_downsample=cross_embed_downsample,
                           combine_upsample_fmaps=combine_upsample_fmaps,
                           cond_on_text_encodings=cond_on_text_encodings, self_cond=self_cond,
                           cond_on_video_embeds=cond_on_video_embeds,
                           lowres_noise_cond=lowres_noise_cond,
                           scale_skip_connection=scale_skip_connection,
                           cosine_sim_self_attn=cosine_sim_self_attn,
                           cosine_sim_cross_attn=cosine_sim_cross_attn)
        bad = [k for k, v in unsupported.items() if v]
        if bad or not init_cross_embed or not pixel_shuffle_upsample or final_conv_ksize != 1:
            raise NotImplementedError(f"Unet3D options outside the MI355X hot path: {bad}")
        self.compute_dtype = None  # None: f32 unless under torch.autocast(bf16)

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
        self.dim = dim
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
        self.skip_connect_scale = 1.0
        self.num_time_tokens = num_time_tokens
        self.cond_dim = cond_dim

        attn_kwargs = dict(heads=attn_heads, dim_head=attn_dim_head, cosine_sim=cosine_sim_self_attn)
        groups = cast_tuple(resnet_groups, n_stages)
        n_blocks = cast_tuple(num_resnet_blocks, n_stages)
        rb = partial(ResnetBlock3D, cosine_sim_cross_attn=cosine_sim_cross_attn,
                     weight_standardization=resnet_weight_standardization)
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
                Downsample3D(d_in, dim_out=d_out) if not is_last else _Conv1x1(d_in, d_out, 1),
            ]))
        mid = dims[-1]
        self.mid_block1 = rb(mid, mid, cond_dim=cond_dim, time_cond_dim=tcd, groups=groups[-1])
        self.mid_attn = RearrangeToSequence(Residual(Attention(mid, **attn_kwargs))) \
            if attend_at_middle else None
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
        self.to_out = nn.Conv3d(out_dim_in, self.channels_out, kernel_size=(1, 1, 1))
        zero_init_(self.to_out)
        self.checkpoint_during_training = checkpoint_during_training
        # sampling precision switch (not a reference argument): True runs the
        # eligible 3x3 convs of a no-grad forward in MX-fp8 (BASELINE config 5,
        # ops.mx8_convs); training always stays bf16 / f32.  DV_FP8=1 sets it.
        import os
        self.fp8 = os.environ.get("DV_FP8", "0") == "1"
        # also the mid attention's PV in MX-fp8 (ops.mx8_convs(attention=True));
        # off: measured slower than the bf16 kernel on MI355X
        self.fp8_attention = False

    # dalle2_video.py:652-681 — `cond_on_image_embeds` is swallowed by **kwargs
    # so the rebuilt unet keeps cond_on_video_embeds=False.
    def cast_model_parameters(self, *, lowres_cond, lowres_noise_cond, channels, channels_out,
                              cond_on_image_embeds, cond_on_text_encodings):
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

    # ---- conditioning ----------------------------------------------------
    def _conditioning(self, time, batch, device, video_cond_drop_prob, text_cond_drop_prob):
        th = ops.linear_small(ops.sinusoidal(time, self.dim), self.to_time_hiddens[1].weight,
                              self.to_time_hiddens[1].bias, act_out=ops.ACT_OUT_GELU)
        tt = ops.linear_small(th, self.to_time_tokens[0].weight, self.to_time_tokens[0].bias)
        t = ops.linear_small(th, self.to_time_cond[0].weight, self.to_time_cond[0].bias)
        # dalle2_video.py:772-779: two keep-masks drawn from the device RNG; at this
        # configuration their values are dead (no video/text tokens), but the draws stay
        prob_mask_like((batch,), 1 - video_cond_drop_prob, device=device)
        prob_mask_like((batch,), 1 - text_cond_drop_prob, device=device)
        tt = tt.reshape(-1, self.cond_dim)
        c = ops.layer_norm(tt, self.norm_cond.weight, self.norm_cond.bias,
                           eps=self.norm_cond.eps).reshape(batch, self.num_time_tokens, self.cond_dim)
        mid_c = ops.layer_norm(tt, self.norm_mid_cond.weight, self.norm_mid_cond.bias,
                               eps=self.norm_mid_cond.eps).reshape(batch, self.num_time_tokens,
                                                                   self.cond_dim)
        return t, c, mid_c

    def _resnet_blocks(self):
        """(block, uses mid_c) for every ResnetBlock3D in forward order."""
        out = []
        for _, init_block, blocks, _, _ in self.downs:
            out += [(init_block, False)] + [(b, False) for b in blocks]
        out += [(self.mid_block1, True), (self.mid_block2, True)]
        for init_block, blocks, _, _ in self.ups:
            out += [(init_block, False)] + [(b, False) for b in blocks]
        out.append((self.final_resnet_block, False))
        return out

    def _grouped_projections(self, t, c, mid_c, nb, dtype):
        """Every ResnetBlock3D's time_mlp(t) in ONE launch, and every cross-attention
        to_kv(c) / to_kv(mid_c) in one launch per context (ops.linear_group):
        {id(block): (scale_shift, kv)}.  Same arithmetic as the per-block
        Linear layers (dalle2_video.py:182-185, 195-201)."""
        blks = self._resnet_blocks()
        timed = [b for b, _ in blks if exists(b.time_mlp)]
        ss = ops.linear_group(t, [b.time_mlp[1].weight for b in timed],
                              [b.time_mlp[1].bias for b in timed], act_in=ACT_SILU)
        pre = {id(b): [s, None] for b, s in zip(timed, ss)}
        for use_mid, ctx in ((False, c), (True, mid_c)):
            xa = [b for b, m in blks if m == use_mid and exists(b.cross_attn)]
            if not xa:
                continue
            kvs = ops.linear_group(ctx.reshape(-1, ctx.shape[-1]),
                                   [b.cross_attn.to_kv.weight for b in xa], [None] * len(xa))
            for b, kv in zip(xa, kvs):
                pre.setdefault(id(b), [None, None])[1] = kv
        # every block's cross-attention fold (weights x context only) in one go
        folds = {}
        for b, _ in blks:
            if exists(b.cross_attn) and id(b) in pre and pre[id(b)][1] is not None:
                folds[id(b)] = b.cross_attn.make_fold(pre[id(b)][1], nb, dtype)
        ops.xattn_fold_batched(folds.values())
        return {k: (v[0], v[1], folds.get(k)) for k, v in pre.items()}

    def forward_cl(self, x, time, *, batch, lowres_cl=None, video_cond_drop_prob=0.0,
                   text_cond_drop_prob=0.0):
        """Core denoiser on channels-last frames x (batch*T, H, W, C8); returns
        channels-last (batch*T, H, W, channels_out)."""
        if getattr(self, "fp8", False) and not torch.is_grad_enabled():
            with ops.mx8_convs(attention=getattr(self, "fp8_attention", False)):
                return self._forward_cl(x, time, batch=batch, lowres_cl=lowres_cl,
                                        video_cond_drop_prob=video_cond_drop_prob,
                                        text_cond_drop_prob=text_cond_drop_prob)
        return self._forward_cl(x, time, batch=batch, lowres_cl=lowres_cl,
                                video_cond_drop_prob=video_cond_drop_prob,
                                text_cond_drop_prob=text_cond_drop_prob)

    def _forward_cl(self, x, time, *, batch, lowres_cl=None, video_cond_drop_prob=0.0,
                    text_cond_drop_prob=0.0):
        x = self.init_conv.forward_cl(x)
        r = x
        t, c, mid_c = self._conditioning(time, batch, x.device, video_cond_drop_prob,
                                         text_cond_drop_prob)
        pre = self._grouped_projections(t, c, mid_c, batch, x.dtype)

        mark = ops.backward_mark  # backward progress marks (trainer's overlapped all-reduce)

        def run(blk, x, cond, x1=None, skip_in=None, skip_out=None):
            ss, kv, fold = pre.get(id(blk), (None, None, None))
            mark(x)
            return blk.forward_cl(x, t, cond, batch, x1=x1, ss=ss, kv=kv, fold=fold,
                                  skip_in=skip_in, skip_out=skip_out)

        # every skip (r and the hiddens) carries an ops.SkipGrad: its up-path
        # readers park their input gradient there and its down-path reader adds
        # them in its own kernel -- no autograd sum of strided gradient views
        skip_r = ops.SkipGrad()
        pending = skip_r  # the SkipGrad of the next down-path block's input
        hiddens = []
        for _, init_block, blocks, attn, post in self.downs:
            x = run(init_block, x, c, skip_in=pending)
            pending = None
            for blk in blocks:
                x = run(blk, x, c, skip_in=pending)
                pending = ops.SkipGrad()
                hiddens.append((x, pending))
            hiddens.append((x, pending))  # after the Identity attention
            mark(x)
            x = post.forward_cl(x, skip_in=pending)
            pending = None
        x = run(self.mid_block1, x, mid_c)
        if exists(self.mid_attn):
            mark(x)
            x = self.mid_attn.forward_cl(x, batch)
        x = run(self.mid_block2, x, mid_c)
        for init_block, blocks, attn, up in self.ups:
            hx, hs = hiddens.pop()
            x = run(init_block, x, c, x1=hx, skip_out=hs)
            for blk in blocks:
                hx, hs = hiddens.pop()
                x = run(blk, x, c, x1=hx, skip_out=hs)
            if not isinstance(up, nn.Identity):
                mark(x)
                x = up.forward_cl(x)
        x = run(self.final_resnet_block, x, None, x1=r, skip_out=skip_r)
        mark(x)
        return ops.conv(x, self.to_out.weight, self.to_out.bias, x1=lowres_cl)

    def forward(self, x, time, *, video_embed=None, lowres_cond_video=None,
                lowres_noise_level=None, text_encodings=None, video_cond_drop_prob=0.0,
                text_cond_drop_prob=0.0, blur_sigma=None, blur_kernel_size=None,
                disable_checkpoint=False, self_cond=None):
        batch = x.shape[0]
        assert not (self.lowres_cond and not exists(lowres_cond_video)), \
            "low resolution conditioning image must be present"
        if exists(lowres_noise_level):
            raise AssertionError("lowres_noise_cond must be set to True on instantiation of the "
                                 "unet in order to conditiong on lowres noise")
        dt = _compute_dtype(self, x)
        xin = torch.cat((x, lowres_cond_video), dim=1) if exists(lowres_cond_video) else x
        xcl = ops.to_cl(xin, dt)
        lcl = ops.to_cl(lowres_cond_video, dt) if exists(lowres_cond_video) else None
        y = self.forward_cl(xcl, time, batch=batch, lowres_cl=lcl,
                            video_cond_drop_prob=video_cond_drop_prob,
                            text_cond_drop_prob=text_cond_drop_prob)
        return ops.from_cl(y, batch, self.channels_out, x.shape[2])


class UnetTemporalConv(nn.Module):
    """Reference marks it 'probably doesn't work' (dalle2_video.py:957) and
    train_decoder.py never builds it: outside the MI355X hot path."""

    def __init__(self, *args, **kwargs):
        raise NotImplementedError("UnetTemporalConv is outside the MI355X hot path (SURVEY §2)")


# ---------------------------------------------------------------------------
# LowresVideoConditioner (dalle2_video.py:1044-1166) — cascade SR stage
# ---------------------------------------------------------------------------


def resize_video_to(video, size, clamp_range=None, nearest=True):
    """Per-frame nearest resize of an NCTHW clip (temporal_apply(resize_image_to))."""
    if video.shape[-1] == size:
        return video
    if not nearest:
        raise NotImplementedError("bilinear resize is outside the hot path")
    return ops.resize_nearest(video, size, clamp_range)


class LowresVideoConditioner(nn.Module):
    def __init__(self, downsample_first=True, use_blur=True, blur_prob=0.5, blur_sigma=0.6,
                 blur_kernel_size=3, use_noise=False, input_video_range=None,
                 normalize_video_fn=identity, unnormalize_video_fn=identity):
        super().__init__()
        if use_noise:
            raise NotImplementedError("Imagen-style lowres noising is outside the hot path")
        self.downsample_first = downsample_first
        self.input_video_range = input_video_range
        self.use_blur = use_blur
        self.blur_prob = blur_prob
        self.blur_sigma = blur_sigma
        self.blur_kernel_size = blur_kernel_size
        self.use_noise = use_noise
        self.normalize_video = normalize_video_fn
        self.unnormalize_video = unnormalize_video_fn
        self.noise_scheduler = None
        # the trainer's graphed calls draw the blur decision themselves (the
        # same one random.random() per call) and pin it here for the call
        self.forced_blur = None

    def forward(self, cond_fmap, *, target_frame_size, downsample_frame_size=None,
                target_frame_number=None, downsample_frame_number=None, should_blur=True,
                blur_sigma=None, blur_kernel_size=None):
        if self.downsample_first and exists(downsample_frame_size):
            cond_fmap = resize_video_to(cond_fmap, downsample_frame_size,
                                        clamp_range=self.input_video_range)
        if self.use_blur and should_blur and (
                self.forced_blur if self.forced_blur is not None else random.random() < self.blur_prob):
            sigma = default(blur_sigma, self.blur_sigma)
            ks = default(blur_kernel_size, self.blur_kernel_size)
            if isinstance(sigma, tuple):
                sigma = random.uniform(*map(float, sigma))
            if isinstance(ks, tuple):
                ks = random.randrange(int(ks[0]), int(ks[1]) + 1)
            cond_fmap = ops.gaussian_blur(cond_fmap, int(ks), float(sigma))
        cond_fmap = resize_video_to(cond_fmap, target_frame_size, clamp_range=self.input_video_range)
        return cond_fmap, None


# ---------------------------------------------------------------------------
# one DDPM denoise step as a replayable HIP graph (sampling loop, config 4)
# ---------------------------------------------------------------------------


class _DenoiseStepGraph:
    """x <- p_sample(unet, x, t) in place (dalle2_video.py:1621-1664 inside the
    loop at :1707-1735).  The loop state `x` and the timestep buffer `t` are
    fixed device buffers; the first two calls run eagerly (every lazily
    allocated workspace exists afterwards), the third captures the step —
    Unet3D forward (two with classifier-free guidance), `randn_like` noise on
    the device generator and the posterior update written back into x — and
    every call from then on sets t and replays the graph."""

    EAGER_CALLS = 2

    def __init__(self, decoder, unet, x, video_embed, noise_scheduler, cond_scale, lowres_cond_vid,
                 clip_denoised):
        self.decoder, self.unet, self.x = decoder, unet, x
        self.video_embed, self.sched, self.cond_scale = video_embed, noise_scheduler, cond_scale
        self.lowres, self.clip = lowres_cond_vid, clip_denoised
        self.t = torch.zeros(x.shape[0], dtype=torch.long, device=x.device)
        self.calls = 0
        self.graph = None

    def _body(self):
        x, unet = self.x, self.unet
        if self.cond_scale == 1:
            # forward without the NCTHW round trip: the update reads the
            # channels-last prediction directly
            dt = _compute_dtype(unet, x)
            xin = torch.cat((x, self.lowres), dim=1) if exists(self.lowres) else x
            lcl = ops.to_cl(self.lowres, dt) if exists(self.lowres) else None
            eps = unet.forward_cl(ops.to_cl(xin, dt), self.t, batch=x.shape[0], lowres_cl=lcl)
        else:
            eps = unet.forward_with_cond_scale(x, self.t, video_embed=self.video_embed,
                                               cond_scale=self.cond_scale,
                                               lowres_cond_video=self.lowres)
        noise = torch.randn_like(x)
        ops.p_sample_step(x, eps, noise, self.t, self.sched, self.clip, out=x, want_x0=False)

    def __call__(self, time):
        self.t.fill_(time)
        self.calls += 1
        if self.calls <= self.EAGER_CALLS or ops.TIMER is not None:
            self._body()
            return
        if self.graph is None:
            torch.cuda.synchronize()
            self.graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.graph, capture_error_mode="thread_local"):
                self._body()
                ops.gn_graph_boundary(self.x.device)
        self.graph.replay()


# ---------------------------------------------------------------------------
# VideoDecoder (dalle2_video.py:1169-2299)
# ---------------------------------------------------------------------------


def _move_module(module, device):
    """`module.to(device)` for the host <-> GPU moves of one_unet_in_gpu, as ONE
    copy per dtype through a pinned host buffer kept on the module: the
    parameters, their gradients and the buffers become views of one flat
    tensor on the target device (pinned host memory, or a fresh GPU buffer).
    Module.to() moves ~440 tensors through pageable memory one by one.
    Other devices / mixed layouts fall back to Module.to()."""
    device = torch.device(device)
    ts = []
    for p in module.parameters():
        ts.append(p)
        if p.grad is not None:
            ts.append(p.grad)
    ts += [b for b in module.buffers()]
    if not ts or all(t.device == device for t in ts) or \
            (device.type == "cuda" and device.index is None and all(t.is_cuda for t in ts)):
        return
    src_dev = ts[0].device
    if device.type not in ("cpu", "cuda") or any(t.device != src_dev for t in ts) or \
            not torch.cuda.is_available() or (src_dev.type == "cpu") == (device.type == "cpu"):
        module.to(device)
        return
    groups = {}
    for t in ts:
        groups.setdefault(t.dtype, []).append(t)
    cache = module.__dict__.setdefault("_dv_pinned", {})
    for dt, group in groups.items():
        n = sum(t.numel() for t in group)
        if device.type == "cpu":
            flat = cache.get(dt)
            if flat is None or flat.numel() != n:
                flat = cache[dt] = torch.empty(n, dtype=dt, pin_memory=True)
            gflat = torch.empty(n, dtype=dt, device=src_dev)
            off = 0
            for t in group:
                gflat[off:off + t.numel()].copy_(t.data.reshape(-1))
                off += t.numel()
            flat.copy_(gflat, non_blocking=True)
        else:
            flat = torch.empty(n, dtype=dt, device=device)
            cpu_flat = cache.get(dt)
            if cpu_flat is None or cpu_flat.numel() != n or any(
                    not _views_of(t, cpu_flat) for t in group):
                module.to(device)  # not laid out by a previous host move
                return
            flat.copy_(cpu_flat, non_blocking=True)
        off = 0
        for t in group:
            t.data = flat[off:off + t.numel()].view(t.shape)
            off += t.numel()
    if device.type == "cpu":
        torch.cuda.current_stream(src_dev).synchronize()  # host views are read-ready


def _views_of(t, flat):
    return t.device.type == "cpu" and t.untyped_storage().data_ptr() == flat.untyped_storage().data_ptr()


class VideoDecoder(nn.Module):
    def __init__(self, unet, *, clip=None, frame_size=None, channels=3, vae=tuple(),
                 timesteps=1000, sample_timesteps=None, video_cond_drop_prob=0.1,
                 text_cond_drop_prob=0.5, loss_type="l2", beta_schedule=None,
                 predict_x_start=False, predict_v=False,
                 predict_x_start_for_latent_diffusion=False, frame_sizes=None, frame_numbers=None,
                 random_crop_sizes=None, use_noise_for_lowres_cond=False,
                 use_blur_for_lowres_cond=True, lowres_downsample_first=True, blur_prob=0.5,
                 blur_sigma=0.6, blur_kernel_size=3, lowres_noise_sample_level=0.2,
                 clip_denoised=True, clip_x_start=True, clip_adapter_overrides=dict(),
                 learned_variance=True, learned_variance_constrain_frac=False,
                 vb_loss_weight=0.001, unconditional=False, auto_normalize_video=True,
                 use_dynamic_thres=False, dynamic_thres_percentile=0.95,
                 p2_loss_weight_gamma=0.0, p2_loss_weight_k=1, ddim_sampling_eta=0.0):
        super().__init__()
        if exists(clip):
            raise NotImplementedError("CLIP adapters are outside the MI355X hot path")
        self.clip = None
        if exists(frame_size) or exists(frame_sizes):
            assert exists(frame_size) ^ exists(frame_sizes), \
                "only one of image_size or image_sizes must be given"
            frame_size = default(frame_size, lambda: frame_sizes[-1])
        else:
            raise Exception("either image_size, image_sizes, or clip must be given to decoder")
        self.channels = channels
        self.normalize_video = normalize_neg_one_to_one if auto_normalize_video else identity
        self.unnormalize_video = unnormalize_zero_to_one if auto_normalize_video else identity
        self.auto_normalize_video = auto_normalize_video
        unets = cast_tuple(unet)
        num_unets = len(unets)
        self.num_unets = num_unets
        self.unconditional = unconditional
        vaes = pad_tuple_to_length(cast_tuple(vae), num_unets,
                                   fillvalue=NullVQGanVAE(channels=self.channels))
        learned_variance = pad_tuple_to_length(cast_tuple(learned_variance), num_unets,
                                               fillvalue=False)
        if any(learned_variance):
            raise NotImplementedError("learned_variance=True is outside the MI355X hot path "
                                      "(train_decoder.py passes learned_variance=False)")
        self.learned_variance = learned_variance
        self.learned_variance_constrain_frac = learned_variance_constrain_frac
        self.vb_loss_weight = vb_loss_weight
        use_noise = cast_tuple(use_noise_for_lowres_cond, num_unets - 1, validate=False)
        use_blur = cast_tuple(use_blur_for_lowres_cond, num_unets - 1, validate=False)
        if len(use_noise) < num_unets:
            use_noise = (False, *use_noise)
        if len(use_blur) < num_unets:
            use_blur = (False, *use_blur)
        assert not use_noise[0], "first unet will never need low res noise conditioning"
        assert not use_blur[0], "first unet will never need low res blur conditioning"
        assert num_unets == 1 or all((n or b) for n, b in zip(use_noise[1:], use_blur[1:]))
        self.unets = nn.ModuleList([])
        self.vaes = nn.ModuleList([])
        for ind, (one_unet, one_vae, lv, noise_cond) in enumerate(
                zip(unets, vaes, learned_variance, use_noise)):
            assert isinstance(one_unet, Unet3D)
            assert isinstance(one_vae, NullVQGanVAE), "only the identity (pixel-space) VAE"
            is_first = ind == 0
            unet_channels = default(one_vae.encoded_dim, self.channels)
            unet_channels_out = unet_channels * (1 if not lv else 2)
            one_unet = one_unet.cast_model_parameters(
                lowres_cond=not is_first, lowres_noise_cond=noise_cond,
                cond_on_image_embeds=not unconditional and is_first,
                cond_on_text_encodings=not unconditional and one_unet.cond_on_text_encodings,
                channels=unet_channels, channels_out=unet_channels_out)
            self.unets.append(one_unet)
            self.vaes.append(one_vae.copy_for_eval())
        self.sample_timesteps = cast_tuple(sample_timesteps, num_unets)
        self.ddim_sampling_eta = ddim_sampling_eta
        if not exists(beta_schedule):
            beta_schedule = ("cosine", *(("cosine",) * max(num_unets - 2, 0)),
                             *(("linear",) * int(num_unets > 1)))
        beta_schedule = cast_tuple(beta_schedule, num_unets)
        p2 = cast_tuple(p2_loss_weight_gamma, num_unets)
        self.noise_schedulers = nn.ModuleList([])
        for ind, (bs, g, st) in enumerate(zip(beta_schedule, p2, self.sample_timesteps)):
            assert not exists(st) or st <= timesteps, \
                f"sampling timesteps {st} must be less than or equal to the number of training timesteps {timesteps} for unet {ind + 1}"
            self.noise_schedulers.append(NoiseScheduler(beta_schedule=bs, timesteps=timesteps,
                                                        loss_type=loss_type,
                                                        p2_loss_weight_gamma=g,
                                                        p2_loss_weight_k=p2_loss_weight_k))
        frame_sizes = default(frame_sizes, (frame_size,))
        frame_sizes = tuple(sorted(set(frame_sizes)))
        assert self.num_unets == len(frame_sizes), \
            f"you did not supply the correct number of u-nets ({self.num_unets}) for resolutions {frame_sizes}"
        self.frame_sizes = frame_sizes
        self.sample_channels = cast_tuple(self.channels, len(frame_sizes))
        self.frame_numbers = frame_numbers
        self.random_crop_sizes = cast_tuple(random_crop_sizes, len(frame_sizes))
        assert not exists(self.random_crop_sizes[0])
        if any(exists(c) for c in self.random_crop_sizes):
            raise NotImplementedError("random crops (kornia) are outside the MI355X hot path")
        self.predict_x_start = (cast_tuple(predict_x_start, num_unets)
                                if not predict_x_start_for_latent_diffusion else (False,) * num_unets)
        self.predict_v = cast_tuple(predict_v, num_unets)
        if any(self.predict_x_start) or any(self.predict_v):
            raise NotImplementedError("x0 / v prediction is outside the MI355X hot path")
        self.input_video_range = (-1.0 if not auto_normalize_video else 0.0, 1.0)
        lowres_conditions = tuple(u.lowres_cond for u in self.unets)
        assert lowres_conditions == (False, *((True,) * (num_unets - 1)))
        self.lowres_conds = nn.ModuleList([])
        for ui, n, b in zip(range(num_unets), use_noise, use_blur):
            if ui == 0:
                self.lowres_conds.append(None)
                continue
            self.lowres_conds.append(LowresVideoConditioner(
                downsample_first=lowres_downsample_first, use_blur=b, use_noise=n,
                blur_prob=blur_prob, blur_sigma=blur_sigma, blur_kernel_size=blur_kernel_size,
                input_video_range=self.input_video_range,
                normalize_video_fn=self.normalize_video,
                unnormalize_video_fn=self.unnormalize_video))
        self.lowres_noise_sample_level = lowres_noise_sample_level
        self.video_cond_drop_prob = video_cond_drop_prob
        self.text_cond_drop_prob = text_cond_drop_prob
        self.can_classifier_guidance = video_cond_drop_prob > 0.0 or text_cond_drop_prob > 0.0
        self.clip_denoised = clip_denoised
        self.clip_x_start = clip_x_start
        if use_dynamic_thres:
            raise NotImplementedError("dynamic thresholding is outside the MI355X hot path")
        self.use_dynamic_thres = use_dynamic_thres
        self.dynamic_thres_percentile = dynamic_thres_percentile
        self.register_buffer("_dummy", torch.Tensor([True]), persistent=False)
        # the DDPM loop replays one captured HIP graph per denoise step
        # (DV_SAMPLE_GRAPHS=0: launch every step eagerly)
        import os
        self.sample_graphs = os.environ.get("DV_SAMPLE_GRAPHS", "1") != "0"

    @property
    def device(self):
        return self._dummy.device

    @property
    def condition_on_text_encodings(self):
        # Q4: the reference tests isinstance(unet, Unet) (the 2-D class): always False
        return False

    def get_unet(self, unet_number):
        assert 0 < unet_number <= self.num_unets
        return self.unets[unet_number - 1]

    @contextmanager
    def one_unet_in_gpu(self, unet_number=None, unet=None, cuda="cuda"):
        assert exists(unet_number) ^ exists(unet)
        if exists(unet_number):
            unet = self.get_unet(unet_number)
        cuda, cpu = torch.device(cuda), torch.device("cpu")
        self.to(cuda)
        devices = [next(u.parameters()).device for u in self.unets]
        for u in self.unets:
            _move_module(u, cpu)
        _move_module(unet, cuda)
        yield
        for u, d in zip(self.unets, devices):
            _move_module(u, d)

    # ---- training (p_losses, dalle2_video.py:1908-2006) -------------------
    def p_losses(self, unet, x_start, times, *, video_embed, noise_scheduler,
                 lowres_cond_video=None, text_encodings=None, predict_x_start=False,
                 predict_v=False, noise=None, learned_variance=False, clip_denoised=False,
                 is_latent_diffusion=False, lowres_noise_level=None):
        noise = default(noise, lambda: torch.randn_like(x_start))
        dt = _compute_dtype(unet, x_start)
        B, C, T = x_start.shape[:3]
        # x_t = sqrt(ac[t]) * (2 x0 - 1) + sqrt(1 - ac[t]) * eps, written channels-last
        xn = ops.q_sample_cl(x_start, noise, times, noise_scheduler.sqrt_alphas_cumprod,
                             noise_scheduler.sqrt_one_minus_alphas_cumprod, dt,
                             normalize=not is_latent_diffusion)
        lcl = None
        if exists(lowres_cond_video):
            lv = lowres_cond_video if is_latent_diffusion else self.normalize_video(lowres_cond_video)
            lcl = ops.to_cl(lv, dt)
            lc = lv.shape[1]
            if C + lc > xn.shape[-1]:
                raise DVError("lowres conditioning needs C + C_lowres <= 8 channels")
            xn[..., C:C + lc] = lcl[..., :lc]  # the channel concat (dalle2_video.py:744)
        pred = unet.forward_cl(xn, times, batch=B, lowres_cl=lcl,
                               video_cond_drop_prob=self.video_cond_drop_prob,
                               text_cond_drop_prob=self.text_cond_drop_prob)
        sw = None
        if noise_scheduler.has_p2_loss_reweighting:
            sw = noise_scheduler.p2_loss_weight.gather(-1, times)
        return ops.mse_loss_cl(pred, noise, sw)

    def forward(self, video, video_embed=None, text=None, text_encodings=None, unet_number=None,
                return_lowres_cond_video=False):
        assert not (self.num_unets > 1 and not exists(unet_number)), \
            f"you must specify which unet you want trained, from a range of 1 to {self.num_unets}, if you are training cascading DDPM (multiple unets)"
        unet_number = default(unet_number, 1)
        ui = unet_number - 1
        unet = self.get_unet(unet_number)
        noise_scheduler = self.noise_schedulers[ui]
        lowres_conditioner = self.lowres_conds[ui]
        target_frame_size = self.frame_sizes[ui]
        b, c, t, h, w = video.shape
        assert c == self.channels
        assert h >= target_frame_size and w >= target_frame_size
        times = torch.randint(0, noise_scheduler.num_timesteps, (b,), device=video.device,
                              dtype=torch.long)
        assert not exists(text_encodings) and not exists(text), \
            "decoder specified not to be conditioned on text, yet it is presented"
        lowres_cond_video = None
        if exists(lowres_conditioner):
            lowres_cond_video, _ = lowres_conditioner(
                video, target_frame_size=target_frame_size,
                downsample_frame_size=self.frame_sizes[ui - 1])
        video = resize_video_to(video, target_frame_size)
        loss = self.p_losses(unet, video, times, video_embed=video_embed,
                             lowres_cond_video=lowres_cond_video,
                             noise_scheduler=noise_scheduler)
        if not return_lowres_cond_video:
            return loss
        return loss, lowres_cond_video

    # ---- sampling (dalle2_video.py:1531-1906, 2053-2186) ------------------
    @torch.no_grad()
    def p_sample(self, unet, x, t, video_embed, noise_scheduler, text_encodings=None,
                 cond_scale=1.0, lowres_cond_vid=None, self_cond=None, predict_x_start=False,
                 predict_v=False, learned_variance=False, clip_denoised=True,
                 lowres_noise_level=None, noise=None):
        assert not (cond_scale != 1.0 and not self.can_classifier_guidance)
        pred = unet.forward_with_cond_scale(x, t, video_embed=video_embed,
                                            cond_scale=cond_scale,
                                            lowres_cond_video=lowres_cond_vid)
        noise = default(noise, lambda: torch.randn_like(x))
        out, x0 = ops.p_sample_step(x, pred, noise, t, noise_scheduler, clip_denoised)
        return out, x0

    @torch.no_grad()
    def p_sample_loop_ddpm(self, unet, shape, video_embed, noise_scheduler, predict_x_start=False,
                           predict_v=False, learned_variance=False, clip_denoised=True,
                           lowres_cond_vid=None, text_encodings=None, cond_scale=1,
                           is_latent_diffusion=False, lowres_noise_level=None):
        """dalle2_video.py:1667-1755.  On the GPU every denoise step after the
        first two is a replay of one captured HIP graph (_DenoiseStepGraph):
        the Unet3D forward(s), the device-side noise draw and the in-place
        posterior update, with no host launches in between."""
        b = shape[0]
        vid = torch.randn(shape, device=self.device)
        if not is_latent_diffusion:
            lowres_cond_vid = maybe(self.normalize_video)(lowres_cond_vid)
        if vid.is_cuda and self.sample_graphs:
            with ops.private_pack_cache():
                step = _DenoiseStepGraph(self, unet, vid, video_embed, noise_scheduler, cond_scale,
                                         lowres_cond_vid, clip_denoised)
                for time in reversed(range(0, noise_scheduler.num_timesteps)):
                    step(time)
                del step
            return self.unnormalize_video(vid)
        # the eager loop packs its (unchanging) weights into a private cache too, so
        # sampling never adds entries the trainer's per-update refresh would repack
        with (ops.private_pack_cache() if vid.is_cuda else nullcontext()):
            for time in reversed(range(0, noise_scheduler.num_timesteps)):
                times = torch.full((b,), time, device=self.device, dtype=torch.long)
                vid, _ = self.p_sample(unet, vid, times, video_embed=video_embed,
                                       cond_scale=cond_scale, lowres_cond_vid=lowres_cond_vid,
                                       noise_scheduler=noise_scheduler, clip_denoised=clip_denoised)
        return self.unnormalize_video(vid)

    @torch.no_grad()
    def p_sample_loop(self, *args, noise_scheduler, timesteps=None, **kwargs):
        num_timesteps = noise_scheduler.num_timesteps
        timesteps = default(timesteps, num_timesteps)
        assert timesteps <= num_timesteps
        if timesteps < num_timesteps:
            # the reference DDIM path raises TypeError for Unet3D
            raise TypeError("p_sample_loop_ddim is broken for Unet3D in the reference "
                            "(image_embed= / lowres_cond_img= keywords, dalle2_video.py:1832-1841)")
        return self.p_sample_loop_ddpm(*args, noise_scheduler=noise_scheduler, **kwargs)

    @torch.no_grad()
    def sample(self, video=None, video_embed=None, text=None, text_encodings=None, batch_size=1,
               cond_scale=1.0, start_at_unet_number=1, stop_at_unet_number=None,
               distributed=False, one_unet_in_gpu_at_time=True, cuda="cuda"):
        assert self.unconditional or exists(video_embed), \
            "image embed must be present on sampling from decoder unless if trained unconditionally"
        if not self.unconditional:
            batch_size = video_embed.shape[0]
        assert not exists(text_encodings) and not exists(text)
        was_training = self.training
        self.eval()
        vid = None
        if start_at_unet_number > 1:
            assert exists(video)
            assert video.shape[0] == batch_size
            vid = resize_video_to(video, self.frame_sizes[start_at_unet_number - 2])
        is_cuda = next(self.parameters()).is_cuda
        cond_scale = cast_tuple(cond_scale, self.num_unets)
        for (unet_number, unet, vae, channel, frame_size, frame_number, noise_scheduler,
             lowres_cond, sample_timesteps, unet_cond_scale) in zip(
                range(1, self.num_unets + 1), self.unets, self.vaes, self.sample_channels,
                self.frame_sizes, self.frame_numbers, self.noise_schedulers, self.lowres_conds,
                self.sample_timesteps, cond_scale):
            if unet_number < start_at_unet_number:
                continue
            ctxm = (self.one_unet_in_gpu(unet=unet, cuda=cuda)
                    if is_cuda and one_unet_in_gpu_at_time else nullcontext())
            with ctxm:
                lowres_cond_vid = None
                shape = (batch_size, channel, frame_number, frame_size, frame_size)
                if unet.lowres_cond:
                    lowres_cond_vid = resize_video_to(vid, frame_size,
                                                      clamp_range=self.input_video_range)
                vid = self.p_sample_loop(unet, shape, video_embed=video_embed,
                                         cond_scale=unet_cond_scale,
                                         lowres_cond_vid=lowres_cond_vid,
                                         noise_scheduler=noise_scheduler,
                                         timesteps=sample_timesteps,
                                         clip_denoised=True)
            if exists(stop_at_unet_number) and stop_at_unet_number == unet_number:
                break
        self.train(was_training)
        return vid


class DALLE2Video(nn.Module):
    """The prior+decoder chain (dalle2_video.py:2302-2370) needs a trained
    dalle2-pytorch DiffusionPrior, which is outside the MI355X hot path."""

    def __init__(self, *, prior, decoder, temporal_emb=False, prior_num_samples=2,
                 decoder_cuda="cuda"):
        super().__init__()
        raise NotImplementedError("DALLE2Video (prior + decoder) is outside the MI355X hot path")
