"""Autograd-visible ops of the HIP path, over channels-last frame tensors.

An activation is a (NF, H, W, C) tensor (NF = batch*frames) whose channel
dimension is unit-stride; its pixel stride `ld` may exceed C (a channel
slice of a wider buffer).  Every op calls libdv_hip through `_lib.call`; there
is no torch-compute fallback.
"""
from __future__ import annotations

import torch

from . import _lib
from ._lib import ACT_NONE, call, dt, ptr, require_gpu, stream


def cl_ld(t: torch.Tensor) -> int:
    """Pixel stride of a channels-last frame tensor (asserts the layout)."""
    if t.dim() != 4 or (t.stride(3) != 1 and t.shape[3] > 1):
        raise _lib.DVError(f"expected a channels-last (NF,H,W,C) tensor, got {tuple(t.shape)} "
                           f"strides {t.stride()}")
    nf, h, w, c = t.shape
    ld = t.stride(2) if w > 1 else (t.stride(1) if h > 1 else max(c, t.stride(0) if nf > 1 else c))
    if (w > 1 and h > 1 and t.stride(1) != w * ld) or (nf > 1 and h * w > 1 and t.stride(0) != h * w * ld):
        raise _lib.DVError(f"non-uniform pixel stride {t.stride()}")
    return ld


def _pad_channels(t: torch.Tensor, mult: int = 8) -> torch.Tensor:
    c = t.shape[-1]
    cp = (c + mult - 1) // mult * mult
    if cp == c and t.is_contiguous():
        return t
    out = torch.zeros(*t.shape[:-1], cp, dtype=t.dtype, device=t.device)
    out[..., :c] = t
    return out


def pack_conv_weight(weight: torch.Tensor, dtype, pad_to: int, mode: int) -> torch.Tensor:
    cout, cin = weight.shape[0], weight.shape[1]
    k = weight.shape[-1]
    rows = cout if mode == 0 else cin
    out = (torch.empty if mode == 0 else torch.zeros)(rows, k * k, pad_to, dtype=dtype,
                                                      device=weight.device)
    w = weight.detach()
    if w.dtype != torch.float32 or not w.is_contiguous():
        w = w.float().contiguous()
    call("dv_pack_conv_weight", _lib.DV_BF16 if dtype == torch.bfloat16 else _lib.DV_F32,
         ptr(w), ptr(out), cout, cin, k, pad_to, mode, stream())
    return out


class ConvFn(torch.autograd.Function):
    """y = conv_(1,k,k)(cat(x0, x1)) + bias (+ res).  dalle2_video.py:107 etc."""

    @staticmethod
    def forward(ctx, x0, x1, weight, bias, res, ksize):
        require_gpu(x0, x1, weight, bias, res)
        nf, h, w, c0 = x0.shape
        c1 = 0 if x1 is None else x1.shape[3]
        cin = c0 + c1
        cout, cin_real = weight.shape[0], weight.shape[1]
        if cin_real > cin:
            raise _lib.DVError(f"conv: weight expects {cin_real} input channels, got {cin}")
        wp = pack_conv_weight(weight, x0.dtype, cin, 0)
        y = torch.empty(nf, h, w, cout, dtype=x0.dtype, device=x0.device)
        ld0 = cl_ld(x0)
        ld1 = cl_ld(x1) if x1 is not None else 0
        ldr = cl_ld(res) if res is not None else 0
        b = None if bias is None else bias.detach().float().contiguous()
        call("dv_conv_fwd", dt(x0), ptr(x0), ld0, c0, ptr(x1), ld1, ptr(wp), ptr(b), ptr(res), ldr,
             ptr(y), cout, nf, h, w, cin, cout, ksize, ACT_NONE, stream())
        ctx.save_for_backward(x0, x1, weight)
        ctx.meta = (ksize, c0, c1, bias is not None, res is not None)
        return y

    @staticmethod
    def backward(ctx, dy):
        x0, x1, weight = ctx.saved_tensors
        ksize, c0, c1, has_bias, has_res = ctx.meta
        nf, h, w, _ = x0.shape
        cin = c0 + c1
        cout, cin_real = weight.shape[0], weight.shape[1]
        dy8 = _pad_channels(dy.contiguous())
        cout8 = dy8.shape[3]
        dx0 = dx1 = dw = db = None
        if ctx.needs_input_grad[0] or ctx.needs_input_grad[1]:
            wpd = pack_conv_weight(weight, dy.dtype, cout8, 1)
            alloc = torch.empty if cin_real == cin else torch.zeros
            dx = alloc(nf, h, w, cin, dtype=dy.dtype, device=dy.device)
            call("dv_conv_fwd", dt(dy8), ptr(dy8), cout8, cout8, None, 0, ptr(wpd), None, None, 0,
                 ptr(dx), cin, nf, h, w, cout8, cin_real, ksize, ACT_NONE, stream())
            dx0 = dx[..., :c0]
            dx1 = dx[..., c0:] if x1 is not None else None
        if ctx.needs_input_grad[2]:
            ws = torch.zeros(cout8, ksize * ksize, cin, dtype=torch.float32, device=dy.device)
            ld0 = cl_ld(x0)
            ld1 = cl_ld(x1) if x1 is not None else 0
            call("dv_conv_wgrad", dt(dy8), ptr(dy8), cout8, ptr(x0), ld0, c0, ptr(x1), ld1, ptr(ws),
                 nf, h, w, cin, cout8, ksize, stream())
            dw = torch.empty(weight.shape, dtype=torch.float32, device=dy.device)
            call("dv_unpack_wgrad", ptr(ws), ptr(dw), cout8, cin, ksize, cout, cin_real, 0, stream())
        if has_bias and ctx.needs_input_grad[3]:
            db = torch.zeros(cout, dtype=torch.float32, device=dy.device)
            call("dv_bias_grad", dt(dy8), ptr(dy8), cout8, ptr(db), nf * h * w, cout, stream())
        dres = dy if has_res else None
        return dx0, dx1, dw, db, dres, None


def conv(x0, weight, bias=None, x1=None, res=None):
    """(1,k,k) 'same' convolution over channels-last frames (weight in torch
    Conv3d layout (cout, cin, 1, k, k) or Linear layout (cout, cin))."""
    k = weight.shape[-1] if weight.dim() == 5 else 1
    return ConvFn.apply(x0, x1, weight, bias, res, k)
