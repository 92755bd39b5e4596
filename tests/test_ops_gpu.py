"""HIP ops (GN, LN, cross-attention, MQA, shuffles, layout, loss, small
linears) vs plain-PyTorch fp32 CPU references of the same op (forward + grads).
fp32 mode: rel-err <= 2e-5; bf16 mode: <= 2e-2."""
import math

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DTYPES = [(torch.float32, 2e-5), (torch.bfloat16, 2.5e-2)]


def rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def grads_match(outs_gpu, outs_ref, tol):
    for i, (a, b) in enumerate(zip(outs_gpu, outs_ref)):
        if b is None:
            continue
        e = rel(a, b)
        assert e < tol, f"grad {i}: rel-err {e:.3e} >= {tol}"


def _leaf(t, dev=None, dtype=None):
    t = t.detach()
    if dev is not None:
        t = t.to(dev)
    if dtype is not None:
        t = t.to(dtype)
    return t.clone().requires_grad_()


@pytest.mark.parametrize("dtype,tol", DTYPES)
@pytest.mark.parametrize("with_ss,with_res,nb,C", [(True, False, 2, 64), (False, True, 2, 64),
                                                   (True, False, 4, 512), (True, True, 3, 1024)])
def test_group_norm_act(dtype, tol, with_ss, with_res, nb, C):
    """GroupNorm (+FiLM, SiLU, residual): the reduce's last workgroup finishes the
    statistics / parameter gradients in sample chunks (C=512, 1024 take several)."""
    from dalle2_video import ops

    g = torch.Generator().manual_seed(3)
    T, H, W, G = 3, 8, 8, 8
    z = torch.randn(nb * T, H, W, C, generator=g) * 2 + 0.5
    gamma = 1 + 0.1 * torch.randn(C, generator=g)
    beta = 0.1 * torch.randn(C, generator=g)
    ss = 0.3 * torch.randn(nb, 2 * C, generator=g) if with_ss else None
    res = torch.randn(nb * T, H, W, C, generator=g) if with_res else None
    gy = torch.randn(nb * T, H, W, C, generator=g)
    # reference: torch GroupNorm on (b, c, t, h, w)
    zr = _leaf(z.to(dtype).float())
    gr, br = _leaf(gamma), _leaf(beta)
    ssr = _leaf(ss) if with_ss else None
    x5 = zr.reshape(nb, T, H, W, C).permute(0, 4, 1, 2, 3)
    y5 = F.group_norm(x5, G, gr, br, eps=1e-5)
    if with_ss:
        y5 = y5 * (ssr[:, :C, None, None, None] + 1) + ssr[:, C:, None, None, None]
    y5 = F.silu(y5)
    yr = y5.permute(0, 2, 3, 4, 1).reshape(nb * T, H, W, C)
    if with_res:
        yr = yr + res.to(dtype).float()
    (yr * gy).sum().backward()
    zd = _leaf(z, "cuda", dtype)
    gd, bd = _leaf(gamma, "cuda"), _leaf(beta, "cuda")
    ssd = _leaf(ss, "cuda") if with_ss else None
    resd = res.to("cuda", dtype) if with_res else None
    y = ops.group_norm_act(zd, gd, bd, nb, G, 1e-5, scale_shift=ssd, res=resd)
    assert rel(y.float(), yr) < tol
    (y.float() * gy.cuda()).sum().backward()
    grads_match([zd.grad.float(), gd.grad, bd.grad] + ([ssd.grad] if with_ss else []),
                [zr.grad, gr.grad, br.grad] + ([ssr.grad] if with_ss else []), tol * 2)


@pytest.mark.parametrize("dtype,tol", DTYPES)
@pytest.mark.parametrize("C,bias,res", [(512, False, True), (64, True, False)])
@pytest.mark.parametrize("rows", [8, 300, 4096])  # direct atomics / block partials / split column sum
def test_layer_norm(dtype, tol, C, bias, res, rows):
    from dalle2_video import ops

    g = torch.Generator().manual_seed(5)
    x = torch.randn(rows, C, generator=g) * 3 + 1
    w = 1 + 0.1 * torch.randn(C, generator=g)
    b = 0.1 * torch.randn(C, generator=g) if bias else None
    r = torch.randn(rows, C, generator=g) if res else None
    gy = torch.randn(rows, C, generator=g)
    xr, wr = _leaf(x.to(dtype).float()), _leaf(w)
    br = _leaf(b) if bias else None
    yr = F.layer_norm(xr, (C,), wr, br, eps=1e-5)
    if res:
        yr = yr + r.to(dtype).float()
    (yr * gy).sum().backward()
    xd, wd = _leaf(x, "cuda", dtype), _leaf(w, "cuda")
    bd = _leaf(b, "cuda") if bias else None
    y = ops.layer_norm(xd, wd, bd, r.to("cuda", dtype) if res else None, eps=1e-5)
    assert rel(y.float(), yr) < tol
    (y.float() * gy.cuda()).sum().backward()
    grads_match([xd.grad.float(), wd.grad] + ([bd.grad] if bias else []),
                [xr.grad, wr.grad] + ([br.grad] if bias else []), tol * 2)


def _ref_cross_attention(x_tok, ctx, g1, null_kv, wq, wkv, wo, g2, eps):
    # dalle2-pytorch CrossAttention + residual (see oracle/dv_ref.py)
    b = x_tok.shape[0]
    ln = lambda t, g: (t - t.mean(-1, keepdim=True)) * (t.var(-1, unbiased=False, keepdim=True) + eps).rsqrt() * g
    xn = ln(x_tok, g1)
    q = xn @ wq.t()
    kv = ctx @ wkv.t()
    k, v = kv.chunk(2, dim=-1)
    sp = lambda t: t.reshape(t.shape[0], t.shape[1], 8, 64).transpose(1, 2)
    q, k, v = sp(q), sp(k), sp(v)
    nk = null_kv[0].expand(b, 8, 1, 64)
    nv = null_kv[1].expand(b, 8, 1, 64)
    k, v = torch.cat((nk, k), dim=2), torch.cat((nv, v), dim=2)
    s = (q * 64 ** -0.25) @ (k * 64 ** -0.25).transpose(-1, -2)
    a = s.softmax(-1)
    o = (a @ v).transpose(1, 2).reshape(b, -1, 512)
    return ln(o @ wo.t(), g2) + x_tok


@pytest.mark.parametrize("dtype,tol", DTYPES)
@pytest.mark.parametrize("C,T,H,nb", [(64, 2, 8, 2), (256, 2, 8, 2), (16, 2, 4, 2), (8, 2, 2, 2), (48, 3, 3, 2),
                                      (512, 2, 8, 2), (192, 2, 8, 2), (128, 4, 16, 2), (32, 2, 8, 2),
                                      (128, 16, 32, 2),  # C >= 128: channel-split waves below 1024 token tiles
                                      (64, 2, 8, 3), (48, 3, 3, 4)])  # clips (<= 4: to_kv's 8 rows)
def test_cross_attention(dtype, tol, C, T, H, nb):
    # (16,2,4), (8,2,2), (48,3,3): channel counts below / not a multiple of one
    # 32-channel MFMA tile and tokens per clip (T*H*W) not a multiple of 32
    from dalle2_video import ops

    g = torch.Generator().manual_seed(7)
    W = H
    x = torch.randn(nb * T, H, W, C, generator=g)
    ctx = torch.randn(nb, 2, 64, generator=g)
    g1 = 1 + 0.1 * torch.randn(C, generator=g)
    g2 = 1 + 0.1 * torch.randn(C, generator=g)
    null_kv = torch.randn(2, 64, generator=g)
    wq = torch.randn(512, C, generator=g) / C ** 0.5
    wkv = torch.randn(1024, 64, generator=g) / 8
    wo = torch.randn(C, 512, generator=g) / 512 ** 0.5
    gy = torch.randn(nb * T, H, W, C, generator=g)
    ref_in = [_leaf(x.to(dtype).float()), _leaf(ctx), _leaf(g1), _leaf(null_kv), _leaf(wq),
              _leaf(wkv), _leaf(wo), _leaf(g2)]
    xt = ref_in[0].reshape(nb, -1, C)
    yr = _ref_cross_attention(xt, ref_in[1], ref_in[2], ref_in[3], ref_in[4], ref_in[5], ref_in[6],
                              ref_in[7], 1e-5).reshape(nb * T, H, W, C)
    (yr * gy).sum().backward()
    dev_in = [_leaf(x, "cuda", dtype)] + [_leaf(t, "cuda") for t in (ctx, g1, null_kv, wq, wkv, wo, g2)]
    eps = 1e-5
    y = ops.cross_attention(dev_in[0], dev_in[1], dev_in[2], dev_in[3], dev_in[4], dev_in[5],
                            dev_in[6], dev_in[7], nb, eps)
    assert rel(y.float(), yr) < tol
    (y.float() * gy.cuda()).sum().backward()
    grads_match([t.grad.float() for t in dev_in], [t.grad for t in ref_in], tol * 3)


@pytest.mark.parametrize("dtype,tol", DTYPES)
@pytest.mark.parametrize("N,qmag", [(64, 2), (96, 2), (97, 2), (1024, 2), (97, 40), (1024, 40)])
def test_mqa(dtype, tol, N, qmag):
    # qmag 40: |q| max|k| scale log2 e ~ 200 > 64 -- the bf16 forward keeps the
    # online running max (the bounded no-max path covers qmag 2)
    from dalle2_video import ops

    g = torch.Generator().manual_seed(11)
    B, H, D = 2, 16, 32
    q = torch.randn(B * N, H * D, generator=g) * qmag
    kv = torch.randn(B * N, 2 * D, generator=g) * 2
    null_kv = torch.randn(2, D, generator=g)
    gy = torch.randn(B * N, H * D, generator=g)
    qr, kvr, nr = _leaf(q.to(dtype).float()), _leaf(kv.to(dtype).float()), _leaf(null_kv)
    qh = qr.reshape(B, N, H, D).transpose(1, 2)
    k = torch.cat((nr[0].expand(B, 1, D), kvr[:, :D].reshape(B, N, D)), dim=1)
    v = torch.cat((nr[1].expand(B, 1, D), kvr[:, D:].reshape(B, N, D)), dim=1)
    s = torch.einsum("bhid,bjd->bhij", qh, k) / D
    o = torch.einsum("bhij,bjd->bhid", s.softmax(-1), v).transpose(1, 2).reshape(B * N, H * D)
    (o * gy).sum().backward()
    qd, kvd, nd = _leaf(q, "cuda", dtype), _leaf(kv, "cuda", dtype), _leaf(null_kv, "cuda")
    y = ops.mqa(qd, kvd, nd, B, N, H, 1.0 / D)
    assert rel(y.float(), o) < tol
    (y.float() * gy.cuda()).sum().backward()
    grads_match([qd.grad.float(), kvd.grad.float(), nd.grad], [qr.grad, kvr.grad, nr.grad], tol * 2)


@pytest.mark.parametrize("dtype,tol", DTYPES)
@pytest.mark.parametrize("nf,H,W,C", [(3, 4, 6, 16), (64, 32, 32, 64), (31, 5, 48, 40), (1, 70001, 1, 8)])
def test_shuffles(dtype, tol, nf, H, W, C):
    """Space-to-depth and SiLU + pixel shuffle (forward and backward): Cfg2's 64x64 -> 32x32
    level, a ragged one, and more low-res rows than the grid's 65,535 (row pairs per trip
    plus lone rows)."""
    from dalle2_video import ops

    g = torch.Generator().manual_seed(13)
    x = torch.randn(nf, 2 * H, 2 * W, C, generator=g)
    xr = _leaf(x.to(dtype).float())
    # reference: Downsample3D's rearrange 'b c t (h s1) (w s2) -> b (c s1 s2) t h w' per frame
    yr = F.pixel_unshuffle(xr.permute(0, 3, 1, 2), 2).permute(0, 2, 3, 1)
    gy = torch.randn(yr.shape, generator=g)
    (yr * gy).sum().backward()
    xd = _leaf(x, "cuda", dtype)
    y = ops.space_to_depth(xd)
    assert rel(y.float(), yr) < 1e-6
    (y.float() * gy.cuda()).sum().backward()
    assert rel(xd.grad.float(), xr.grad) < tol
    z = torch.randn(nf, H, W, 4 * C, generator=g)
    zr = _leaf(z.to(dtype).float())
    ur = F.pixel_shuffle(F.silu(zr).permute(0, 3, 1, 2), 2).permute(0, 2, 3, 1)
    gu = torch.randn(ur.shape, generator=g)
    (ur * gu).sum().backward()
    zd = _leaf(z, "cuda", dtype)
    u = ops.silu_pixel_shuffle(zd)
    assert rel(u.float(), ur) < tol
    (u.float() * gu.cuda()).sum().backward()
    assert rel(zd.grad.float(), zr.grad) < tol * 2


@pytest.mark.parametrize("dtype,tol", DTYPES)
def test_layout_and_loss(dtype, tol):
    from dalle2_video import ops

    g = torch.Generator().manual_seed(17)
    B, C, T, H, W = 2, 3, 4, 8, 8
    x = torch.randn(B, C, T, H, W, generator=g)
    y = ops.to_cl(x.cuda(), dtype)
    assert y.shape == (B * T, H, W, 8)
    assert torch.equal(y[..., 3:].float().cpu(), torch.zeros(B * T, H, W, 5))
    back = ops.from_cl(y, B, C, T)
    assert rel(back, x.to(dtype).float()) < 1e-7
    # q_sample + mse loss
    sched_a = torch.rand(1000, generator=g)
    sched_b = torch.rand(1000, generator=g)
    times = torch.tensor([3, 977])
    x0 = torch.rand(B, C, T, H, W, generator=g)
    noise = torch.randn(B, C, T, H, W, generator=g)
    xn = ops.q_sample_cl(x0.cuda(), noise.cuda(), times.cuda(), sched_a.cuda(), sched_b.cuda(), dtype)
    ref = sched_a[times].reshape(B, 1, 1, 1, 1) * (2 * x0 - 1) + sched_b[times].reshape(B, 1, 1, 1, 1) * noise
    assert rel(ops.from_cl(xn, B, C, T), ref) < tol
    pred = torch.randn(B, C, T, H, W, generator=g)
    pc = ops.to_cl(pred.cuda(), dtype).requires_grad_()
    loss = ops.mse_loss_cl(pc, noise.cuda())
    predr = _leaf(pred.to(dtype).float())
    lr = F.mse_loss(predr, noise)
    lr.backward()
    assert abs(loss.item() - lr.item()) / lr.item() < tol
    loss.backward()
    gd = ops.from_cl(pc.grad, B, C, T)
    assert rel(gd, predr.grad) < tol


def test_linear_small():
    from dalle2_video import ops

    g = torch.Generator().manual_seed(19)
    B, K, N = 4, 64, 256
    x = torch.randn(B, K, generator=g)
    w = torch.randn(N, K, generator=g) / 8
    b = torch.randn(N, generator=g)
    gy = torch.randn(B, N, generator=g)
    for act_in, act_out in [(0, 2), (1, 0)]:
        xr, wr, br = _leaf(x), _leaf(w), _leaf(b)
        xi = F.silu(xr) if act_in == 1 else xr
        yr = xi @ wr.t() + br
        if act_out == 2:
            yr = F.gelu(yr)
        (yr * gy).sum().backward()
        xd, wd, bd = _leaf(x, "cuda"), _leaf(w, "cuda"), _leaf(b, "cuda")
        y = ops.linear_small(xd, wd, bd, act_in, act_out)
        assert rel(y, yr) < 2e-6
        (y * gy.cuda()).sum().backward()
        grads_match([xd.grad, wd.grad, bd.grad], [xr.grad, wr.grad, br.grad], 2e-6)
    t = torch.tensor([0, 5, 537, 999])
    emb = ops.sinusoidal(t.cuda(), 64).cpu()
    half = 32
    f = torch.exp(torch.arange(half) * -(math.log(10000) / (half - 1)))
    a = t.float()[:, None] * f[None]
    assert rel(emb, torch.cat((a.sin(), a.cos()), -1)) < 2e-7


@pytest.mark.parametrize("act_in,ns,K", [(1, (128, 1024, 70, 512), 256), (0, (1024,) * 3, 64),
                                         (1, tuple(64 + 8 * i for i in range(50)), 32),
                                         (0, (100, 33), 512), (1, (40, 130), 36), (0, (65,), 4)])
def test_linear_group(act_in, ns, K):
    """Grouped small linears (time MLPs / to_kv): every entry's output and the
    dx / dW / db gradients vs per-layer fp32 torch; 50 entries span 2 launches."""
    from dalle2_video import ops

    g = torch.Generator().manual_seed(23)
    B = 4 if K != 64 else 8
    x = torch.randn(B, K, generator=g)
    ws = [torch.randn(n, K, generator=g) / 8 for n in ns]
    bs = [torch.randn(n, generator=g) if (act_in or i % 2) else None for i, n in enumerate(ns)]
    gys = [torch.randn(B, n, generator=g) for n in ns]
    xr = _leaf(x)
    wr = [_leaf(w) for w in ws]
    br = [None if b is None else _leaf(b) for b in bs]
    xi = F.silu(xr) if act_in == 1 else xr
    yr = [xi @ w.t() + (0 if b is None else b) for w, b in zip(wr, br)]
    sum((y * gy).sum() for y, gy in zip(yr, gys)).backward()
    xd = _leaf(x, "cuda")
    wd = [_leaf(w, "cuda") for w in ws]
    bd = [None if b is None else _leaf(b, "cuda") for b in bs]
    yd = ops.linear_group(xd, wd, bd, act_in=act_in)
    for a, b in zip(yd, yr):
        assert rel(a, b) < 2e-6
    sum((y * gy.cuda()).sum() for y, gy in zip(yd, gys)).backward()
    grads_match([xd.grad] + [w.grad for w in wd] + [b.grad for b in bd if b is not None],
                [xr.grad] + [w.grad for w in wr] + [b.grad for b in br if b is not None], 2e-6)


@pytest.mark.parametrize("N,B,qmag", [(2048, 2, 2), (4100, 1, 2), (8192, 2, 2), (2048, 2, 40)])
def test_mqa_forward_streamed_long_sequence(parity_log, N, B, qmag):
    """K/V-chunked flash forward (config 5: 32 x 16 x 16 = 8,192 mid tokens)
    vs a plain f32 softmax attention computed on the GPU head by head (the
    CPU reference would need the full (B, 16, N, N) scores).  qmag 40 puts
    the score bound above 64: the online-max path instead of the bounded one."""
    from dalle2_video import ops

    g = torch.Generator().manual_seed(13)
    H, D = 16, 32
    q = (torch.randn(B * N, H * D, generator=g) * qmag).cuda().to(torch.bfloat16)
    kv = (torch.randn(B * N, 2 * D, generator=g) * 2).cuda().to(torch.bfloat16)
    null_kv = torch.randn(2, D, generator=g).cuda()
    with torch.no_grad():
        y = ops.mqa(q, kv, null_kv, B, N, H, 1.0 / D).float()
        qf, kvf = q.float(), kv.float()
        ref = torch.empty_like(y)
        for b in range(B):
            k = torch.cat((null_kv[0][None], kvf[b * N:(b + 1) * N, :D]), 0)
            v = torch.cat((null_kv[1][None], kvf[b * N:(b + 1) * N, D:]), 0)
            for hh in range(H):
                qh = qf[b * N:(b + 1) * N, hh * D:(hh + 1) * D]
                ref[b * N:(b + 1) * N, hh * D:(hh + 1) * D] = ((qh @ k.t()) / D).softmax(-1) @ v
    e = rel(y, ref)
    parity_log(N=N, B=B, qmag=qmag, fwd_rel=e)
    assert e < 2.5e-2


def test_mqa_bf16_backward_long_sequence():
    """A bf16 mid attention longer than the bf16 backward's LDS limit (NKP >
    1280; config 5 trains at 8,193 keys) runs forward and backward on the f32
    kernels when gradients are needed: same values as the f32 path on the
    same (bf16-rounded) inputs, bf16 outputs and input gradients."""
    from dalle2_video import ops

    g = torch.Generator().manual_seed(21)
    B, N, H, D = 1, 2048, 16, 32
    q = torch.randn(B * N, H * D, generator=g).to(torch.bfloat16)
    kv = (torch.randn(B * N, 2 * D, generator=g) * 2).to(torch.bfloat16)
    null_kv = torch.randn(2, D, generator=g)
    gy = torch.randn(B * N, H * D, generator=g).cuda()
    outs = []
    for dtype in (torch.bfloat16, torch.float32):
        qd = _leaf(q.float(), "cuda", dtype)
        kvd = _leaf(kv.float(), "cuda", dtype)
        nd = _leaf(null_kv, "cuda")
        y = ops.mqa(qd, kvd, nd, B, N, H, 1.0 / D)
        assert y.dtype == dtype
        (y.float() * gy).sum().backward()
        assert qd.grad.dtype == dtype and kvd.grad.dtype == dtype
        outs.append([y.float(), qd.grad.float(), kvd.grad.float(), nd.grad])
    for a, b in zip(*outs):
        assert rel(a, b) < 1e-2  # one bf16 rounding of each output / gradient
    with torch.no_grad():  # no gradients: the bf16 streamed forward itself
        y = ops.mqa(q.cuda(), kv.cuda(), null_kv.cuda(), B, N, H, 1.0 / D)
    assert y.dtype == torch.bfloat16 and rel(y.float(), outs[1][0]) < 2.5e-2


@pytest.mark.parametrize("ngemm,nb,P,n", [(3, 4, 1000, 64), (3, 2, 4096, 128), (2, 1, 77, 256), (1, 3, 300, 64)])
def test_gemm_tn_batched_multi(ngemm, nb, P, n):
    """The one-launch form of the cross-attention token reductions: problem g,
    batch b gets out_g[b] += A_g[b rows]^T B_g[b rows] (f32 atomics on a
    pre-filled output), for operands of different leading dimensions."""
    import ctypes

    from dalle2_video._lib import call, stream

    g = torch.Generator().manual_seed(11)
    dev, m = "cuda", 32
    lds_a = [32, 40, 32][:ngemm]
    lds_b = [n, n + 8, 2 * n][:ngemm]
    A = [torch.randn(nb * P, la, generator=g).to(torch.bfloat16) for la in lds_a]
    B = [torch.randn(nb * P, lb, generator=g).to(torch.bfloat16) for lb in lds_b]
    O = [torch.randn(nb, m, n, generator=g) for _ in range(ngemm)]
    Ad = [t.to(dev) for t in A]
    Bd = [t.to(dev) for t in B]
    Od = [t.to(dev) for t in O]
    arr = lambda T, xs: (T * 3)(*(list(xs) + [xs[0]] * (3 - len(xs))))
    call("dv_gemm_tn_batched_multi", 1, ngemm, arr(ctypes.c_void_p, [t.data_ptr() for t in Ad]),
         arr(ctypes.c_int, lds_a), arr(ctypes.c_void_p, [t.data_ptr() for t in Bd]),
         arr(ctypes.c_int, lds_b), arr(ctypes.c_void_p, [t.data_ptr() for t in Od]), P, nb, m, n, stream())
    torch.cuda.synchronize()
    for a, b, o, od in zip(A, B, O, Od):
        ref = o.double() + torch.einsum("bri,brj->bij", a[:, :m].double().reshape(nb, P, m),
                                        b[:, :n].double().reshape(nb, P, n))
        assert rel(od, ref) < 1e-5
