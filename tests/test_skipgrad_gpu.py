"""Unet skip-gradient hand-off (ops.SkipGrad): the up-path convs reading a
hidden as the second input of their channel concat park dX1, and the hidden's
down-path reader adds the parked gradients in its own kernel -- a second dgrad
epilogue residual (dv_conv_fwd / dv_conv_fwd8 res2) or the depth-to-space
residual inputs (dv_shuffle r0 / r1) -- instead of autograd summing strided
views (dalle2_video.py:926-936 hiddens).  Checked against the same graph with
no hand-off (autograd sums) on every dgrad kernel family the consumer can hit,
and against an fp64 CPU reference of the whole graph."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def _graph(ops, x, ys, wd_a, wd_b, wups, gs, k, skip, consumer, order_ok=True):
    """Down readers of x: two convs sharing a GradSink (A recorded first: the
    second reader in the backward; B: the first), then len(ys) up convs
    reading (y_i, x).  consumer: 'A' / 'B' takes the SkipGrad.  order_ok=False
    records the up convs FIRST, so the consumer runs before the parkers."""
    sink = ops.GradSink()
    outs = []

    def down():
        za = ops.conv(x, wd_a, sink=sink, skip_in=skip if consumer == "A" else None)
        zb = ops.conv(x, wd_b, sink=sink, skip_in=skip if consumer == "B" else None)
        return [za, zb]

    def ups():
        return [ops.conv(y, w, x1=x, skip_out=skip) for y, w in zip(ys, wups)]

    if order_ok:
        outs = down() + ups()
    else:
        outs = ups() + down()
    return sum((o.float() * g).sum() for o, g in zip(outs, gs))


CASES = [
    # nf, h, w, c, k, n_up
    (4, 64, 64, 64, 3, 1),   # 64x64 stripe dgrad (the level-0 hidden)
    (4, 32, 32, 128, 3, 2),  # glds dgrad, two parked skips (res + res2 beside the sink)
    (16, 8, 8, 256, 3, 1),   # 8x8 window dgrad
    (8, 16, 16, 128, 3, 2),  # 16x16 window dgrad, two skips
    (8, 32, 32, 64, 1, 1),   # 1x1 consumer: the streamed 1x1 kernel with one residual
    (16, 8, 8, 256, 1, 2),   # 1x1 consumer, two skips
]


@pytest.mark.parametrize("consumer", ["A", "B"])
@pytest.mark.parametrize("dtype,tol", [(torch.float32, 2e-6), (torch.bfloat16, 1e-2)])
@pytest.mark.parametrize("case", CASES)
def test_skip_handoff_matches_autograd_sum(case, dtype, tol, consumer):
    from dalle2_video import ops

    nf, h, w, c, k, nup = case
    g = torch.Generator().manual_seed(nf * 1000 + h + c + k + nup)
    x = torch.randn(nf, h, w, c, generator=g)
    ys = [torch.randn(nf, h, w, c, generator=g) for _ in range(nup)]
    wa = torch.randn(c, c, 1, k, k, generator=g) / (c * k * k) ** 0.5
    wb = torch.randn(c, c, 1, k, k, generator=g) / (c * k * k) ** 0.5
    wu = [torch.randn(c, 2 * c, 1, k, k, generator=g) / (2 * c * k * k) ** 0.5 for _ in range(nup)]
    gs = [torch.randn(nf, h, w, c, generator=g) for _ in range(2 + nup)]

    # fp64 CPU reference of x's gradient (on the dtype-rounded operands)
    xr = x.to(dtype).double().requires_grad_()
    cv = lambda t, wt: F.conv2d(t.permute(0, 3, 1, 2), wt[:, :, 0].to(dtype).double(),
                                padding=k // 2).permute(0, 2, 3, 1)
    outs = [cv(xr, wa), cv(xr, wb)] + [cv(torch.cat([y.to(dtype).double(), xr], -1), wt)
                                       for y, wt in zip(ys, wu)]
    sum((o * gg.double()).sum() for o, gg in zip(outs, gs)).backward()

    dev = "cuda"
    grads = {}
    for tag, skip in (("plain", None), ("handoff", ops.SkipGrad())):
        xd = x.to(dev, dtype).requires_grad_()
        loss = _graph(ops, xd, [y.to(dev, dtype) for y in ys], wa.to(dev), wb.to(dev),
                      [t.to(dev) for t in wu], [t.to(dev) for t in gs], k, skip, consumer)
        loss.backward()
        grads[tag] = xd.grad
        if skip is not None:
            # every up-path gradient was handed over, and taken
            assert skip.n_parked == nup and skip.closed and not skip.parked
    assert rel(grads["plain"], xr.grad) < tol * 2
    assert rel(grads["handoff"], xr.grad) < tol * 2
    assert rel(grads["handoff"], grads["plain"]) < tol * 2


def test_skip_handoff_consumer_first_falls_back():
    """Consumer run before the parkers (not the unet's order): the hand-off
    closes empty and the late parkers return their gradients to autograd."""
    from dalle2_video import ops

    nf, h, w, c, k = 4, 16, 16, 64, 3
    g = torch.Generator().manual_seed(7)
    x = torch.randn(nf, h, w, c, generator=g)
    ys = [torch.randn(nf, h, w, c, generator=g) for _ in range(2)]
    wa, wb = (torch.randn(c, c, 1, k, k, generator=g) / (9 * c) ** 0.5 for _ in range(2))
    wu = [torch.randn(c, 2 * c, 1, k, k, generator=g) / (18 * c) ** 0.5 for _ in range(2)]
    gs = [torch.randn(nf, h, w, c, generator=g) for _ in range(4)]
    res = {}
    for tag, skip in (("plain", None), ("handoff", ops.SkipGrad())):
        xd = x.cuda().bfloat16().requires_grad_()
        loss = _graph(ops, xd, [y.cuda().bfloat16() for y in ys], wa.cuda(), wb.cuda(),
                      [t.cuda() for t in wu], [t.cuda() for t in gs], k, skip, "A", order_ok=False)
        loss.backward()
        res[tag] = xd.grad
        if skip is not None:
            assert skip.closed and skip.n_parked == 0
    assert rel(res["handoff"], res["plain"]) < 1e-6


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 2e-6), (torch.bfloat16, 1e-2)])
@pytest.mark.parametrize("nup", [1, 2, 3])
def test_space_to_depth_adds_parked_skips(dtype, tol, nup):
    """Downsample3D as the hidden's down-path reader: the depth-to-space
    backward adds the parked skip gradients (two in its kernel, a third by a
    fallback add)."""
    from dalle2_video import ops

    nf, H, W, c = 4, 32, 32, 64
    g = torch.Generator().manual_seed(11 + nup)
    x = torch.randn(nf, H, W, c, generator=g)
    ys = [torch.randn(nf, H, W, c, generator=g) for _ in range(nup)]
    wdn = torch.randn(128, 4 * c, 1, 1, 1, generator=g) / (4 * c) ** 0.5
    wu = [torch.randn(c, 2 * c, 1, 3, 3, generator=g) / (18 * c) ** 0.5 for _ in range(nup)]
    gd = torch.randn(nf, H // 2, W // 2, 128, generator=g)
    gu = [torch.randn(nf, H, W, c, generator=g) for _ in range(nup)]

    xr = x.to(dtype).double().requires_grad_()
    s2d = xr.reshape(nf, H // 2, 2, W // 2, 2, c).permute(0, 1, 3, 5, 2, 4).reshape(nf, H // 2, W // 2, 4 * c)
    ref = (torch.einsum("nhwk,ok->nhwo", s2d, wdn[:, :, 0, 0, 0].to(dtype).double()) * gd.double()).sum()
    for y, wt, gg in zip(ys, wu, gu):
        u = F.conv2d(torch.cat([y.to(dtype).double(), xr], -1).permute(0, 3, 1, 2),
                     wt[:, :, 0].to(dtype).double(), padding=1).permute(0, 2, 3, 1)
        ref = ref + (u * gg.double()).sum()
    ref.backward()

    grads = {}
    for tag, skip in (("plain", None), ("handoff", ops.SkipGrad())):
        xd = x.to("cuda", dtype).requires_grad_()
        d = ops.conv(ops.space_to_depth(xd, skip_in=skip), wdn.cuda())
        loss = (d.float() * gd.cuda()).sum()
        for y, wt, gg in zip(ys, wu, gu):
            u = ops.conv(y.to("cuda", dtype), wt.cuda(), x1=xd, skip_out=skip)
            loss = loss + (u.float() * gg.cuda()).sum()
        loss.backward()
        grads[tag] = xd.grad
        if skip is not None:
            assert skip.n_parked == nup and skip.closed and not skip.parked
    assert rel(grads["plain"], xr.grad) < tol * 2
    assert rel(grads["handoff"], xr.grad) < tol * 2
