"""GroupNorm folded into the next conv's input staging (round 6): ResnetBlock3D's
block1 GroupNorm + FiLM + SiLU (reference dalle2_video.py:99-133, 183-205)
is not run as its own apply pass when block1's output feeds block2's conv
alone; the stripe kernel stages z and applies silu(A z + B) to each window row
in LDS (dv_conv_fwd_gn_in), writing y for block2's weight gradient and the
GroupNorm's saved mean / rstd.

  * a 64-channel ResnetBlock3D at 64^2 (bf16, 2 clips x 4 frames), forward
    and backward, fold on (ops.GN_FOLD) vs off: the same arithmetic except the
    order in which the GroupNorm sums are combined, so outputs and every
    gradient agree to bf16 rounding flips (<= 5e-3 relative); the folded launch
    must have run
  * the folded block vs a torch f32 restatement (F.conv3d / F.group_norm on
    the same bf16 weights and input) within the bf16 tolerance of
    tests/test_cfg2_gpu.py (2.5e-2)
  * no-grad (sampling: y not stored) matches the training forward (to the
    run-to-run order of the statistics atomics: flips only)
  * several blocks in a row (the rotating sums buffers, ops._GnSums: the
    folded conv takes over the deferred GroupNorm's zeroing) match fold off
  * an up-path block (64 + 64 skip channels in): block1's dual-source conv
    accumulates the statistics in its second pass, so its GroupNorm folds too
"""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def _block(seed=0, nblocks=1, dim=64):
    from dalle2_video.dalle2_video import ResnetBlock3D
    torch.manual_seed(seed)
    blocks = [ResnetBlock3D(dim, 64, time_cond_dim=128) for _ in range(nblocks)]
    for b in blocks:
        for p in b.parameters():  # non-trivial norms / FiLM (default init is 1 / 0)
            p.data.add_(0.05 * torch.randn_like(p))
    return [b.cuda() for b in blocks]


def _run(blocks, x, te, fold, grad=True, calls=None, x1=None):
    from dalle2_video import ops
    ops.GN_FOLD = fold
    orig = ops.call

    def rec(name, *a):
        if calls is not None:
            calls.append(name)
        return orig(name, *a)

    ops.call = rec
    try:
        for b in blocks:
            for p in b.parameters():
                p.grad = None
        xd = x.clone().requires_grad_(grad)
        x1d = None if x1 is None else x1.clone().requires_grad_(grad)
        with torch.set_grad_enabled(grad):
            h = xd
            for b in blocks:
                h = b.forward_cl(h, te, None, 2, x1=x1d)
            out = {"y": h.detach().float().clone()}
            if grad:
                g = torch.Generator(device="cuda").manual_seed(7)
                (h.float() * torch.randn(h.shape, device="cuda", generator=g)).sum().backward()
                out["dx"] = xd.grad.float()
                if x1d is not None:
                    out["dx1"] = x1d.grad.float()
                for i, b in enumerate(blocks):
                    for n, p in b.named_parameters():
                        if p.grad is not None:
                            out[f"{i}.{n}"] = p.grad.float().clone()
        torch.cuda.synchronize()
        return out
    finally:
        ops.call = orig
        ops.GN_FOLD = True


def _inputs(seed=1):
    g = torch.Generator().manual_seed(seed)
    x = torch.randn(8, 64, 64, 64, generator=g).bfloat16().cuda()
    te = torch.randn(2, 128, generator=g).cuda()
    return x, te


def test_fold_matches_unfolded_block():
    (blk,) = _block()
    x, te = _inputs()
    calls = []
    a = _run([blk], x, te, True, calls=calls)
    b = _run([blk], x, te, False)
    assert "dv_conv_fwd_gn_in" in calls, "the folded conv did not run"
    assert set(a) == set(b)
    for k in a:
        r = rel(a[k], b[k])
        assert r <= 5e-3, f"{k}: fold vs unfolded rel {r:.2e}"


def test_fold_vs_torch_f32():
    (blk,) = _block(seed=3)
    x, te = _inputs(seed=4)
    got = _run([blk], x, te, True)["y"]
    # f32 restatement of ResnetBlock3D (dalle2_video.py:136-205) on the same values
    xf = x.float()
    xc = xf.reshape(2, 4, 64, 64, 64).permute(0, 4, 1, 2, 3)  # (b, c, t, h, w)
    ss = blk.time_mlp(te)
    scale, shift = ss.chunk(2, dim=1)

    def block(m, v, sc=None):
        v = F.conv3d(v, m.project.weight.float(), m.project.bias.float(), padding=(0, 1, 1))
        v = F.group_norm(v, 8, m.norm.weight.float(), m.norm.bias.float(), 1e-5)
        if sc is not None:
            v = v * (sc[0][:, :, None, None, None] + 1) + sc[1][:, :, None, None, None]
        return F.silu(v)

    h = block(blk.block1, xc, (scale, shift))
    ref = block(blk.block2, h) + xc
    ref = ref.permute(0, 2, 3, 4, 1).reshape(8, 64, 64, 64)
    r = rel(got, ref)
    assert r <= 2.5e-2, f"folded block vs torch f32 rel {r:.2e}"


def test_fold_no_grad_equals_training_forward():
    (blk,) = _block(seed=5)
    x, te = _inputs(seed=6)
    a = _run([blk], x, te, True)["y"]
    calls = []
    b = _run([blk], x, te, True, grad=False, calls=calls)["y"]
    assert "dv_conv_fwd_gn_in" in calls
    r = rel(b, a)
    assert r <= 5e-3, f"no-grad vs training forward rel {r:.2e}"


def test_fold_chain_of_blocks():
    blocks = _block(seed=8, nblocks=3)
    x, te = _inputs(seed=9)
    a = _run(blocks, x, te, True)
    b = _run(blocks, x, te, False)
    for k in a:
        r = rel(a[k], b[k])
        assert r <= 5e-3, f"{k}: fold vs unfolded rel {r:.2e}"


def test_fold_dual_source_block():
    (blk,) = _block(seed=10, dim=128)
    x, te = _inputs(seed=11)
    x1, _ = _inputs(seed=12)
    calls = []
    a = _run([blk], x, te, True, calls=calls, x1=x1)
    b = _run([blk], x, te, False, x1=x1)
    assert calls.count("dv_conv_fwd_gn_in") == 1, calls
    for k in a:
        r = rel(a[k], b[k])
        assert r <= 5e-3, f"{k}: fold vs unfolded rel {r:.2e}"
    # against torch f32 (dalle2_video.py:136-205 with a concatenated skip)
    xc = torch.cat([x.float(), x1.float()], -1).reshape(2, 4, 64, 64, 128).permute(0, 4, 1, 2, 3)
    scale, shift = blk.time_mlp(te).chunk(2, dim=1)

    def block(m, v, sc=None):
        v = F.conv3d(v, m.project.weight.float(), m.project.bias.float(), padding=(0, 1, 1))
        v = F.group_norm(v, 8, m.norm.weight.float(), m.norm.bias.float(), 1e-5)
        if sc is not None:
            v = v * (sc[0][:, :, None, None, None] + 1) + sc[1][:, :, None, None, None]
        return F.silu(v)

    ref = block(blk.block2, block(blk.block1, xc, (scale, shift))) + F.conv3d(
        xc, blk.res_conv.weight.float(), blk.res_conv.bias.float())
    ref = ref.permute(0, 2, 3, 4, 1).reshape(8, 64, 64, 64)
    r = rel(a["y"], ref)
    assert r <= 2.5e-2, f"folded up-path block vs torch f32 rel {r:.2e}"


def test_deferred_output_materialises_for_other_consumers():
    """A deferred GroupNorm output read by a conv that cannot fold it (here a
    1x1 conv) gets the plain apply first: same values as the two-pass form."""
    from dalle2_video import ops
    g = torch.Generator().manual_seed(13)
    nb, C = 2, 64
    x = torch.randn(8, 64, 64, C, generator=g).bfloat16().cuda()
    w1 = (0.05 * torch.randn(C, C, 1, 3, 3, generator=g)).cuda()
    gamma = (1 + 0.1 * torch.randn(C, generator=g)).cuda()
    beta = (0.1 * torch.randn(C, generator=g)).cuda()
    ss = (0.2 * torch.randn(nb, 2 * C, generator=g)).cuda()
    w2 = (0.05 * torch.randn(C, C, 1, 1, 1, generator=g)).cuda()
    outs = []
    for defer in (True, False):
        with torch.no_grad():
            st = ops.gn_stats(nb, C, 4 * 64 * 64, x.device)
            z = ops.conv(x, w1, None, gn=st)
            y = ops.group_norm_act(z, gamma, beta, nb, 8, 1e-5, scale_shift=ss, stats=st, defer=defer)
            assert (getattr(y, "_dv_gn_in", None) is not None) == (defer and st.used)
            outs.append(ops.conv(y, w2).float())
            outs.append(y.float())
    torch.cuda.synchronize()
    assert rel(outs[0], outs[2]) <= 5e-3 and rel(outs[1], outs[3]) <= 5e-3
