"""HIP implicit-GEMM conv (fwd / dgrad / wgrad / bias-grad) vs torch fp32 CPU."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

CASES = [
    # nf, h, w, c0, c1, cout, k
    (2, 8, 8, 64, 0, 64, 3),
    (3, 5, 7, 16, 8, 40, 3),
    (4, 16, 16, 128, 64, 128, 3),
    (2, 8, 8, 8, 0, 32, 7),
    (1, 12, 12, 8, 0, 16, 15),
    (5, 4, 4, 256, 0, 512, 1),
    (2, 6, 6, 64, 0, 3, 1),
    (1, 33, 9, 32, 32, 96, 3),
    (3, 9, 11, 128, 64, 192, 3),    # glds path: dual source, ragged pixel and channel tiles
    (32, 64, 64, 64, 0, 64, 3),     # glds path: 256x64 tile (M >= 512 tiles)
    (2, 7, 5, 256, 0, 64, 3),       # wgrad 64x256 tile (K = 2304)
    (3, 4, 6, 24, 16, 32, 3),       # cout 32 < one 64-channel A tile, dual source
    # row-window wgrad (bf16, cin/cout % 64 == 0, W | 64): every window width
    (4, 32, 32, 64, 64, 64, 3),     # W=32, dual source (up-path skip concat)
    (2, 8, 8, 512, 256, 512, 3),    # W=8, 12 channel chunks x 3 tap rows, one split
    (8, 16, 16, 256, 0, 64, 1),     # 1x1 (Downsample3D-like), many splits
    (16, 8, 8, 64, 0, 128, 3),      # W=8, 2 cout tiles
    (2, 64, 64, 64, 64, 64, 3),     # window wgrad W=64: two 32-column blocks, dual source
    (2, 32, 64, 64, 0, 128, 3),     # window wgrad W=64, H=32 (non-square: 8 row blocks x 2 column blocks)
    (3, 32, 16, 64, 0, 64, 3),      # window wgrad W=16, H=32 (four 8-row stages per frame)
    (16, 32, 32, 128, 0, 64, 1),    # 1x1 stripe wgrad (res_conv-like), 2 channel chunks
    (8, 16, 16, 64, 64, 128, 1),    # 1x1 stripe wgrad, dual source
    # stripe forward / dgrad (64 input channels, W in {32, 64, 128})
    (8, 32, 32, 64, 0, 128, 3),     # W=32, 2 cout tiles (dgrad: 128 -> 64 implicit GEMM)
    (4, 64, 64, 64, 0, 64, 3),      # W=64, forward and dgrad both stripe
    (2, 128, 128, 64, 0, 64, 3),    # W=128 (config 5's 128x128 stage): one-row stages, late stage-2 rows
    (1, 128, 128, 64, 0, 128, 3),   # W=128, 2 cout tiles
    # dual-source 64 + 64 -> cout 3x3 forward as two stripe passes (64^2 up-path block1 convs)
    (1, 128, 128, 64, 64, 64, 3),   # W=128
    (2, 64, 64, 64, 64, 128, 3),    # W=64, 2 cout tiles
    # 8x8-frame forward / dgrad (H = W = 8, 16-channel chunks, two frames per block)
    (4, 8, 8, 48, 16, 64, 3),       # dual source at a 16-channel boundary, dgrad 64 -> 48 + 16
    (6, 8, 8, 128, 0, 192, 3),      # three channel blocks (no XCD regrouping), 8 chunks
    # window conv at the Cfg2 8x8 shapes and a 32-tile W=16 grid (32-channel tiles)
    (64, 8, 8, 512, 0, 256, 3),     # the Cfg2 8x8 512 -> 256 shape
    (64, 8, 8, 512, 0, 512, 3),     # Cfg2 8x8 512 -> 512: 256 tiles
    (16, 16, 16, 64, 64, 64, 3),    # W=16, dual source, 32 tiles
    # 1x1 streaming kernel (K = 64 / 128, cout = 64 / 128): ragged / tiny / persistent
    (3, 9, 11, 64, 64, 64, 1),      # dual source, 297 pixels (ragged last tile)
    (2, 6, 6, 64, 0, 128, 1),       # fewer pixels than one tile
    (64, 64, 64, 64, 64, 64, 1),    # the 64x64 up-path res_conv: 2,048 tiles over persistent workgroups
    # small-channel direct forward (bf16, cin <= 16, cout <= 32, w % 32 == 0: dv_conv_small_fwd)
    (2, 8, 64, 8, 0, 8, 3),         # the 256x256 unet's dim-8 Block3D conv
    (2, 5, 32, 8, 8, 8, 3),         # up-path skip concat 8 + 8 (CP 16), 5 rows < one 8-row band
    (1, 9, 96, 8, 8, 16, 3),        # concat 8 + 8 -> 16, 96 = 3 x 32-column blocks
    (2, 4, 64, 16, 0, 8, 1),        # 1x1 16 -> 8
    (1, 6, 32, 16, 0, 24, 7),       # cin 16 (CP 16), second output tile half padded
    (2, 8, 64, 8, 0, 8, 15),        # 15x15 window
]


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 2e-6), (torch.bfloat16, 1.5e-2)])
@pytest.mark.parametrize("case", CASES)
def test_conv_fwd_bwd(case, dtype, tol):
    from dalle2_video import ops

    nf, h, w, c0, c1, cout, k = case
    g = torch.Generator().manual_seed(hash(case) % 1000)
    cin = c0 + c1
    x = torch.randn(nf, h, w, cin, generator=g)
    wt = torch.randn(cout, cin, 1, k, k, generator=g) / (cin * k * k) ** 0.5
    b = torch.randn(cout, generator=g)
    res = torch.randn(nf, h, w, cout, generator=g)
    gy = torch.randn(nf, h, w, cout, generator=g)
    # reference in fp64 on the (bf16-rounded) inputs: long pixel reductions
    # (wgrad / bias grad over 131k pixels) would otherwise measure the CPU's error
    xr = x.to(dtype).double().clone().requires_grad_()
    wr = wt.to(dtype).double().requires_grad_()
    br = b.double().requires_grad_()
    yr = F.conv2d(xr.permute(0, 3, 1, 2), wr[:, :, 0], br, padding=k // 2).permute(0, 2, 3, 1)
    yr = yr + res.to(dtype).double()
    (yr * gy.double()).sum().backward()

    dev = "cuda"
    xd = x.detach().to(dev, dtype)
    x0 = xd[..., :c0].clone().requires_grad_() if c1 else xd.clone().requires_grad_()
    x1 = xd[..., c0:].clone().requires_grad_() if c1 else None
    wd = wt.to(dev).requires_grad_()
    bd = b.to(dev).requires_grad_()
    y = ops.conv(x0, wd, bd, x1=x1, res=res.to(dev, dtype))
    assert rel(y.float(), yr) < tol
    (y.float() * gy.to(dev)).sum().backward()
    dx = torch.cat([x0.grad] + ([x1.grad] if c1 else []), dim=-1)
    assert rel(dx.float(), xr.grad) < tol * 2
    assert rel(wd.grad, wr.grad) < tol * 2
    assert rel(bd.grad, br.grad) < tol


@pytest.mark.parametrize("dtype,tol", [(torch.float32, 2e-6), (torch.bfloat16, 1.5e-2)])
def test_linear_weight_as_1x1_conv(dtype, tol):
    """nn.Linear weights (cout, cin) run as 1x1 convs over tokens (mid attention)."""
    from dalle2_video import ops

    g = torch.Generator().manual_seed(2)
    x = torch.randn(4, 4, 4, 512, generator=g)
    w = torch.randn(64, 512, generator=g) / 512 ** 0.5
    xr, wr = x.to(dtype).float().clone().requires_grad_(), w.clone().requires_grad_()
    yr = xr @ wr.t()
    gy = torch.randn(yr.shape, generator=g)
    (yr * gy).sum().backward()
    xd = x.detach().to("cuda", dtype).requires_grad_()
    wd = w.detach().cuda().requires_grad_()
    y = ops.conv(xd, wd)
    assert rel(y.float(), yr) < tol
    (y.float() * gy.cuda()).sum().backward()
    assert rel(xd.grad.float(), xr.grad) < tol * 2
    assert rel(wd.grad, wr.grad) < tol * 2


@pytest.mark.parametrize("case", [(32, 64, 64, 64, 0, 64, 3), (16, 32, 32, 128, 0, 128, 3),
                                  (64, 8, 8, 512, 0, 512, 3), (64, 64, 64, 64, 64, 64, 1)])
def test_stripe_wgrad_bf16_partials(case, parity_log):
    """The row-window wgrad's split-K partials are stored in bf16 and summed
    in f32 (half the partial bytes).  Rounding each of S partials is an error
    of the order of ONE bf16 rounding of the gradient (random-sign partials:
    rms 2^-8/sqrt(12) relative, whatever S) -- the rounding the reference's
    autocast gradient itself carries (its conv weight gradient is a bf16
    tensor cast to f32).  Checked against fp64 on the same bf16 x and dY."""
    from dalle2_video import ops

    nf, h, w, c0, c1, cout, k = case
    g = torch.Generator().manual_seed(7)
    cin = c0 + c1
    x = torch.randn(nf, h, w, cin, generator=g).bfloat16()
    wt = torch.randn(cout, cin, 1, k, k, generator=g) / (cin * k * k) ** 0.5
    gy = torch.randn(nf, h, w, cout, generator=g).bfloat16()
    xr = x.double()
    wr = wt.bfloat16().double().requires_grad_()
    yr = F.conv2d(xr.permute(0, 3, 1, 2), wr[:, :, 0], padding=k // 2).permute(0, 2, 3, 1)
    (yr * gy.double()).sum().backward()
    xd = x.cuda()
    x0 = xd[..., :c0].contiguous() if c1 else xd
    x1 = xd[..., c0:].contiguous() if c1 else None
    wd = wt.cuda().requires_grad_()
    y = ops.conv(x0, wd, None, x1=x1)
    y.backward(gy.cuda())
    err = rel(wd.grad, wr.grad)
    parity_log(config=f"stripe wgrad bf16 partials {case}", dw_rel=err)
    # one bf16 rounding is 2^-9 relative at most, 1.1e-3 rms
    assert err < 2.5e-3, err


@pytest.mark.parametrize("case", [(64, 16, 16, 64, 64), (64, 8, 8, 128, 128), (64, 64, 64, 64, 64),
                                  (64, 32, 32, 128, 128)])
def test_window_wgrad_repeatable(case):
    """The row-window 3x3 wgrad (split-K partials + one ordered sum) has no
    atomics: repeated launches on the same inputs must give the same bits.
    Guards the race fixed in round 6 -- a wave that finished its last stage
    early wrote the halves-sum scratch over the ring while another wave still
    read its operands (a rare wrong split partial, seen as an occasional
    non-finite gradient at the 16^2 / 8^2 up-path convs)."""
    from dalle2_video import _lib, ops

    nf, h, w, cin, cout = case
    g = torch.Generator().manual_seed(3)
    x = torch.randn(nf, h, w, cin, generator=g).bfloat16().cuda()
    dy = torch.randn(nf, h, w, cout, generator=g).bfloat16().cuda()
    ws = ops._wgrad_workspace("bf16", nf, h, w, cin, cin, False, cout, 3, x.device)
    dw = torch.empty(cout, cin, 1, 3, 3, device="cuda")
    db = torch.empty(cout, device="cuda")

    def run():
        _lib.call("dv_conv_wgrad", _lib.DV_BF16, _lib.ptr(dy), cout, _lib.ptr(x), cin, cin, None, 0,
                  _lib.ptr(dw), 0, _lib.ptr(db), 0, _lib.ptr(ws), ws.numel(), nf, h, w, cin, cout, cout, cin, 3,
                  _lib.stream())

    run()
    w0, b0 = dw.clone(), db.clone()
    assert torch.isfinite(w0).all()
    n = 2000  # launches back to back, each result kept on the device and compared at the end
    outs = torch.empty(n, dw.numel() + db.numel(), device="cuda")
    for i in range(n):
        run()
        outs[i, :dw.numel()].copy_(dw.reshape(-1))
        outs[i, dw.numel():].copy_(db)
    ref = torch.cat([w0.reshape(-1), b0])
    diff = int((outs != ref).any(dim=1).sum())
    assert diff == 0, f"{diff} of {n} launches differ"


def test_batched_repack_matches_single_packs():
    """PackCache.refresh (one flat-tile launch over every cached image) writes the
    same bytes as packing each weight alone, for both layouts and both dtypes,
    a row-tiled 1x1 / 3x3 mix and an entry larger than the rest."""
    from dalle2_video import ops
    shapes = [(64, 64, 3), (512, 768, 3), (3, 64, 3), (128, 256, 1), (40, 24, 3), (256, 256, 1), (16, 8, 15)]
    cache = ops.PackCache()
    cache.enabled = True
    g = torch.Generator(device="cuda").manual_seed(3)
    wts, imgs = [], []
    for co, ci, k in shapes:
        w = torch.randn(co, ci, 1, k, k, device="cuda", generator=g)
        wts.append(w)
        for dtype in (torch.bfloat16, torch.float32):
            for mode in (0, 1, 2, 3):
                if k == 15 and mode >= 2:
                    continue
                pad = ((ci if mode % 2 == 0 else co) + 15) // 16 * 16
                out, stale = cache.lookup(w, w, dtype, co, ci, k, pad, mode)
                assert stale
                imgs.append((w, dtype, pad, mode, out))
    for w in wts:  # new weights, then one batched repack
        w.copy_(torch.randn(w.shape, device="cuda", generator=g))
    cache.refresh()
    torch.cuda.synchronize()
    for w, dtype, pad, mode, out in imgs:
        ref = ops.pack_conv_weight(w, dtype, pad, mode, cache=False)
        assert torch.equal(out.view(torch.int16) if dtype == torch.bfloat16 else out.view(torch.int32),
                           ref.view(torch.int16) if dtype == torch.bfloat16 else ref.view(torch.int32)), \
            (tuple(w.shape), dtype, mode)


def test_paired_repack_matches_single_packs():
    """The bf16 3x3 weights whose cache holds exactly one forward and one dgrad
    image are repacked by dv_pack_conv_weight_pairs (one read of the weight for
    both images); every (forward, dgrad) mode combination, beside a weight the
    pairing rejects (cout % 64 != 0), writes the same bytes as single packs."""
    from dalle2_video import ops
    # (the last pair: a weight 4 B past a 16-B boundary, a view into a flat buffer --
    # the tile loads fall back from 16-B to dword pieces)
    cases = [((64, 64, 3), 2, 3, 0), ((512, 768, 3), 2, 3, 0), ((128, 48, 3), 0, 1, 0), ((64, 16, 3), 0, 3, 0),
             ((192, 64, 3), 2, 1, 0), ((40, 24, 3), 0, 1, 0), ((128, 32, 3), 2, 3, 1)]
    cache = ops.PackCache()
    cache.enabled = True
    g = torch.Generator(device="cuda").manual_seed(5)
    imgs = []
    for (co, ci, k), mf, md, off in cases:
        flat = torch.randn(off + co * ci * k * k, device="cuda", generator=g)
        w = flat[off:].view(co, ci, 1, k, k)
        for mode in (mf, md):
            pad = ci if mode % 2 == 0 else co
            out, stale = cache.lookup(w, w, torch.bfloat16, co, ci, k, pad, mode)
            assert stale
            imgs.append((w, pad, mode, out))
    pairs, rest = cache._pair(list(cache.entries.values()))
    assert len(pairs) == 6 and len(rest) == 2
    for w, _, _, _ in imgs:
        w.copy_(torch.randn(w.shape, device="cuda", generator=g))
    cache.refresh()
    torch.cuda.synchronize()
    for w, pad, mode, out in imgs:
        ref = ops.pack_conv_weight(w, torch.bfloat16, pad, mode, cache=False)
        assert torch.equal(out.view(torch.int16), ref.view(torch.int16)), (tuple(w.shape), mode)
