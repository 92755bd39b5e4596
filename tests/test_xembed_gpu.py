"""Direct CrossEmbedLayer3D kernels (dv_cross_embed_fwd / _wgrad) against a
torch f32 reference of the reference layer (dalle2_video.py:208-244: one
Conv3d (1,k,k) per kernel size, outputs concatenated along channels) on the
same bf16-rounded inputs and weights.

Tolerances: forward — f32 accumulation, one bf16 rounding of the output:
rel 1e-2 of the output norm, max-abs 2 bf16 ulps of the largest output;
gradients — exact bf16 products, f32 sums in another order: rel 1e-4."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _ref(x_cl, weights, biases):
    xs = x_cl.float().permute(0, 3, 1, 2)  # (nf, C, h, w)
    outs = []
    for w, b in zip(weights, biases):
        k = w.shape[-1]
        wb = w[:, :, 0].to(torch.bfloat16).float()
        outs.append(F.conv2d(xs[:, :w.shape[1]], wb, b, padding=k // 2))
    return torch.cat(outs, 1).permute(0, 2, 3, 1)


CASES = [
    # nf, h, w, cin, ld, (k, cout) per branch
    (64, 64, 64, 3, 8, ((3, 32), (7, 16), (15, 16))),   # Cfg2 unet1 init_conv (dim 64)
    (8, 32, 32, 3, 8, ((3, 8), (7, 4), (15, 4))),       # Cfg1 (dim 16)
    (4, 64, 128, 6, 8, ((3, 16), (7, 8), (15, 8))),     # upsampler unet: video + lowres cond (CP 8)
    (2, 16, 32, 3, 4, ((3, 64), (7, 32), (15, 32))),    # dim 128, 4-channel pixel stride
    (4, 16, 256, 6, 8, ((3, 4), (7, 2), (15, 2))),      # Cfg4 unet2 (dim 8): one zero-padded tile
    (2, 8, 64, 3, 4, ((3, 16), (7, 8))),                # 24 channels: second tile half padded
]


@pytest.mark.parametrize("nf,h,w,cin,ld,branches", CASES)
def test_cross_embed_forward_and_grads_vs_torch(nf, h, w, cin, ld, branches, parity_log):
    from dalle2_video import ops

    g = torch.Generator(device="cuda").manual_seed(nf * h + cin)
    x = torch.randn(nf, h, w, ld, device="cuda", generator=g).bfloat16()
    x[..., cin:] = 7.0  # padding channels must be ignored
    weights = [(torch.randn(co, cin, 1, k, k, device="cuda", generator=g) / (cin * k * k) ** 0.5).requires_grad_()
               for k, co in branches]
    biases = [torch.randn(co, device="cuda", generator=g).requires_grad_() for _, co in branches]
    assert ops.cross_embed_ok(x, weights)
    y = ops.cross_embed(x, weights, biases)
    ref = _ref(x, weights, [b.detach() for b in biases])
    err = ((y.float() - ref).norm() / ref.norm()).item()
    mx = (y.float() - ref).abs().max().item()
    tol_mx = 2 * 2.0 ** -7 * ref.abs().max().item()
    dy = torch.randn(y.shape, device="cuda", generator=g).bfloat16()
    y.backward(dy)
    # reference gradients from the same bf16 values (f32 math)
    xs = x.float().permute(0, 3, 1, 2)[:, :cin]
    dys = dy.float().permute(0, 3, 1, 2)
    gw_err, gb_err = [], []
    c0 = 0
    for (k, co), wt, bt in zip(branches, weights, biases):
        d = dys[:, c0:c0 + co]
        gw = torch.nn.grad.conv2d_weight(xs, (co, cin, k, k), d, padding=k // 2)
        gb = d.sum((0, 2, 3))
        gw_err.append(((wt.grad[:, :, 0] - gw).norm() / gw.norm()).item())
        gb_err.append(((bt.grad - gb).norm() / gb.norm()).item())
        c0 += co
    parity_log(op="cross_embed", shape=[nf, h, w, cin], fwd_rel=err, fwd_maxabs=mx, dw_rel=max(gw_err),
               db_rel=max(gb_err))
    assert err < 1e-2 and mx <= tol_mx, (err, mx, tol_mx)
    assert max(gw_err) < 1e-4, gw_err
    assert max(gb_err) < 1e-4, gb_err


def test_cross_embed_accumulates_and_matches_padded_conv():
    """A second backward adds into .grad; the direct path equals the padded
    implicit-GEMM conv (the f32 / fallback path) on the same layer."""
    from dalle2_video import dalle2_video as D, ops

    torch.manual_seed(0)
    layer = D.CrossEmbedLayer3D(3, (3, 7, 15), dim_out=64, stride=1).cuda()
    x = torch.randn(16, 32, 32, 8, device="cuda").bfloat16()
    y = layer.forward_cl(x)
    weights = [c.weight for c in layer.convs]
    kmax = 15
    wpad = torch.cat([F.pad(w, [(kmax - w.shape[-1]) // 2] * 4) for w in weights], 0)
    bcat = torch.cat([c.bias for c in layer.convs])
    y2 = ops.conv(x, wpad.detach(), bcat.detach(), cache=False)
    assert ((y.float() - y2.float()).norm() / y2.float().norm()).item() < 1e-2
    dy = torch.randn_like(y)
    y.backward(dy)
    g1 = [c.weight.grad.clone() for c in layer.convs]
    layer.forward_cl(x).backward(dy)
    for c, a in zip(layer.convs, g1):
        assert ((c.weight.grad - 2 * a).norm() / a.norm()).item() < 1e-5
