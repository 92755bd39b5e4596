"""MX-fp8 PV mid attention (dv_mqa_fwd_fp8, BASELINE config 5 sampling): the
K/V-streamed forward with P and V in e4m3 (an e8m0 scale per 32 keys) on
v_mfma_scale_f32_32x32x64_f8f6f4, QK^T in bf16.  Checked against an f32
reference of the same attention (dalle2-pytorch Attention as the oracle
restates it: null key/value at key 0, logit factor 1/dim_head, reference
dalle2_video.py:431, 551, 921-922) on a subset of query rows, and against the
bf16 streamed kernel over every row.  fp8 tolerance: 6e-2 relative (e4m3 keeps
3 mantissa bits: ~3.6 % RMS rounding per element on P and on V; measured 3.7-4.1e-2)."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def rel(a, b):
    a, b = a.double(), b.double()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def reference_rows(q, kv, null_kv, B, N, H, scale, rows):
    out = []
    for b in range(B):
        qb = q[b * N:(b + 1) * N].float().view(N, H, 32)[rows]  # (r, H, 32)
        k = torch.cat([null_kv[0:1].float(), kv[b * N:(b + 1) * N, :32].float()])
        v = torch.cat([null_kv[1:2].float(), kv[b * N:(b + 1) * N, 32:].float()])
        s = torch.einsum("rhd,jd->rhj", qb, k) * scale
        out.append(torch.einsum("rhj,jd->rhd", s.softmax(-1), v).reshape(len(rows), H * 32))
    return torch.cat(out)


@pytest.mark.parametrize("N", [8192, 2000])  # config 5's 8,193 keys; 2,016 keys: an odd tile count in the last chunk
@pytest.mark.parametrize("qmag", [1.0, 8.0])  # diffuse / peaked attention
def test_mqa_fp8_pv_matches_reference(N, qmag):
    from dalle2_video import ops

    B, H = 2, 16
    scale = 1.0 / 32
    g = torch.Generator(device="cuda").manual_seed(N + int(qmag))
    q = (torch.randn(B * N, H * 32, device="cuda", generator=g) * qmag).bfloat16()
    kv = torch.randn(B * N, 64, device="cuda", generator=g).bfloat16()
    null_kv = torch.randn(2, 32, device="cuda", generator=g)
    with torch.no_grad():
        o16 = ops.mqa(q, kv, null_kv, B, N, H, scale)
        ops.TIMER = ops.KernelTimer()
        try:
            with ops.mx8_convs(attention=True):
                o8 = ops.mqa(q, kv, null_kv, B, N, H, scale)
            names = set(ops.TIMER.summary())
        finally:
            ops.TIMER = None
    assert "attn:mqa_fwd8" in names, names  # the fp8 kernel ran, not the bf16 one
    assert torch.isfinite(o8.float()).all()
    rows = torch.arange(0, N, max(1, N // 256), device="cuda")[:256]
    ref = reference_rows(q, kv, null_kv, B, N, H, scale, rows)
    sel = torch.cat([b * N + rows for b in range(B)])
    e8, e16 = rel(o8[sel].float(), ref), rel(o16[sel].float(), ref)
    print(f"N={N} qmag={qmag}: fp8 rel {e8:.3e}, bf16 rel {e16:.3e}, fp8 vs bf16 (all rows) {rel(o8.float(), o16.float()):.3e}")
    assert e16 < 1e-2
    assert e8 < 6e-2
    assert rel(o8.float(), o16.float()) < 6e-2


def test_mqa_fp8_not_taken_with_grad_or_short_clips():
    """Training (autograd) and the whole-clip-in-LDS kernel (NKP <= 1280) stay
    on the bf16 path inside mx8_convs(attention=True); without attention=True
    (the default fp8 sampling mode) every clip length stays bf16."""
    from dalle2_video import ops

    B, H = 1, 16
    for N, grad, att in ((1024, False, True), (4096, True, True), (4096, False, False)):
        q = torch.randn(B * N, H * 32, device="cuda").bfloat16().requires_grad_(grad)
        kv = torch.randn(B * N, 64, device="cuda").bfloat16()
        null_kv = torch.randn(2, 32, device="cuda")
        ops.TIMER = ops.KernelTimer()
        try:
            with ops.mx8_convs(attention=att), torch.set_grad_enabled(grad):
                ops.mqa(q, kv, null_kv, B, N, H, 1.0 / 32)
            names = set(ops.TIMER.summary())
        finally:
            ops.TIMER = None
        assert "attn:mqa_fwd8" not in names, (N, grad, names)
