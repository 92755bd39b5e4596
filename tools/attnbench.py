"""Mid-attention (MQA) micro-benchmark through ops.mqa:
  Cfg2 shape (B=4, N=1024 tokens, 16 heads x 32, 1,025 keys): fwd and fwd+bwd
  config-5 shape (B=2, N=8192 tokens, 8,193 keys): fwd (streamed K / V)
Each line also carries the rel-err against a torch f32 reference of the same
bf16 operands.  Run under rocprofv3 --kernel-trace --stats for the per-kernel
split; DV_HIP_LIB=<other build> for an A/B on the same box."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dalle2-video_amd"))
import torch  # noqa: E402

from dalle2_video import ops  # noqa: E402

PEAK = 2516.6
D = 32


def reference(q, kv, nkv, B, N, H):
    qf = q.float().reshape(B, N, H, D)
    k = torch.cat((nkv[0].float().expand(B, 1, D), kv[:, :D].float().reshape(B, N, D)), 1)
    v = torch.cat((nkv[1].float().expand(B, 1, D), kv[:, D:].float().reshape(B, N, D)), 1)
    out = torch.empty(B, N, H, D, device=q.device)
    for b in range(B):
        for s in range(0, N, 1024):
            p = torch.softmax(qf[b, s:s + 1024].reshape(-1, D) @ k[b].t() / D, -1)
            out[b, s:s + 1024] = (p @ v[b]).reshape(-1, H, D)
    return out.reshape(B * N, H * D)


def timed(fn, it):
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it


def case(B, N, H, bwd, it):
    g = torch.Generator(device="cuda").manual_seed(0)
    q = (2 * torch.randn(B * N, H * D, device="cuda", generator=g)).bfloat16().requires_grad_()
    kv = (2 * torch.randn(B * N, 2 * D, device="cuda", generator=g)).bfloat16().requires_grad_()
    nkv = torch.randn(2, D, device="cuda", generator=g).requires_grad_()
    gy = torch.randn(B * N, H * D, device="cuda", generator=g).bfloat16()
    flop = 4.0 * B * H * N * (N + 1) * D
    with torch.no_grad():
        o = ops.mqa(q, kv, nkv, B, N, H, 1.0 / D).float()
        ref = reference(q, kv, nkv, B, N, H)
        err = ((o - ref).norm() / ref.norm()).item()
        bad = ~torch.isfinite(o)
        if bad.any():
            rows = bad.reshape(B * N * H, D).any(-1).nonzero().flatten()
            print(f"  non-finite: {bad.sum().item()} values in {rows.numel()} of {B * N * H} rows; "
                  f"first rows {rows[:8].tolist()}; row % 256 histogram "
                  f"{torch.bincount((rows % 256) // 32, minlength=8).tolist()}", flush=True)

    def fwd():
        with torch.no_grad():
            ops.mqa(q, kv, nkv, B, N, H, 1.0 / D)

    def step():
        y = ops.mqa(q, kv, nkv, B, N, H, 1.0 / D)
        y.backward(gy)

    for _ in range(3):
        (step if bwd else fwd)()
    torch.cuda.synchronize()
    fms = timed(fwd, it)
    line = f"B={B} N={N}: fwd {fms * 1e3:.1f} us ({flop / fms / 1e9:.0f} TF/s, {flop / fms / 1e9 / PEAK:.3f})"
    if bwd:
        ams = timed(step, it)
        line += (f"  fwd+bwd {ams * 1e3:.1f} us ({3 * flop / ams / 1e9:.0f} TF/s, "
                 f"{3 * flop / ams / 1e9 / PEAK:.3f} of bf16 peak)")
    print(line + f"  fwd rel-err {err:.2e}", flush=True)


if __name__ == "__main__":
    case(4, 1024, 16, True, 20)
    if "--short" not in sys.argv:
        case(2, 8192, 16, False, 5)
