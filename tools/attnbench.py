"""Mid-attention (MQA) micro-benchmark at the Cfg2 shape (B=4, N=1024 tokens,
16 heads x 32, 1,025 keys): fwd and bwd through ops.mqa; run under
rocprofv3 --kernel-trace --stats for the per-kernel split."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dalle2-video_amd"))
import torch  # noqa: E402

from dalle2_video import ops  # noqa: E402

B, N, H, D = 4, 1024, 16, 32
g = torch.Generator(device="cuda").manual_seed(0)
q = torch.randn(B * N, H * D, device="cuda", generator=g).bfloat16().requires_grad_()
kv = torch.randn(B * N, 2 * D, device="cuda", generator=g).bfloat16().requires_grad_()
nkv = torch.randn(2, D, device="cuda", generator=g).requires_grad_()
gy = torch.randn(B * N, H * D, device="cuda", generator=g).bfloat16()
flop = 4.0 * B * H * N * (N + 1) * D


def step():
    y = ops.mqa(q, kv, nkv, B, N, H, 1.0 / D)
    y.backward(gy)


for _ in range(3):
    step()
torch.cuda.synchronize()
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
it = 20
s.record()
for _ in range(it):
    y = ops.mqa(q, kv, nkv, B, N, H, 1.0 / D)
e.record()
torch.cuda.synchronize()
fms = s.elapsed_time(e) / it
s.record()
for _ in range(it):
    step()
e.record()
torch.cuda.synchronize()
ams = s.elapsed_time(e) / it
print(f"mqa fwd {fms * 1e3:.1f} us ({flop / fms / 1e9:.0f} TF/s)  fwd+bwd {ams * 1e3:.1f} us "
      f"({3 * flop / ams / 1e9:.0f} TF/s, {3 * flop / ams / 1e9 / 2516.6:.3f} of bf16 peak)")
