"""Micro-benchmark of GroupNorm(+FiLM+SiLU) fwd/bwd at the Cfg2 shapes (bf16)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dalle2-video_amd"))
import torch  # noqa: E402

from dalle2_video import ops  # noqa: E402
from kbench import timeit  # noqa: E402


def case(nb, T, H, C):
    nf = nb * T
    z = torch.randn(nf, H, H, C, device="cuda", dtype=torch.bfloat16, requires_grad=True)
    g = torch.randn(C, device="cuda", requires_grad=True)
    b = torch.randn(C, device="cuda", requires_grad=True)
    ss = torch.randn(nb, 2 * C, device="cuda", requires_grad=True)
    y = ops.group_norm_act(z, g, b, nb, 8, 1e-5, scale_shift=ss)
    dy = torch.randn_like(y)
    fwd = lambda: ops.group_norm_act(z, g, b, nb, 8, 1e-5, scale_shift=ss)
    bwd = lambda: y.backward(dy, retain_graph=True)
    tf, tb = timeit(fwd), timeit(bwd)
    n = z.numel() * 2
    print(f"gn nb={nb} T={T} {H}x{H} C={C}: fwd {tf*1e3:7.1f} us ({3*n/tf/1e9:6.0f} GB/s alg) | "
          f"bwd {tb*1e3:7.1f} us ({5*n/tb/1e9:6.0f} GB/s alg)")


if __name__ == "__main__":
    for H, C in ((64, 64), (32, 64), (32, 128), (16, 128), (16, 256), (8, 256), (8, 512)):
        case(4, 16, H, C)
