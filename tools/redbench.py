"""Micro-benchmark: split-partial reduction (S x N f32) strategies on the GPU."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dalle2-video_amd"))
import torch  # noqa: E402

from kbench import timeit  # noqa: E402

for S, N in ((256, 36864), (128, 73728), (4, 2359296)):
    part = torch.randn(S, N, device="cuda")
    out = torch.empty(N, device="cuda")
    t_sum = timeit(lambda: torch.sum(part, dim=0, out=out))
    t_copy = timeit(lambda: part.clone())
    print(f"S={S} N={N} ({S*N*4/1e6:.1f} MB): torch.sum {t_sum*1e3:7.1f} us "
          f"({S*N*4/t_sum/1e6:6.0f} GB/s) | clone {t_copy*1e3:7.1f} us", flush=True)

# the same reduction right after the partials were rewritten by a kernel
for S, N in ((256, 36864),):
    part = torch.randn(S, N, device="cuda")
    out = torch.empty(N, device="cuda")

    def rw_sum():
        part.mul_(1.0)
        torch.sum(part, dim=0, out=out)

    t_rw = timeit(rw_sum)
    t_mul = timeit(lambda: part.mul_(1.0))
    print(f"S={S} N={N}: mul_+sum {t_rw*1e3:7.1f} us, mul_ alone {t_mul*1e3:7.1f} us", flush=True)
