"""Host cost per C-ABI launch (ctypes call + hipLaunchKernel) against a torch
launch and a bare ctypes call:  python tools/launch_cost_probe.py"""
import ctypes
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dalle2-video_amd"))
import torch  # noqa: E402

from dalle2_video import _lib  # noqa: E402
from dalle2_video._lib import call, ptr, stream  # noqa: E402

x = torch.zeros(1024, device="cuda")
torch.cuda.synchronize()
L = _lib.lib()


def timeit(name, f, n=200):
    for _ in range(10):
        f()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        f()
    t1 = time.perf_counter()
    torch.cuda.synchronize()
    print(f"{name:40s} {(t1 - t0) / n * 1e6:7.2f} us/call", flush=True)


F = ctypes.c_float
timeit("ctypes dv_abi_version", lambda: L.dv_abi_version())
timeit("torch x.zero_()", lambda: x.zero_())
timeit("stream()", lambda: stream())
timeit("call dv_adamw n=1024", lambda: call("dv_adamw", ptr(x), ptr(x), ptr(x), ptr(x), 1024, 1024, F(1e-4), F(0.9),
                                             F(0.99), F(1e-8), F(0.01), F(0.5), F(0.5), None, stream()))
s = stream()
px = ctypes.c_void_p(x.data_ptr())
timeit("raw L.dv_adamw, prebuilt args", lambda: L.dv_adamw(px, px, px, px, 1024, 1024, F(1e-4), F(0.9), F(0.99),
                                                           F(1e-8), F(0.01), F(0.5), F(0.5), None, s))
timeit("hipGetLastError-only C call (dv_last_error)", lambda: L.dv_last_error())
