"""Same-process A/B of the config-5 mid attention forward (B 2, 8,192 tokens,
16 heads x 32, MQA): the bf16 K/V-streamed kernel (dv_mqa_fwd, bounded-score
and online-max paths) against the MX-fp8 PV kernel (dv_mqa_fwd_fp8).  Times
the attention launches only (prep excluded), as a captured graph of R
back-to-back launches replayed (no event brackets between launches):
    python tools/mqa8_ab.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dalle2-video_amd"))
import ctypes  # noqa: E402

import torch  # noqa: E402

from dalle2_video import _lib  # noqa: E402
from dalle2_video._lib import call, ptr, stream  # noqa: E402

PEAK_BF16, PEAK_FP8 = 2516.6, 5033.2
B, N, H = 2, 8192, 16
NKP = (N + 1 + 31) // 32 * 32
scale = 1.0 / 32


def graph_us(fn, reps=20, iters=10):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        g.replay()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / (iters * reps)


def main():
    flops = 4.0 * B * H * N * (N + 1) * 32
    for qmag in (1.0, 8.0):
        g = torch.Generator(device="cuda").manual_seed(5)
        q = (torch.randn(B * N, H * 32, device="cuda", generator=g) * qmag).bfloat16()
        kv = torch.randn(B * N, 64, device="cuda", generator=g).bfloat16()
        nkv = torch.randn(2, 32, device="cuda", generator=g)
        kp = torch.empty(B, NKP, 32, dtype=torch.bfloat16, device="cuda")
        vp = torch.empty_like(kp)
        kmax = torch.empty(B * ((NKP + 63) // 64), dtype=torch.float32, device="cuda")
        call("dv_mqa_prep", _lib.DV_BF16, ptr(kv), 64, ptr(nkv), ptr(kp), ptr(vp), B, N, NKP,
             ctypes.c_float(scale), ptr(kmax), stream())
        o = torch.empty(B * N, H * 32, dtype=torch.bfloat16, device="cuda")
        lse = torch.empty(B, H, N, dtype=torch.float32, device="cuda")
        need = ctypes.c_longlong(0)
        call("dv_mqa_fwd_fp8_ws", B, NKP, ctypes.byref(need))
        v8 = torch.empty(need.value, dtype=torch.uint8, device="cuda")
        legs = {
            "bf16 (bounded scores when |q| max|k| <= 64)": lambda: call(
                "dv_mqa_fwd", _lib.DV_BF16, ptr(q), H * 32, ptr(kp), ptr(vp), ptr(o), H * 32, ptr(lse), B, N, NKP,
                H, ctypes.c_float(scale), ptr(kmax), stream()),
            "bf16 online max": lambda: call(
                "dv_mqa_fwd", _lib.DV_BF16, ptr(q), H * 32, ptr(kp), ptr(vp), ptr(o), H * 32, ptr(lse), B, N, NKP,
                H, ctypes.c_float(scale), None, stream()),
            "fp8 PV (+ V quantisation)": lambda: call(
                "dv_mqa_fwd_fp8", ptr(q), H * 32, ptr(kp), ptr(vp), ptr(v8), need.value, ptr(o), H * 32, ptr(lse),
                B, N, NKP, H, stream()),
        }
        for name, fn in legs.items():
            us = graph_us(fn)
            tf = flops / (us * 1e-6) / 1e12
            blend = 2 / (1 / PEAK_BF16 + 1 / PEAK_FP8) if "fp8" in name else PEAK_BF16
            print(f"qmag {qmag:3.0f}  {name:46s} {us:7.1f} us  {tf:6.1f} TF/s  frac {tf / blend:.3f}", flush=True)


if __name__ == "__main__":
    main()
