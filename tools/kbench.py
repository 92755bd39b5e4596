"""Micro-benchmark of individual HIP kernels at the Cfg2 (B=4,T=16,64x64) shapes."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dalle2-video_amd"))
import torch  # noqa: E402

from dalle2_video import ops  # noqa: E402


def timeit(fn, iters=20, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters


def conv_case(nf, h, w, cin, cout, k, dtype=torch.bfloat16):
    x = torch.randn(nf, h, w, cin, device="cuda", dtype=dtype)
    wt = (torch.randn(cout, cin, 1, k, k, device="cuda") / (cin * k * k) ** 0.5).requires_grad_()
    b = torch.randn(cout, device="cuda")
    flops = 2.0 * nf * h * w * cout * cin * k * k
    y = torch.empty(nf, h, w, cout, device="cuda", dtype=dtype)
    from dalle2_video._lib import call, ptr, stream, dt
    if ops.window_ok(x, None, cin, cin, cout, cin, cin, cout, 0, k, h, w, nf):
        wp = ops.pack_conv_weight(wt, dtype, cin, 2)
        def fwd():
            call("dv_conv_fwd8", dt(x), ptr(x), cin, cin, None, 0, ptr(wp), ptr(b), None, 0, None, 0, ptr(y),
                 cout, nf, h, w, cin, cout, 0, None, 0, 0, stream())
    else:
        wp = ops.pack_conv_weight(wt, dtype, cin, 0)
        def fwd():
            call("dv_conv_fwd", dt(x), ptr(x), cin, cin, None, 0, ptr(wp), ptr(b), None, 0, None, 0, ptr(y),
                 cout, nf, h, w, cin, cout, k, 0, None, 0, 0, stream())
    ms = timeit(fwd)
    dy = torch.randn_like(y)
    ws = ops._wgrad_workspace(ops._lib.dtype_name(x), nf, h, w, cin, cin, False, cout, k, x.device)
    dw = torch.empty(cout, cin, 1, k, k, device="cuda")
    db = torch.empty(cout, device="cuda")
    def wgrad():
        call("dv_conv_wgrad", dt(x), ptr(dy), cout, ptr(x), cin, cin, None, 0, ptr(dw), 0, ptr(db), 0,
             ptr(ws), ws.numel(), nf, h, w, cin, cout, cout, cin, k, stream())
    msw = timeit(wgrad)
    print(f"conv nf={nf} {h}x{w} {cin}->{cout} k={k} {str(dtype)[6:]}: fwd {ms*1e3:8.1f} us "
          f"{flops/ms/1e9:7.1f} TF/s | wgrad {msw*1e3:8.1f} us {flops/msw/1e9:7.1f} TF/s")


def gemm_case(nb, rows, m, n):
    from dalle2_video._lib import call, ptr, stream
    a = torch.randn(nb * rows, m, device="cuda", dtype=torch.bfloat16)
    b = torch.randn(nb * rows, n, device="cuda", dtype=torch.bfloat16)
    o = torch.zeros(nb, m, n, device="cuda")
    ms = timeit(lambda: call("dv_gemm_tn_batched", 1, ptr(a), m, ptr(b), n, ptr(o), rows, nb, m, n, stream()))
    print(f"gemm_tn_batched nb={nb} rows={rows} {m}x{n}: {ms*1e3:8.1f} us")


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "one":
        conv_case(64, 64, 64, 64, 64, 3)
        sys.exit(0)
    if len(sys.argv) > 1 and sys.argv[1] == "fwd1":  # forward only, for counter passes
        x = torch.randn(64, 64, 64, 64, device="cuda", dtype=torch.bfloat16)
        wt = torch.randn(64, 64, 1, 3, 3, device="cuda") / 24
        b = torch.randn(64, device="cuda")
        wp = ops.pack_conv_weight(wt, torch.bfloat16, 64, 0)
        y = torch.empty_like(x)
        from dalle2_video._lib import call, ptr, stream, dt
        for _ in range(20):
            call("dv_conv_fwd", dt(x), ptr(x), 64, 64, None, 0, ptr(wp), ptr(b), None, 0, None, 0, ptr(y),
                 64, 64, 64, 64, 64, 64, 3, 0, None, 0, 0, stream())
        torch.cuda.synchronize()
        sys.exit(0)
    if len(sys.argv) > 1 and sys.argv[1] == "fwd8":  # the 8x8-stage 512->512 forward, for counter passes
        x = torch.randn(64, 8, 8, 512, device="cuda", dtype=torch.bfloat16)
        wt = torch.randn(512, 512, 1, 3, 3, device="cuda") / 68
        b = torch.randn(512, device="cuda")
        wp = ops.pack_conv_weight(wt, torch.bfloat16, 512, 2)
        y = torch.empty_like(x)
        from dalle2_video._lib import call, ptr, stream, dt
        for _ in range(20):
            call("dv_conv_fwd8", dt(x), ptr(x), 512, 512, None, 0, ptr(wp), ptr(b), None, 0, None, 0, ptr(y),
                 512, 64, 8, 8, 512, 512, 0, None, 0, 0, stream())
        torch.cuda.synchronize()
        sys.exit(0)
    if len(sys.argv) > 1 and sys.argv[1] == "fwd":
        for c in ((64, 16, 16, 128, 128), (64, 32, 32, 192, 128), (64, 64, 64, 128, 64), (64, 16, 16, 384, 256),
                  (64, 16, 16, 256, 256), (64, 8, 8, 256, 256), (64, 8, 8, 512, 512), (64, 8, 8, 768, 512),
                  (64, 32, 32, 128, 128), (64, 8, 8, 512, 256), (64, 16, 16, 256, 128)):
            conv_case(*c, 3)
        sys.exit(0)
    gemm_case(4, 16384, 32, 64)
    gemm_case(4, 4096, 32, 128)
    gemm_case(4, 1024, 32, 256)
    for dt_ in (torch.bfloat16,):
        conv_case(64, 64, 64, 64, 64, 3, dt_)
        conv_case(64, 64, 64, 128, 64, 3, dt_)
        conv_case(64, 32, 32, 128, 128, 3, dt_)
        conv_case(64, 16, 16, 256, 256, 3, dt_)
        conv_case(64, 8, 8, 512, 512, 3, dt_)
        conv_case(64, 8, 8, 768, 512, 3, dt_)
        conv_case(64, 32, 32, 256, 64, 1, dt_)
        conv_case(64, 64, 64, 8, 32, 3, dt_)
        conv_case(64, 64, 64, 8, 16, 15, dt_)
    conv_case(64, 64, 64, 64, 64, 3, torch.float32)
