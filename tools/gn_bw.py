"""GroupNorm passes vs plain streaming copies at the Cfg2 stage shapes (bf16).

Per shape: the forward apply alone (statistics already in the sums buffer, as
after a conv statistics epilogue), the forward apply with a residual, the
backward (reduce + apply) -- each against torch's own streaming kernels that
move the same bytes (clone: 4 B/elem, add: 6 B/elem), so the table shows how
far each GroupNorm pass sits from what a plain copy achieves on this box.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dalle2-video_amd"))
import torch  # noqa: E402

from dalle2_video import ops  # noqa: E402
from dalle2_video._lib import call, ptr, stream, dt  # noqa: E402


def timeit(fn, iters=50):
    """ms per call of fn, replayed from a captured HIP graph (no host launch cost)."""
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    st = torch.cuda.Stream()
    with torch.cuda.stream(st):
        with torch.cuda.graph(g, stream=st):
            for _ in range(iters):
                fn()
    g.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(3):
        g.replay()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / (3 * iters)


def case(nb, T, H, C, iters=50):
    nf = nb * T
    P = T * H * H
    dev = "cuda"
    z = torch.randn(nf, H, H, C, device=dev, dtype=torch.bfloat16)
    r = torch.randn_like(z)
    y = torch.empty_like(z)
    g = torch.randn(C, device=dev)
    b = torch.randn(C, device=dev)
    ss = torch.randn(nb, 2 * C, device=dev)
    mean = torch.empty(nb * 8, device=dev)
    rstd = torch.empty_like(mean)
    sums = torch.zeros(8, nb * C * 2, device=dev)
    sums[:, 1::2] = 1.0
    nxt = torch.zeros(8 * nb * C * 2, device=dev)
    f = ops.ctypes_float(1e-5)

    def apply(res):
        call("dv_gn_fwd", dt(z), ptr(z), C, ptr(y), C, ptr(res), C if res is not None else 0, nb, P, C, 8, f,
             ptr(g), ptr(b), ptr(ss), 1, ptr(mean), ptr(rstd), ptr(sums), ptr(nxt), nxt.numel(), 1, stream())

    dy = torch.randn_like(z)
    dz = torch.empty_like(z)
    dg, db = torch.zeros(C, device=dev), torch.zeros(C, device=dev)
    dss = torch.empty(nb, 2 * C, device=dev)
    sums2 = torch.zeros(2, ops._GnSums.CAP, device=dev)  # the step's buffers: R = min(8, CAP / (nb*C*2))

    def bwd():  # reduce + apply; the two buffers alternate as in ops._GnSums
        call("dv_gn_bwd", dt(z), ptr(dy), C, ptr(z), C, ptr(dz), C, nb, P, C, 8, ptr(g), ptr(b), ptr(ss), 1,
             ptr(mean), ptr(rstd), ptr(dg), ptr(db), ptr(dss), ptr(sums2[0]), ptr(sums2[1]), sums2.shape[1], 1,
             stream())
        call("dv_gn_bwd", dt(z), ptr(dy), C, ptr(z), C, ptr(dz), C, nb, P, C, 8, ptr(g), ptr(b), ptr(ss), 1,
             ptr(mean), ptr(rstd), ptr(dg), ptr(db), ptr(dss), ptr(sums2[1]), ptr(sums2[0]), sums2.shape[1], 1,
             stream())

    sums3 = torch.zeros(2, ops._GnSums.CAP, device=dev)

    def fwd_full():  # reduce + apply (no conv statistics epilogue); buffers alternate
        for i in (0, 1):
            call("dv_gn_fwd", dt(z), ptr(z), C, ptr(y), C, None, 0, nb, P, C, 8, f, ptr(g), ptr(b), ptr(ss), 1,
                 ptr(mean), ptr(rstd), ptr(sums3[i]), ptr(sums3[1 - i]), sums3.shape[1], 0, stream())

    n = z.numel() * 2  # bytes of one bf16 tensor
    t_app = timeit(lambda: apply(None), iters)
    t_appr = timeit(lambda: apply(r), iters)
    t_bwd = timeit(bwd, iters) / 2
    t_fwd = timeit(fwd_full, iters) / 2
    t_cp = timeit(lambda: y.copy_(z), iters)
    t_add = timeit(lambda: torch.add(z, r, out=y), iters)
    gb = lambda nbytes, ms: nbytes / ms / 1e9
    print(f"nb={nb} T={T} {H:3d}x{H:<3d} C={C:3d} {n/1e6:6.1f} MB | apply {t_app*1e3:6.1f} us "
          f"{gb(2*n, t_app):5.2f} TB/s | apply+res {t_appr*1e3:6.1f} us {gb(3*n, t_appr):5.2f} | "
          f"bwd(red+app) {t_bwd*1e3:6.1f} us {gb(5*n, t_bwd):5.2f} | fwd(red+app) {t_fwd*1e3:6.1f} us | copy {t_cp*1e3:6.1f} us "
          f"{gb(2*n, t_cp):5.2f} | add {t_add*1e3:6.1f} us {gb(3*n, t_add):5.2f}", flush=True)


if __name__ == "__main__":
    for H, C in ((64, 64), (32, 128), (32, 64), (16, 256), (16, 128), (8, 512), (8, 256)):
        case(4, 16, H, C)
