"""Per-call device time at the Cfg2 64^2 shape (bf16, 4 clips x 16 frames, 64
channels): the 3x3 stripe conv with its statistics epilogue, the GroupNorm
apply it replaces when folded (dv_gn_fwd over the conv's sums), and the
folded conv (dv_conv_fwd_gn_in, with and without storing y).  Each as N calls
replayed from one HIP graph.  With the diagnostic build (make -C
dalle2-video_amd/csrc stamp; DV_HIP_LIB=<libdv_hip_stamp.so>) also the stripe
kernel's per-workgroup phases, plain vs folded (stamps: 0 entry, 1 prologue
done, 2 stage 0 done, 4 stage 1's MFMA loop, 5 its epilogue, 6 its DMA wait,
7 its barrier, 3 end; median us per workgroup).

  python tools/gn_fold_probe.py
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dalle2-video_amd"))
import torch  # noqa: E402

from dalle2_video import _lib, ops  # noqa: E402

N = 8
L = _lib.lib()
STAMPS = hasattr(L, "dv_debug_stamps")
if STAMPS:
    L.dv_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_longlong]


PRO = os.environ.get("DV_STAMP_PRO") == "1"  # the library was built with -DDV_STAMP_PRO


def phases(fn, nblk=256):
    import numpy as np
    fn()
    torch.cuda.synchronize()
    buf = np.zeros(nblk * 8, dtype=np.uint64)
    assert L.dv_debug_stamps(buf.ctypes.data, buf.size) == 0
    t = buf.reshape(nblk, 8).astype(np.int64)
    med = lambda a, b: np.median(t[:, b] - t[:, a]) / 100
    if PRO:  # stamps 7, 4..6 in the prologue: stage 0 DMA issued, all DMA issued, stage 0 + weights landed, weights in registers
        return (f"span {(t[:, 3].max() - t[:, 0].min()) / 100:6.2f}  issue-D0 {med(0, 7):5.2f}  issue-W,D1,D2 {med(7, 4):5.2f}  landed {med(4, 5):5.2f}"
                f"  wregs {med(5, 6):5.2f}  to-loop {med(6, 1):5.2f}  stage0 {med(1, 2):5.2f}  rest {med(2, 3):5.2f}"
                f"  total {med(0, 3):5.2f}  start-skew {(t[:, 0].max() - t[:, 0].min()) / 100:5.2f}")
    return (f"span {(t[:, 3].max() - t[:, 0].min()) / 100:6.2f}  prologue {med(0, 1):5.2f}  stage0 {med(1, 2):5.2f}"
            f"  s1 loop {med(2, 4):5.2f}  epi {med(4, 5):5.2f}  wait {med(5, 6):5.2f}  bar {med(6, 7):5.2f}"
            f"  rest {med(7, 3):5.2f}  total {med(0, 3):5.2f}")


def timed(fn):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(N):
            fn()
    g.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(5):
        g.replay()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / (5 * N) * 1e3


def main():
    torch.manual_seed(0)
    nb, T, H, C = 4, 16, 64, 64
    nf, P = nb * T, T * H * H
    dev = "cuda"
    z = torch.randn(nf, H, H, C, device=dev).bfloat16()
    y = torch.empty_like(z)
    out = torch.empty_like(z)
    w = torch.randn(C, C, 1, 3, 3, device=dev) * 0.05
    wp = ops.pack_conv_weight(w, torch.bfloat16, C, 0, False)
    bias = torch.zeros(C, device=dev)
    R = 8
    sums = torch.zeros(3, 1 << 16, device=dev)
    # plausible statistics in replica 0 (sum, sum of squares per clip / channel)
    sums[0, :nb * C * 2].view(nb, C, 2)[..., 0] = 0.0
    sums[0, :nb * C * 2].view(nb, C, 2)[..., 1] = float(P)
    gamma, beta = torch.ones(C, device=dev), torch.zeros(C, device=dev)
    ss = 0.1 * torch.randn(nb, 2 * C, device=dev)
    mean = torch.empty(nb * 8, device=dev)
    rstd = torch.empty_like(mean)
    st = _lib.stream

    def conv_stats():
        _lib.call("dv_conv_fwd", _lib.dt(z), _lib.ptr(z), C, C, None, 0, _lib.ptr(wp), _lib.ptr(bias), None, 0,
                  None, 0, _lib.ptr(out), C, nf, H, H, C, C, 3, _lib.ACT_NONE, _lib.ptr(sums[1]), P, R, st())

    def apply(act=_lib.ACT_SILU):
        _lib.call("dv_gn_fwd", _lib.dt(z), _lib.ptr(z), C, _lib.ptr(y), C, None, 0, nb, P, C, 8,
                  ops.ctypes_float(1e-5), _lib.ptr(gamma), _lib.ptr(beta), _lib.ptr(ss), act,
                  _lib.ptr(mean), _lib.ptr(rstd), _lib.ptr(sums[0]), _lib.ptr(sums[2]), sums.shape[1], R, st())

    def fold(store):
        d = ops.DvGnIn()
        d.sums, d.rstride, d.R, d.P, d.groups, d.eps = sums[0].data_ptr(), nb * C * 2, R, P, 8, 1e-5
        d.gamma, d.beta, d.ss, d.mean, d.rstd = (gamma.data_ptr(), beta.data_ptr(), ss.data_ptr(),
                                                 mean.data_ptr(), rstd.data_ptr())
        d.y, d.ldy = (y.data_ptr() if store else None), C
        d.zero, d.zero_n = sums[2].data_ptr(), sums.shape[1]
        _lib.call("dv_conv_fwd_gn_in", ctypes.byref(d), _lib.ptr(z), C, _lib.ptr(wp), _lib.ptr(bias),
                  _lib.ptr(out), C, nf, H, H, C, C, _lib.ptr(sums[1]), P, R, st())

    t_conv = timed(conv_stats)
    t_apply = timed(apply)
    t_fold = timed(lambda: fold(True))
    t_fold_ns = timed(lambda: fold(False))
    print(f"64^2 x 64, 4 clips x 16 frames (us per call): conv+stats {t_conv:6.1f}  gn apply {t_apply:6.1f}  "
          f"sum {t_conv + t_apply:6.1f}  |  folded conv (y stored) {t_fold:6.1f}  (y not stored) {t_fold_ns:6.1f}",
          flush=True)
    print(f"  gn apply without the SiLU {timed(lambda: apply(_lib.ACT_NONE)):6.1f} us", flush=True)
    if STAMPS:
        print(f"  plain : {phases(conv_stats)}", flush=True)
        print(f"  folded: {phases(lambda: fold(True))}", flush=True)


if __name__ == "__main__":
    main()
