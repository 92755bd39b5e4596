"""GroupNorm at the Cfg2 shapes (bf16, 4 clips x 16 frames), forward and
backward: per-call device time of the single-launch form (dv_gn_path 3) vs the
two launches (dv_gn_path 1), each as N calls replayed from one HIP graph; with
the diagnostic build (DV_HIP_LIB=<libdv_hip_stamp.so>) also the single
launch's per-workgroup phases (stamps: 0 entry, 1 rows summed, 2 atomics
acknowledged, 3 clip arrived, 4 group terms, 5 stores drained).

  python tools/gn_coop_probe.py
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dalle2-video_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from dalle2_video import _lib, ops  # noqa: E402

L = _lib.lib()
STAMPS = hasattr(L, "dv_debug_stamps_gn")
if STAMPS:
    L.dv_debug_stamps_gn.argtypes = [ctypes.c_void_p, ctypes.c_longlong]

SHAPES = [(64, 64, False), (64, 64, True), (32, 64, False), (32, 128, False), (16, 128, False),
          (16, 256, False), (8, 256, False), (8, 512, True)]
N = 8


def timed(fn):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(N):
            fn()
        ops.gn_graph_boundary(torch.device("cuda"))
    g.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(5):
        g.replay()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / (5 * N) * 1e3


def phases(nblk):
    buf = np.zeros(nblk * 8, dtype=np.uint64)
    assert L.dv_debug_stamps_gn(buf.ctypes.data, buf.size) == 0
    s = buf.reshape(nblk, 8).astype(np.int64)
    t0 = s[:, 0].min()
    out = [f"span {(s[:, 5].max() - t0) / 100:6.2f}", f"skew {(s[:, 0].max() - t0) / 100:5.2f}"]
    for a, b in ((0, 1), (1, 2), (2, 3), (3, 4), (4, 5)):
        out.append(f"{a}->{b} {np.median(s[:, b] - s[:, a]) / 100:6.2f}")
    out.append(f"arrive-spread {(s[:, 2].max() - s[:, 2].min()) / 100:5.2f}")
    return "  ".join(out)


def main():
    torch.manual_seed(0)
    nb, T = 4, 16
    for H, C, res in SHAPES:
        z = (torch.randn(nb * T, H, H, C, device="cuda") * 2).bfloat16()
        gamma, beta = torch.ones(C, device="cuda"), torch.zeros(C, device="cuda")
        ss = 0.1 * torch.randn(nb, 2 * C, device="cuda")
        r = torch.randn_like(z) if res else None
        dy = torch.randn_like(z)
        line = f"{H:3d}^2 x {C:3d} res={int(res)}"
        for direction in ("fwd", "bwd"):
            for path in (1, 3):
                _lib.call("dv_gn_path", path)
                if direction == "fwd":
                    fn = lambda: ops._gn_forward(z, gamma, beta, ss, r, nb, 8, 1e-5, _lib.ACT_SILU, None)
                else:
                    y, g, b, s, mean, rstd = ops._gn_forward(z, gamma, beta, ss, r, nb, 8, 1e-5, _lib.ACT_SILU, None)
                    dz = torch.empty_like(z)
                    dg, db = torch.zeros(C, device="cuda"), torch.zeros(C, device="cuda")
                    dss = torch.empty(nb, 2 * C, device="cuda")

                    def fn():
                        cur, nxt = ops._gn_sums(z.device).take(nb * C * 2)
                        _lib.call("dv_gn_bwd", _lib.dt(z), _lib.ptr(dy), C, _lib.ptr(z), C, _lib.ptr(dz), C, nb,
                                  T * H * H, C, 8, _lib.ptr(g), _lib.ptr(b), _lib.ptr(s), _lib.ACT_SILU,
                                  _lib.ptr(mean), _lib.ptr(rstd), _lib.ptr(dg), _lib.ptr(db), _lib.ptr(dss),
                                  _lib.ptr(cur), _lib.ptr(nxt), nxt.numel(), 1, _lib.stream())
                us = timed(fn)
                line += f"  {direction}{'-1L' if path == 3 else '-2L'} {us:6.1f}"
                if STAMPS and path == 3:
                    fn()
                    torch.cuda.synchronize()
                    print(f"   [{H}^2 x {C} {direction}] {phases(256)}", flush=True)
        _lib.call("dv_gn_path", 0)
        print(line, flush=True)


if __name__ == "__main__":
    main()
