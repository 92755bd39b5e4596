"""Phase timeline of the cross-attention forward (xattn_fwd_kernel) at the Cfg2
shapes, from the diagnostic build's per-workgroup s_memrealtime stamps (make -C
dalle2-video_amd/csrc stamp; DV_STAMP in dv_xattn.hip):

  DV_HIP_LIB=dalle2-video_amd/csrc/build_stamp/libdv_hip_stamp.so python tools/xattn_stamp.py

Forward stamps: 0 entry, 1 channel loop (scores + LN sums) issued, 2 cross-wave
sums done, 3 softmax + P stored, 4 output statistics summed, 5 output stores
issued, 6 stores drained.  Backward: 0 entry, 1 pass A (LN_out statistics),
2 pass B (dO stored, dP), 3 softmax backward, 4 pass C (dx stored), 5 drained.  s_memrealtime ticks at 100 MHz."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dalle2-video_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from dalle2_video import _lib, ops  # noqa: E402

NST = 8
L = _lib.lib()
L.dv_debug_stamps_xattn.argtypes = [ctypes.c_void_p, ctypes.c_longlong]


def stamps(nblk):
    torch.cuda.synchronize()
    buf = np.zeros(nblk * NST, dtype=np.uint64)
    assert L.dv_debug_stamps_xattn(buf.ctypes.data, buf.size) == 0
    return buf.reshape(nblk, NST).astype(np.int64)


def report(tag, s, idx, wall_us):
    t0 = s[:, 0].min()
    span = (s[:, idx[-1]].max() - t0) * 10 / 1e3
    skew = (s[:, 0].max() - t0) * 10 / 1e3
    parts = []
    for a, b in zip(idx[:-1], idx[1:]):
        d = (s[:, b] - s[:, a]) * 10 / 1e3
        parts.append(f"{a}->{b} {np.median(d):5.2f}")
    tot = np.median((s[:, idx[-1]] - s[:, 0]) * 10 / 1e3)
    print(f"{tag:34s} event {wall_us:6.2f} us  span {span:6.2f}  start-skew {skew:5.2f}  per-WG {tot:6.2f} = "
          + "  ".join(parts), flush=True)


def case(nf, h, w, C, nb):
    g = torch.Generator(device="cuda").manual_seed(0)
    x = torch.randn(nf, h, w, C, device="cuda", generator=g).bfloat16()
    ctx = torch.randn(nb, 2, 64, device="cuda", generator=g)
    g1 = 1 + 0.1 * torch.randn(C, device="cuda", generator=g)
    g2 = 1 + 0.1 * torch.randn(C, device="cuda", generator=g)
    null_kv = torch.randn(2, 64, device="cuda", generator=g)
    wq = torch.randn(512, C, device="cuda", generator=g) / C ** 0.5
    wkv = torch.randn(1024, 64, device="cuda", generator=g) / 8
    wo = torch.randn(C, 512, device="cuda", generator=g) / 512 ** 0.5

    xg = x.clone().requires_grad_()
    gy = torch.randn_like(x)

    def run():
        with torch.no_grad():
            ops.cross_attention(x, ctx, g1, null_kv, wq, wkv, wo, g2, nb, 1e-5)

    def run_bwd():
        ops.cross_attention(xg, ctx, g1, null_kv, wq, wkv, wo, g2, nb, 1e-5).backward(gy)

    for _ in range(3):
        run()
    torch.cuda.synchronize()
    s0, s1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s0.record()
    run()
    s1.record()
    torch.cuda.synchronize()
    ntok = nf * h * w
    tiles = ntok // 32
    split = tiles < 1024 and C >= 128
    nblk = tiles if split else (tiles + 3) // 4
    report(f"xattn fwd {nf}x{h}x{w}x{C}", stamps(nblk), [0, 1, 2, 3, 4, 5, 6], s0.elapsed_time(s1) * 1e3)
    for _ in range(2):
        run_bwd()
    report(f"xattn bwd {nf}x{h}x{w}x{C}", stamps(nblk), [0, 1, 2, 3, 4, 5], 0.0)


if __name__ == "__main__":
    case(64, 8, 8, 512, 4)
    case(64, 8, 8, 256, 4)
    case(64, 16, 16, 256, 4)
    case(64, 16, 16, 128, 4)
    case(64, 32, 32, 128, 4)
    case(64, 32, 32, 64, 4)
