"""Phase timeline of the mid-attention kernels at the Cfg2 shape (B = 4 clips,
N = 1,024 tokens, 16 heads x 32, 1,025 keys) from the diagnostic build's
per-workgroup s_memrealtime stamps (make -C dalle2-video_amd/csrc stamp;
DV_STAMP in dv_attn.hip):

  DV_HIP_LIB=dalle2-video_amd/csrc/build_stamp/libdv_hip_stamp.so python tools/mqa_stamp.py

Stamps per kernel: 0 entry, 1 operands staged (K / V of the clip in LDS for
the forward and dq; the first query tile for dk/dv), 2 loop done, 3 results
stored.  s_memrealtime ticks at 100 MHz."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dalle2-video_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from dalle2_video import _lib, ops  # noqa: E402

NB, NS = 4096, 4
L = _lib.lib()
L.dv_debug_stamps_mqa.argtypes = [ctypes.c_void_p, ctypes.c_longlong]


def stamps():
    torch.cuda.synchronize()
    buf = np.zeros(3 * NB * NS, dtype=np.uint64)
    assert L.dv_debug_stamps_mqa(buf.ctypes.data, buf.size) == 0
    return buf.reshape(3, NB, NS).astype(np.int64)


def report(tag, s):
    s = s[s[:, 0] > 0]
    t0 = s[:, 0].min()
    span = (s[:, 3].max() - t0) * 10 / 1e3
    skew = (s[:, 0].max() - t0) * 10 / 1e3
    ph = [np.median((s[:, b] - s[:, a]) * 10 / 1e3) for a, b in ((0, 1), (1, 2), (2, 3))]
    tot = np.median((s[:, 3] - s[:, 0]) * 10 / 1e3)
    last = (s[:, 0].max() - t0) * 10 / 1e3
    print(f"{tag:8s} {len(s):4d} WGs  span {span:6.2f} us  start-skew {skew:5.2f}  per-WG {tot:6.2f} = "
          f"staging {ph[0]:5.2f} + loop {ph[1]:5.2f} + epilogue {ph[2]:5.2f}  "
          f"(loop min/max {np.min((s[:, 2] - s[:, 1])) / 100:5.2f} / {np.max((s[:, 2] - s[:, 1])) / 100:5.2f})",
          flush=True)


def main():
    g = torch.Generator().manual_seed(3)
    B, N, H, D = 4, 1024, 16, 32
    q = torch.randn(B * N, H * D, generator=g).cuda().bfloat16().requires_grad_()
    kv = (torch.randn(B * N, 2 * D, generator=g) * 2).cuda().bfloat16().requires_grad_()
    null_kv = torch.randn(2, D, generator=g).cuda().requires_grad_()
    gy = torch.randn(B * N, H * D, generator=g).cuda().bfloat16()
    for _ in range(3):
        y = ops.mqa(q, kv, null_kv, B, N, H, 1.0 / D)
        y.backward(gy)
    torch.cuda.synchronize()
    torch.cuda._sleep(200_000)
    y = ops.mqa(q, kv, null_kv, B, N, H, 1.0 / D)
    y.backward(gy)
    s = stamps()
    for k, tag in enumerate(("fwd", "dq", "dkdv")):
        report(tag, s[k])


if __name__ == "__main__":
    main()
