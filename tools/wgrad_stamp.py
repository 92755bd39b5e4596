"""Phase timeline of the window wgrad (conv_wgrad_win_kernel) and the
window conv (conv_fwd_frame_kernel) at the Cfg2 shapes, from the diagnostic
build's per-workgroup s_memrealtime stamps (make -C dalle2-video_amd/csrc
stamp; DV_STAMP in dv_conv.hip):

  DV_HIP_LIB=dalle2-video_amd/csrc/build_stamp/libdv_hip_stamp.so python tools/wgrad_stamp.py

Per shape: the launch span (first workgroup start -> last workgroup end), the
spread of workgroup start times, and the median per-workgroup duration of each
phase (stamps: 0 entry, 1 first stage / chunk landed, 2 main loop done,
3 halves summed (wgrad), 4 stores drained).  s_memrealtime ticks at 100 MHz."""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dalle2-video_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from dalle2_video import _lib, ops  # noqa: E402
from dalle2_video._lib import call, dt, ptr, stream  # noqa: E402

NST = 8
L = _lib.lib()
L.dv_debug_stamps.argtypes = [ctypes.c_void_p, ctypes.c_longlong]


def stamps(nblk):
    torch.cuda.synchronize()
    buf = np.zeros(nblk * NST, dtype=np.uint64)
    assert L.dv_debug_stamps(buf.ctypes.data, buf.size) == 0
    return buf.reshape(nblk, NST).astype(np.int64)


def report(tag, s, idx):
    t0 = s[:, 0].min()
    span = (s[:, idx[-1]].max() - t0) * 10 / 1e3
    skew = (s[:, 0].max() - t0) * 10 / 1e3
    parts = []
    for a, b in zip(idx[:-1], idx[1:]):
        d = (s[:, b] - s[:, a]) * 10 / 1e3
        parts.append(f"{a}->{b} {np.median(d):6.2f}")
    tot = np.median((s[:, idx[-1]] - s[:, 0]) * 10 / 1e3)
    print(f"{tag:44s} span {span:6.2f} us  start-skew {skew:5.2f}  per-WG {tot:6.2f} = " + "  ".join(parts),
          flush=True)


def wgrad_case(nf, h, w, cin, cout):
    g = torch.Generator(device="cuda").manual_seed(0)
    x = torch.randn(nf, h, w, cin, device="cuda", generator=g).bfloat16()
    dy = torch.randn(nf, h, w, cout, device="cuda", generator=g).bfloat16()
    ws = ops._wgrad_workspace(_lib.dtype_name(x), nf, h, w, cin, cin, False, cout, 3, x.device)
    dw = torch.empty(cout, cin, 1, 3, 3, device="cuda")
    db = torch.empty(cout, device="cuda")
    f = lambda: call("dv_conv_wgrad", dt(x), ptr(dy), cout, ptr(x), cin, cin, None, 0, ptr(dw), 0, ptr(db),
                     0, ptr(ws), ws.numel(), nf, h, w, cin, cout, cout, cin, 3, stream())
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    torch.cuda._sleep(200_000)
    f()
    nst = nf * h * w // 128
    tiles = (cout // 64) * (cin // 64)
    want = max(1, min(256 // tiles, nst))
    sps = (nst + want - 1) // want
    S = (nst + sps - 1) // sps
    report(f"wgrad ({nf},{h},{w}) {cin}->{cout} S={S}", stamps(tiles * S), [0, 1, 2, 3, 4])


def frame_case(nf, h, w, cin, cout):
    g = torch.Generator(device="cuda").manual_seed(1)
    x = torch.randn(nf, h, w, cin, device="cuda", generator=g).bfloat16()
    wt = torch.randn(cout, cin, 1, 3, 3, device="cuda", generator=g) / (9 * cin) ** 0.5
    b = torch.randn(cout, device="cuda", generator=g)
    y = torch.empty(nf, h, w, cout, device="cuda", dtype=torch.bfloat16)
    wp = ops.pack_conv_weight(wt, torch.bfloat16, cin, 2, cache=False)
    f = lambda: call("dv_conv_fwd8", dt(x), ptr(x), cin, cin, None, 0, ptr(wp), ptr(b), None, 0, None, 0, ptr(y), cout,
                     nf, h, w, cin, cout, 0, None, 0, 0, stream())
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    torch.cuda._sleep(200_000)
    f()
    m = nf * h * w
    co = 32 if (m // 128) * (cout // 64) <= 128 else 64
    # 8 waves on 128 channels where 64-channel tiles would take two rounds (dv_conv.hip, launch_fwd_frame)
    w8 = w == 16 and co == 64 and cout % 128 == 0 and (m // 128) * (cout // 64) > 256
    cw = 128 if w8 else co
    st = stamps((m // 128) * (cout // cw))
    report(f"frame fwd ({nf},{h},{w}) {cin}->{cout} {'8 waves x ' if w8 else ''}co{cw}", st, [0, 1, 2, 4])
    # wave 0's chunk loop split (shader clock): at the DMA wait, at the barrier, the rest (MFMAs + reads + issue)
    tot = st[:, 7].astype(np.float64)
    wt, bt = np.median(st[:, 5] / tot), np.median(st[:, 6] / tot)
    print(f"  chunk loop (wave 0): DMA wait {100 * wt:4.1f} %  barrier {100 * bt:4.1f} %  "
          f"MFMA + LDS reads + DMA issue {100 * (1 - wt - bt):4.1f} %", flush=True)


def stripe_case(nf, h, w, cin, cout, res=False):
    g = torch.Generator(device="cuda").manual_seed(2)
    x = torch.randn(nf, h, w, cin, device="cuda", generator=g).bfloat16()
    wt = torch.randn(cout, cin, 1, 3, 3, device="cuda", generator=g) / (9 * cin) ** 0.5
    b = torch.randn(cout, device="cuda", generator=g)
    rr = torch.randn(nf, h, w, cout, device="cuda", generator=g).bfloat16() if res else None
    y = torch.empty(nf, h, w, cout, device="cuda", dtype=torch.bfloat16)
    wp = ops.pack_conv_weight(wt, torch.bfloat16, cin, 0, cache=False)
    f = lambda: call("dv_conv_fwd", dt(x), ptr(x), cin, cin, None, 0, ptr(wp), ptr(b), ptr(rr), cout if res else 0,
                     None, 0, ptr(y), cout, nf, h, w, cin, cout, 3, 0, None, 0, 0, stream())
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    torch.cuda._sleep(200_000)
    f()
    ct = cout // 64
    nst = nf * h * w // 128
    bx = max(1, min(256 // ct, nst))
    sps = (nst + bx - 1) // bx
    bx = (nst + sps - 1) // sps
    st = stamps(bx * ct)
    report(f"stripe fwd ({nf},{h},{w}) {cin}->{cout}{' +res' if res else ''} {sps} stages", st, [0, 1, 2, 3])
    report("  stage 1: mfma / epilogue / wait / issue+barrier", st, [2, 4, 5, 6, 7])


for shp in [(64, 64, 64, 64, 64), (64, 32, 32, 64, 64), (64, 32, 32, 128, 128), (64, 16, 16, 256, 256),
            (64, 8, 8, 512, 512)]:
    wgrad_case(*shp)
stripe_case(64, 64, 64, 64, 64)
stripe_case(64, 64, 64, 64, 64, res=True)
stripe_case(64, 64, 64, 64, 128, res=True)
for shp in [(64, 8, 8, 512, 512), (64, 8, 8, 256, 256), (64, 16, 16, 256, 256)]:
    frame_case(*shp)
