"""Per-launch time of the bf16 3x3 row-window wgrad (kernel + split-K sum) at
the Cfg2 shapes; run twice with DV_WG_OLD=0 / 1 on one box for an A/B.
Prints one line per shape and a checksum of dW so the two runs can be diffed."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dalle2-video_amd"))
import torch  # noqa: E402

from dalle2_video import ops  # noqa: E402
from dalle2_video._lib import call, ptr, stream, dt  # noqa: E402

SHAPES = [  # nf, h, w, c0, c1, cout
    (64, 64, 64, 64, 0, 64), (64, 64, 64, 64, 64, 64),
    (64, 32, 32, 64, 0, 64), (64, 32, 32, 128, 0, 128), (64, 32, 32, 128, 64, 128),
    (64, 16, 16, 128, 0, 128), (64, 16, 16, 256, 0, 256), (64, 16, 16, 256, 128, 256),
    (64, 8, 8, 256, 0, 256), (64, 8, 8, 512, 0, 512), (64, 8, 8, 512, 256, 512),
]


def main():
    tag = os.environ.get("DV_WG_OLD", "0")
    tot = 0.0
    for nf, h, w, c0, c1, cout in SHAPES:
        g = torch.Generator(device="cuda").manual_seed(nf * h + c0 + c1 + cout)
        cin = c0 + c1
        x0 = torch.randn(nf, h, w, c0, device="cuda", generator=g).bfloat16()
        x1 = torch.randn(nf, h, w, c1, device="cuda", generator=g).bfloat16() if c1 else None
        dy = torch.randn(nf, h, w, cout, device="cuda", generator=g).bfloat16()
        ws = ops._wgrad_workspace("bf16", nf, h, w, cin, c0, c1 > 0, cout, 3, x0.device)
        dw = torch.empty(cout, cin, 1, 3, 3, device="cuda")
        db = torch.empty(cout, device="cuda")

        def run():
            call("dv_conv_wgrad", dt(x0), ptr(dy), cout, ptr(x0), c0, c0, ptr(x1) if c1 else None, c1,
                 ptr(dw), 0, ptr(db), 0, ptr(ws), ws.numel(), nf, h, w, cin, cout, cout, cin, 3, stream())
        for _ in range(3):
            run()
        torch.cuda.synchronize()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        it = 20
        s.record()
        for _ in range(it):
            run()
        e.record()
        torch.cuda.synchronize()
        us = s.elapsed_time(e) / it * 1e3
        tot += us
        fl = 2.0 * nf * h * w * cout * cin * 9
        # reference checksum (fp32 torch on the same bf16 values)
        xc = x0.float() if not c1 else torch.cat([x0.float(), x1.float()], -1)
        ref = torch.nn.grad.conv2d_weight(xc.permute(0, 3, 1, 2), (cout, cin, 3, 3),
                                          dy.float().permute(0, 3, 1, 2), padding=1)
        err = ((dw[:, :, 0] - ref).norm() / ref.norm()).item()
        derr = ((db - dy.float().sum((0, 1, 2))).norm() / db.norm()).item()
        print(f"DV_WG_OLD={tag} nf={nf} {h}x{w} {c0}+{c1}->{cout}: {us:7.1f} us "
              f"{fl / us / 1e6:7.1f} TF/s  rel-err dW {err:.2e} db {derr:.2e}", flush=True)
    print(f"DV_WG_OLD={tag} total {tot:.1f} us")


if __name__ == "__main__":
    main()
