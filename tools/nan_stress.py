"""Repeat config 3's unet2 training call (bf16, graphs on, blur forced on and
off in turn: the sequence of tests/test_cfg3_trainer_gpu.py) many times and
count the calls whose flat gradient is not finite, naming the parameters.
With poison=1 the split-K partial arena and the wgrad workspace are filled
with NaN before every call: a partial read that no kernel of the call wrote
then shows on every call instead of when stale bits happen to be NaN.
  python tools/nan_stress.py [calls] [gn_path] [poison]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dalle2-video_amd"))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

from dalle2_video import _lib, ops  # noqa: E402
from tests.test_cfg3_trainer_gpu import _clip, _trainer  # noqa: E402


def main():
    calls = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    path = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    poison = len(sys.argv) > 3 and sys.argv[3] == "1"
    _lib.call("dv_gn_path", path)
    dec, tr = _trainer(True, True)
    video = _clip()
    torch.cuda.manual_seed(1)
    tr(video=video, unet_number=2)
    tr.update(2)
    lc = dec.lowres_conds[1]
    opt = tr.optim1
    names = {id(p): n for n, p in dec.unets[1].named_parameters()}
    bad = 0
    for i in range(calls):
        lc.blur_prob = 1.0 if (i // 4) % 2 == 0 else 0.0
        opt.zero_grad()
        if poison:
            for chunks in ops.WGRAD_DEFER.chunks.values():
                for c in chunks:
                    c.fill_(float("nan"))
            for w in list(ops._WS.values()) + list(ops._XE_WS.values()):
                w.fill_(float("nan"))
        torch.cuda.manual_seed(7 + (i % 2))
        loss = tr(video=video, unet_number=2)
        torch.cuda.synchronize()
        G = opt.flat_grad
        if not torch.isfinite(G).all():
            bad += 1
            which = [names[id(p)] for p in opt._flat[5] if not torch.isfinite(p.grad).all()]
            print(f"call {i}: non-finite gradient in {len(which)} params: {which[:6]} loss {loss}", flush=True)
        if i % 16 == 15:
            print(f"{i + 1} calls, {bad} non-finite", flush=True)
    print(f"gn_path {path} poison {int(poison)}: {bad} of {calls} calls non-finite", flush=True)


if __name__ == "__main__":
    main()
