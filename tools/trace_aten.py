"""Which Python call sites launch torch-side GPU kernels (fills, adds, copies,
RNG, clones) in one eager training step + update: a TorchDispatchMode that
records every aten op that is not a view / allocation, with the innermost repo
frames of its Python stack.  Usage: python tools/trace_aten.py"""
import collections
import os
import sys
import traceback

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "dalle2-video_amd"))

import torch  # noqa: E402
from torch.utils._python_dispatch import TorchDispatchMode  # noqa: E402

import bench  # noqa: E402

SKIP = ("empty", "detach", "view", "as_strided", "select", "slice", "alias", "reshape", "_reshape_alias",
        "t.", "transpose", "permute", "expand", "unsqueeze", "squeeze", "split", "chunk", "unbind",
        "_to_copy.default" if False else "__none__", "is_nonzero", "item", "_local_scalar_dense", "set_",
        "record_stream", "lift_fresh", "size", "stride", "numel", "dim", "new_empty", "resize_")


class Rec(TorchDispatchMode):
    def __init__(self):
        super().__init__()
        self.hits = collections.Counter()

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        name = str(func)
        base = name.split(".")[1] if name.startswith("aten.") else name
        if not any(base == s or base.startswith(s) for s in SKIP):
            shapes = tuple(tuple(a.shape) for a in args if isinstance(a, torch.Tensor))[:3]
            frames = [f for f in traceback.extract_stack()[:-1]
                      if ("dalle2_video" in f.filename or "bench.py" in f.filename) and "trace_aten" not in f.filename]
            where = " <- ".join(f"{os.path.basename(f.filename)}:{f.lineno}:{f.name}" for f in frames[-3:][::-1])
            self.hits[(name, str(shapes)[:70], where)] += 1
        return func(*args, **(kwargs or {}))


def main():
    class A:
        batch, frames, size, dtype = 4, 16, 64, "bf16"
        no_graphs = True  # eager: a replayed graph dispatches no aten ops
    dev = torch.device("cuda", 0)
    dec, trainer = bench.build(A, dev)
    g = torch.Generator(device=dev).manual_seed(0)
    video = torch.rand(4, 3, 16, 64, 64, device=dev, generator=g)
    embed = torch.randn(4, 512, device=dev, generator=g)

    def step():
        trainer(video_embed=embed, video=video, unet_number=1)
        trainer.update(1)

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    rec = Rec()
    with rec:
        step()
    torch.cuda.synchronize()
    for (name, shp, where), n in sorted(rec.hits.items(), key=lambda kv: kv[0][2]):
        print(f"{n:3d} {name:32s} {shp:70s} {where}")


if __name__ == "__main__":
    main()
