"""Find which Python call sites launch torch-side fill/copy/add kernels in one
bench step (torch.profiler with stacks).  Usage: python tools/trace_ops.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "dalle2-video_amd"))

import torch  # noqa: E402
from torch.profiler import ProfilerActivity, profile  # noqa: E402

import bench  # noqa: E402


def main():
    class A:
        batch, frames, size, dtype = 4, 16, 64, "bf16"
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
    with profile(activities=[ProfilerActivity.CPU], with_stack=True, record_shapes=True) as prof:
        step()
        torch.cuda.synchronize()
    want = ("aten::fill_", "aten::zero_", "aten::add", "aten::add_", "aten::copy_", "aten::cat",
            "aten::to", "aten::_to_copy", "aten::zeros", "aten::zeros_like", "aten::clone")
    table = prof.key_averages(group_by_stack_n=6).table(sort_by="count", row_limit=60)
    lines = [ln for ln in table.splitlines()]
    print(table[:20000])
    evs = [e for e in prof.key_averages(group_by_stack_n=8) if e.key in want]
    evs.sort(key=lambda e: -e.count)
    for e in evs[:40]:
        print(f"{e.count:4d} {e.key:16s} shapes={str(e.input_shapes)[:80]}")
        for fr in e.stack[:8]:
            if "dalle2_video" in fr or "bench" in fr or "trainer" in fr:
                print("        ", fr)


if __name__ == "__main__":
    main()
