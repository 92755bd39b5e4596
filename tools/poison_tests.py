"""Run GPU tests with the caching allocator's memory pre-filled with NaN, so a
kernel that reads memory nobody wrote (a torch.empty buffer taken as zero,
padding lanes or channels multiplied by zero weights) fails deterministically
instead of only when a previous test left garbage behind.
  python tools/poison_tests.py [--gib N] -- <pytest args>"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dalle2-video_amd"))
sys.path.insert(0, ROOT)


def poison(gib):
    import torch
    nan = float("nan")
    big = [torch.full((1 << 28,), nan, device="cuda") for _ in range(gib)]  # 1 GiB blocks (large pool)
    small = [torch.full((1 << 17,), nan, device="cuda") for _ in range(2048)]  # 512 KiB (small pool)
    tiny = [torch.full((1 << 10,), nan, device="cuda") for _ in range(4096)]
    torch.cuda.synchronize()
    del big, small, tiny  # the blocks stay cached: later allocations reuse NaN-filled memory


if __name__ == "__main__":
    args = sys.argv[1:]
    gib = 48
    if args[:1] == ["--gib"]:
        gib = int(args[1])
        args = args[2:]
    if args[:1] == ["--"]:
        args = args[1:]
    poison(gib)
    import pytest
    sys.exit(pytest.main(args))
