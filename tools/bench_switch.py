"""bench.py with module switches of dalle2_video.ops set first (the same-box
A/B of a kept change against its off state, tools/ab_switch.sh):
  python tools/bench_switch.py GRAD_OVERWRITE=0 [bench.py args]"""
import os
import runpy
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dalle2-video_amd"))
from dalle2_video import ops  # noqa: E402

args = sys.argv[1:]
while args and "=" in args[0] and not args[0].startswith("-"):
    name, val = args.pop(0).split("=", 1)
    if not hasattr(ops, name):
        raise SystemExit(f"ops has no switch {name}")
    setattr(ops, name, type(getattr(ops, name))(int(val)) if isinstance(getattr(ops, name), bool) else val)
sys.argv = [os.path.join(ROOT, "bench.py")] + args
runpy.run_path(sys.argv[0], run_name="__main__")
