"""Host-side time of the pieces of trainer.update() at the benched Cfg2 step
(no device syncs inside update: only the launches' host cost shows):
    python tools/update_host_probe.py"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "dalle2-video_amd"))
import torch  # noqa: E402

import bench  # noqa: E402
from dalle2_video import ops  # noqa: E402

sys.argv = ["bench.py"]
args = bench.parse()
dev = torch.device("cuda", 0)
dec, tr = bench.build(args, dev)
g = torch.Generator(device=dev).manual_seed(1)
video = torch.rand(4, 3, 16, 64, 64, device=dev, generator=g)
embed = torch.randn(4, 512, device=dev, generator=g)
for _ in range(6):
    tr(video_embed=embed, video=video, unet_number=1)
    tr.update(1)
torch.cuda.synchronize()
opt = tr.optim0
rows = []
for _ in range(20):
    tr(video_embed=embed, video=video, unet_number=1)  # ends with the loss sync
    t0 = time.perf_counter()
    tr._check_flat(1)
    t1 = time.perf_counter()
    coef = opt.clip_coefficient(tr.max_grad_norm)
    t2 = time.perf_counter()
    opt.step(clip_coef=coef)
    t3 = time.perf_counter()
    opt.zero_grad()
    t4 = time.perf_counter()
    ops.PACK.refresh()
    t5 = time.perf_counter()
    tr.sched0.step()
    tr.increment_step(1)
    t6 = time.perf_counter()
    rows.append([t1 - t0, t2 - t1, t3 - t2, t4 - t3, t5 - t4, t6 - t5])
    torch.cuda.synchronize()
import statistics as st  # noqa: E402
names = ["check_flat", "clip_coefficient", "opt.step", "zero_grad", "PACK.refresh", "sched+increment"]
for i, n in enumerate(names):
    print(f"{n:18s} median {st.median(r[i] for r in rows) * 1e6:8.1f} us")

# repack-table churn: entries and table rebuilds across steps
n0 = len(ops.PACK.entries)
rebuilt = 0
for _ in range(5):
    tr(video_embed=embed, video=video, unet_number=1)
    rebuilt += ops.PACK._table_key is None
    tr.update(1)
print(f"PACK entries {n0} -> {len(ops.PACK.entries)}, tables rebuilt in {rebuilt} of 5 updates")
t0 = time.perf_counter()
for _ in range(20):
    for e in ops.PACK.entries.values():
        e["epoch"] = ops.PACK.epoch
print(f"epoch loop over {len(ops.PACK.entries)} entries: {(time.perf_counter() - t0) / 20 * 1e6:.1f} us")

# per C-ABI call host time inside update()
from dalle2_video import _lib as LB  # noqa: E402
import dalle2_video.trainer as TR  # noqa: E402
orig = LB.call
acc = {}


def timed(name, *a):
    t0 = time.perf_counter()
    orig(name, *a)
    acc.setdefault(name, []).append(time.perf_counter() - t0)


for mod in (LB, TR, ops):
    if hasattr(mod, "call"):
        mod.call = timed
for _ in range(10):
    tr(video_embed=embed, video=video, unet_number=1)
    acc.clear()
    tr.update(1)
    torch.cuda.synchronize()
for k, v in acc.items():
    print(f"{k:34s} n={len(v)} each {[round(x * 1e6, 1) for x in v]}")

import cProfile  # noqa: E402
import pstats  # noqa: E402
LB.call = orig
for mod in (TR, ops):
    if hasattr(mod, "call"):
        mod.call = orig
pr = cProfile.Profile()
for _ in range(20):
    tr(video_embed=embed, video=video, unet_number=1)
    pr.enable()
    tr.update(1)
    pr.disable()
    torch.cuda.synchronize()
pstats.Stats(pr).sort_stats("tottime").print_stats(18)
