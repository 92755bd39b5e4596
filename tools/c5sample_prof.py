"""Config-5 sampling loop (unet1, 32x128x128 clip, bs 2, 16 DDPM steps, HIP-graph
denoise steps) for a kernel trace: run under rocprofv3 --kernel-trace, then
    python tools/c5sample_prof.py --summary <run_kernel_trace.csv>
prints per-denoise-step kernel time by kernel (steps counted by the mid-attention
launches).  argv: --fp8 for the MX-fp8 mode."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dalle2-video_amd"))


def summary(path):
    import csv
    from collections import defaultdict
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    # the last sample() call: from the last run of 16 consecutive attention launches
    att = [i for i, r in enumerate(rows) if "mqa_fwd" in r["Kernel_Name"]]
    steps = 16
    first = att[-steps]
    # include the launches of the first step before its attention: back to the previous step's end
    prev = att[-steps - 1] if len(att) > steps else 0
    seg = rows[prev + 1:]
    span_steps = [int(rows[a]["Start_Timestamp"]) for a in att[-steps:]]
    per = (span_steps[-1] - span_steps[0]) / (steps - 1) / 1e3
    agg = defaultdict(lambda: [0.0, 0])
    for r in seg:
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
        k = r["Kernel_Name"][:90]
        agg[k][0] += d
        agg[k][1] += 1
    tot = sum(v[0] for v in agg.values()) / steps
    print(f"denoise step wall (attention to attention) {per:.1f} us, kernel sum {tot:.1f} us, "
          f"{sum(v[1] for v in agg.values()) / steps:.0f} launches / step")
    for k, (t, n) in sorted(agg.items(), key=lambda kv: -kv[1][0])[:45]:
        print(f"{t / steps:9.1f} us/step {n / steps:6.1f}/step avg {t / n:7.1f} us  {k}")


def main():
    import torch
    from dalle2_video.dalle2_video import Unet3D, VideoDecoder
    from dalle2_video.utils import deterministic_fill_
    dev = torch.device("cuda")
    u = Unet3D(64, video_embed_dim=512, channels=3, dim_mults=(1, 2, 4, 8))
    dec = VideoDecoder(unet=(u,), frame_sizes=(128,), frame_numbers=(32,), timesteps=16, learned_variance=False)
    u = dec.unets[0]
    deterministic_fill_(u)
    dec = dec.to(dev)
    u.fp8 = "--fp8" in sys.argv
    emb = torch.randn(2, 512, device=dev)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        for _ in range(2):
            dec.sample(video_embed=emb, one_unet_in_gpu_at_time=False)
    torch.cuda.synchronize()
    print("done", flush=True)


if __name__ == "__main__":
    if "--summary" in sys.argv:
        summary(sys.argv[sys.argv.index("--summary") + 1])
    else:
        main()
