#!/usr/bin/env python3
"""Unet3D denoise-steps/sec on MI355X (BASELINE.json metric).

One step = one pass of the hot path over one batch: VideoDecoderTrainer
(video, unet_number=1) + update(1), i.e. p_losses forward + backward of unet1
(dim 64, mults 1/2/4/8) on a synthetic 16x64x64 clip batch of 4 per GPU, the
RCCL gradient all-reduce (N>1) and the fused AdamW update — bf16 activations,
f32 master weights.  Weights: deterministic non-zero fill; data: synthetic
U[0,1] clips resident in HBM.

  python bench.py --gpus N --steps K --warmup W      (N>1 under torch.distributed.run)

Rank 0 prints ONE JSON line.  Extra objects: `roofline` (dominant kernel,
timed live with HIP events on its launch stream) and `cpu_baseline` (the f32
CPU oracle timed on the host cores, rank 0 at N=1 only).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "dalle2-video_amd"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "Unet3D denoise-steps/sec, 16f×64×64 clip bs=4; 1/2/4/8 MI355X"
PEAK_BF16_TFLOPS = 2516.6   # MI355X dense bf16 MFMA (MI355X_MICROARCH.md)
PEAK_F32_TFLOPS = 157.3
STEP_TFLOP = 3.491          # ~3x the 1,163.6 GFLOP forward contractions


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--frames", type=int, default=16)
    ap.add_argument("--size", type=int, default=64)
    ap.add_argument("--dtype", choices=("bf16", "fp32"), default="bf16")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-roofline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--no-graphs", action="store_true",
                    help="launch every kernel eagerly instead of replaying the captured HIP graph")
    return ap.parse_args()


def build(args, device):
    from dalle2_video.dalle2_video import Unet3D, VideoDecoder
    from dalle2_video.trainer import VideoDecoderTrainer
    from dalle2_video.utils import deterministic_fill_

    unet = Unet3D(dim=64, video_embed_dim=512, channels=3, dim_mults=(1, 2, 4, 8),
                  cond_on_text_encodings=False)
    dec = VideoDecoder(unet=(unet,), frame_sizes=(args.size,), frame_numbers=(args.frames,),
                       timesteps=1000, learned_variance=False)
    deterministic_fill_(dec.unets[0])
    dec = dec.to(device)
    trainer = VideoDecoderTrainer(dec, lr=3e-4, wd=1e-2, use_ema=False, amp=args.dtype == "bf16",
                                  use_graphs=not getattr(args, "no_graphs", False))
    return dec, trainer


def cpu_baseline(args):
    """f32 CPU oracle (reference-equivalent op graph) — one timed train step."""
    from oracle import dv_ref as R
    from dalle2_video.utils import deterministic_fill_

    threads = min(args.cpu_threads, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    u = R.Unet3D(64, video_embed_dim=512, channels=3, dim_mults=(1, 2, 4, 8))
    deterministic_fill_(u)
    sched = R.NoiseScheduler(beta_schedule="cosine", timesteps=1000, loss_type="l2")
    opt = R.get_optimizer(u.parameters(), lr=3e-4, wd=1e-2)
    g = torch.Generator().manual_seed(1234)
    x = torch.rand(args.batch, 3, args.frames, args.size, args.size, generator=g)
    t = torch.randint(0, 1000, (args.batch,), generator=g)
    noise = torch.randn(x.shape, generator=g)
    R.train_step(u, sched, opt, x, t, noise)  # warm-up
    n = 2
    t0 = time.perf_counter()
    for _ in range(n):
        R.train_step(u, sched, opt, x, t, noise)
    dt = (time.perf_counter() - t0) / n
    return {"value": round(1.0 / dt, 5), "unit": "denoise-steps/s", "cores": threads, "kind": "port",
            "sample": f"{n} timed train steps (p_losses fwd+bwd+AdamW, f32) of the CPU oracle at "
                      f"{args.frames}x{args.size}x{args.size} bs={args.batch} after 1 warm-up step "
                      f"({dt:.2f} s each)"}


def kernel_key(name):
    """(identifier, integer template args) of a mangled / demangled kernel name
    or of a bench label such as 'conv_fwd_glds_kernel<64,128,6>'."""
    import re
    if name.startswith("_Z"):
        m = re.search(r"_GLOBAL__N_1", name)
        rest = name[m.end():] if m else re.sub(r"^_ZN?", "", name)
        n = re.match(r"(\d+)", rest)
        if n:
            ln = int(n.group(1))
            base = rest[len(n.group(1)):len(n.group(1)) + ln]
            targs = rest[len(n.group(1)) + ln:]
            ints = tuple(int(v) for v in re.findall(r"Li(\d+)E", targs.split("EEv")[0] + "E")) \
                if targs.startswith("I") else ()
            return base, ints
    name = name.replace("void ", "").replace("(anonymous namespace)::", "").strip()
    m = re.match(r"([A-Za-z_]\w*)(<([^>]*)>)?", name)
    if not m:
        return name, ()
    ints = tuple(int(t.strip()) for t in (m.group(3) or "").split(",") if re.fullmatch(r"\s*-?\d+\s*", t))
    return m.group(1), ints


def pmc_traffic(name):
    """HBM bytes per launch of kernel `name` from the newest committed PMC
    summary (profiles/pmc_traffic_*.json, made by tools/pmc_traffic.py from
    rocprofv3 FETCH_SIZE / WRITE_SIZE passes of this bench), or None."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "pmc_traffic_*.json")))
    if not files:
        return None
    table = json.load(open(files[-1]))
    want = kernel_key(name)
    for k, v in table.items():
        if kernel_key(k) == want:
            return v.get("traffic_bytes")
    return None


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    device = torch.device("cuda", local)
    torch.manual_seed(1234 + rank)

    dec, trainer = build(args, device)
    g = torch.Generator(device=device).manual_seed(1234 + rank)
    video = torch.rand(args.batch, 3, args.frames, args.size, args.size, device=device, generator=g)
    embed = torch.randn(args.batch, 512, device=device, generator=g)

    def step():
        trainer(video_embed=embed, video=video, unet_number=1)
        trainer.update(1)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        te = torch.tensor([elapsed], device=device)
        dist.all_reduce(te, op=dist.ReduceOp.MAX)
        elapsed = te.item()

    roof = None
    kernels = None
    attention = None
    if not args.no_roofline:
        # live per-launch HIP-event timing of every conv kernel over K more steps
        from dalle2_video import ops
        ops.TIMER = ops.KernelTimer()
        for _ in range(max(2, min(args.steps, 5))):
            step()
        summ = ops.TIMER.summary()
        event_ovh_us = ops.TIMER.event_overhead_ms * 1e3
        ops.TIMER = None
        name, d = max(summ.items(), key=lambda kv: kv[1]["ms"])
        peak = PEAK_BF16_TFLOPS if args.dtype == "bf16" else PEAK_F32_TFLOPS
        avg_ms = d["ms"] / d["count"]
        achieved = d["flops"] / (d["ms"] * 1e-3) / 1e12
        traffic = pmc_traffic(name)
        roof = {"bound": "mfma", "kernel": name, "achieved": round(achieved, 1), "peak": peak,
                "unit": "TFLOP/s", "frac": round(achieved / peak, 4),
                "traffic": None if traffic is None else round(traffic),
                "traffic_unit": "bytes/launch (2*FETCH_SIZE + WRITE_SIZE, PMC)",
                "algorithmic_bytes_per_launch": round(d["bytes"] / d["count"]),
                "launches_per_step": d["count"] // max(2, min(args.steps, 5)),
                "event_overhead_us_subtracted": round(event_ovh_us, 2),
                "avg_launch_us": round(avg_ms * 1e3, 2),
                "algorithmic_flop_per_launch": round(d["flops"] / d["count"])}
        kernels = {k: {"ms_per_step": round(v["ms"] / max(2, min(args.steps, 5)), 3),
                       "tflops": round(v["flops"] / (v["ms"] * 1e-3) / 1e12, 1)}
                   for k, v in sorted(summ.items(), key=lambda kv: -kv[1]["ms"])}
        # north-star sub-metric: mid-attention QK^T/PV (fwd + bwd) vs the bf16 MFMA peak
        att = [v for k, v in summ.items() if k.startswith("attn:")]
        if att:
            fl = sum(v["flops"] for v in att)
            ms = sum(v["ms"] for v in att)
            nrep = max(2, min(args.steps, 5))
            attention = {"kernels": "mqa_fwd + mqa_bwd (mid self-attention, 16 heads x 32, 1,025 keys)",
                         "flop_per_step": round(fl / nrep), "ms_per_step": round(ms / nrep, 4),
                         "achieved": round(fl / (ms * 1e-3) / 1e12, 1), "peak": peak,
                         "unit": "TFLOP/s", "frac": round(fl / (ms * 1e-3) / 1e12 / peak, 4)}

    base = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        base = cpu_baseline(args)

    if rank == 0:
        sps = args.steps / elapsed  # per GPU
        value = world * sps
        out = {
            "metric": METRIC, "value": round(value, 3), "unit": "denoise-steps/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(1e3 / sps, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": args.dtype, "data": "synthetic",
            "config": {"workload": "unet1 train step: p_losses fwd+bwd + RCCL grad all-reduce + fused AdamW",
                       "clip": [args.frames, args.size, args.size], "batch_per_gpu": args.batch,
                       "global_batch": args.batch * world, "parallelism": f"dp{world}"},
            "step_tflops_algorithmic": round(STEP_TFLOP * sps, 1),
            "roofline": roof, "attention": attention, "cpu_baseline": base, "kernels": kernels,
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
