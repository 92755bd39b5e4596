#!/usr/bin/env python3
"""Unet3D denoise-steps/sec on MI355X (BASELINE.json metric).

One step = one pass of the hot path over one batch (BASELINE config 2):
VideoDecoderTrainer(video, unet_number=1) + update(1), i.e. p_losses forward +
backward of unet1 (dim 64, mults 1/2/4/8) on a synthetic 16x64x64 clip batch
of 4 per GPU, the RCCL gradient all-reduce (N>1) and the fused AdamW update —
bf16 activations, f32 master weights.  Weights: deterministic non-zero fill;
data: synthetic U[0,1] clips resident in HBM.

  python bench.py --gpus N --steps K --warmup W      (N>1 under torch.distributed.run)

Rank 0 prints ONE JSON line.  Extra objects:
  roofline      dominant kernel (HIP events on its launch stream, live)
  conv_shapes   the same per (kernel, GEMM shape) — the actionable rows
  attention     mid MQA QK^T/PV fwd+bwd vs the bf16 MFMA peak (north-star target)
  fp32          the same training step in the reference's f32 arithmetic
  config3       BASELINE config 3's alternating unet1 + unet2 training step (1 GPU)
  sampling      DDPM denoise steps (one Unet3D forward + posterior update,
                HIP-graph replay) at 16x64x64 bs=4 and bs=1, and the config-4
                cascade (base 16x64x64 + SR unet2 to 256x256, 250 steps each)
  cpu_baseline  the f32 CPU oracle on the host cores (rank 0 at N=1 only)
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
PEAK_FP8_TFLOPS = 5033.2    # dense MX-fp8 MFMA, 2x bf16 per clock (MI355X_MICROARCH.md)
PEAK_HBM_TBS = 8.0          # MI355X HBM3E (MI355X_MICROARCH.md)
STEP_TFLOP = 3.491          # ~3x the 1,163.6 GFLOP forward contractions
FWD_TFLOP = 1.1636          # Cfg2 forward contractions (bs=4)


def log(*a):
    """Progress on stderr (stdout carries only the JSON line)."""
    print(f"[bench {time.strftime('%H:%M:%S')}]", *a, file=sys.stderr, flush=True)


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
    ap.add_argument("--cpu-threads", type=int, default=0,
                    help="CPU-baseline threads (0: torch's default, i.e. OMP_NUM_THREADS = this "
                         "process's CPU share: 16 per GPU on the MI355X box, whose sched_getaffinity "
                         "lists all 256 host CPUs)")
    ap.add_argument("--no-graphs", action="store_true",
                    help="launch every kernel eagerly instead of replaying the captured HIP graph")
    ap.add_argument("--no-sampling", action="store_true")
    ap.add_argument("--no-fp32", action="store_true")
    ap.add_argument("--no-config3", action="store_true")
    ap.add_argument("--sample-steps", type=int, default=250,
                    help="DDPM steps of the sampling legs (config 4: 250)")
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
    """f32 CPU oracle (reference-equivalent op graph, oracle/dv_ref.py) on the
    host cores: median of 3 Cfg2 train steps (p_losses fwd+bwd+clip+AdamW)
    after 1 warm-up, and the config-1 forward (1x3x8x32x32) median of 5."""
    import statistics
    from oracle import dv_ref as R
    from dalle2_video.utils import deterministic_fill_

    threads = args.cpu_threads or torch.get_num_threads()
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
    times = []
    for _ in range(3):
        t0 = time.perf_counter()
        R.train_step(u, sched, opt, x, t, noise)
        times.append(time.perf_counter() - t0)
        log(f"cpu train step {times[-1]:.2f} s")
    dt = statistics.median(times)
    # config 1: a single Unet3D forward on an 8-frame 32x32 clip, bs=1
    x1 = torch.randn(1, 3, 8, 32, 32, generator=g)
    t1 = torch.randint(0, 1000, (1,), generator=g)
    with torch.no_grad():
        u(x1, t1)
        f1 = []
        for _ in range(5):
            t0 = time.perf_counter()
            u(x1, t1)
            f1.append(time.perf_counter() - t0)
    return {"value": round(1.0 / dt, 5), "unit": "denoise-steps/s", "cores": threads, "kind": "port",
            "sample": f"median of 3 timed train steps (p_losses fwd+bwd+clip+AdamW, f32) of the CPU "
                      f"oracle at {args.frames}x{args.size}x{args.size} bs={args.batch} after 1 warm-up "
                      f"step ({dt:.2f} s each; {[round(v, 2) for v in times]})",
            "config1_forward_s": round(statistics.median(f1), 4),
            "config1_sample": "config 1 (BASELINE configs[0]): Unet3D forward, random 1x3x8x32x32 clip, "
                              "median of 5 after 1 warm-up"}


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
    # the timed label may name fewer template arguments than the profiled
    # instantiations (conv_fwd_frame_kernel<8> covers <8,3,1,64> and
    # <8,3,1,32>): their dispatch-weighted mean
    tot = n = 0
    for k, v in table.items():
        kk = kernel_key(k)
        if kk[0] == want[0] and kk[1][:len(want[1])] == want[1] and v.get("traffic_bytes") is not None:
            d = v.get("dispatches", 1)
            tot += v["traffic_bytes"] * d
            n += d
    return tot / n if n else None


def fp32_leg(args, device):
    """The same training step in the reference's arithmetic (f32 activations,
    exact f32 MFMA): 3 warm-up + 5 timed steps."""
    import copy
    a = copy.copy(args)
    a.dtype = "fp32"
    dec, trainer = build(a, device)
    g = torch.Generator(device=device).manual_seed(4321)
    video = torch.rand(a.batch, 3, a.frames, a.size, a.size, device=device, generator=g)

    def step():
        trainer(video=video, unet_number=1)
        trainer.update(1)

    for _ in range(3):
        step()
    torch.cuda.synchronize()
    n = 5
    t0 = time.perf_counter()
    for _ in range(n):
        step()
    torch.cuda.synchronize()
    sps = n / (time.perf_counter() - t0)
    del dec, trainer
    return {"value": round(sps, 3), "unit": "denoise-steps/s", "dtype": "fp32", "steps": n,
            "ms_per_step": round(1e3 / sps, 3),
            "mfma_frac": round(STEP_TFLOP * sps / PEAK_F32_TFLOPS, 4),
            "peak": PEAK_F32_TFLOPS, "note": "f32 activations and f32 MFMA (v_mfma_f32_32x32x2f32); "
                                             "frac against the dense f32 MFMA peak"}


def forward_flops(unet, shape, device, lowres=None, batch=None):
    """Algorithmic contraction FLOPs of one no-grad Unet3D forward: the sum of
    the conv / attention FLOPs the ops report to the kernel timer (2*M*N*K per
    conv at its unpadded shape; QK^T + PV for the mid attention).  The folded
    cross-attention projections are not counted, so fractions built on it
    are lower bounds."""
    from dalle2_video import ops
    b, c, t, h, w = shape
    x = torch.randn(*shape, device=device)
    tt = torch.full((b,), 500, device=device, dtype=torch.long)
    ops.TIMER = ops.KernelTimer()
    try:
        with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16), ops.private_pack_cache():
            kw = {} if lowres is None else {"lowres_cond_video": torch.rand(b, c, t, h, w, device=device)}
            unet(x, tt, **kw)
        torch.cuda.synchronize()
        return sum(r[2] for r in ops.TIMER.records)
    finally:
        ops.TIMER = None


def config3_leg(args, device):
    """BASELINE config 3 on one GPU: the reference's alternating training step
    (train_decoder.py:127-138): trainer(unet 1) + update(1), then trainer(unet 2)
    + update(2), on synthetic 224x224 CelebV-Text-shape clips (bs 4 x 16
    frames) that VideoDecoder.forward resizes to 64^2 / 128^2; unet2 (dim 8,
    mults 1..16) is low-res conditioned (64^2 -> 128^2, kornia blur with
    p = 0.5 drawn per call).  Both unets' calls replay captured HIP graphs (one
    per blur decision for unet2).  N>1 of this config is the driver's scaling
    run of the same trainer (bench main leg)."""
    import random
    from dalle2_video.dalle2_video import Unet3D, VideoDecoder
    from dalle2_video.trainer import VideoDecoderTrainer
    from dalle2_video.utils import deterministic_fill_

    random.seed(1234)
    u1 = Unet3D(64, video_embed_dim=512, channels=3, dim_mults=(1, 2, 4, 8), cond_on_text_encodings=False)
    u2 = Unet3D(8, video_embed_dim=512, channels=3, dim_mults=(1, 2, 4, 8, 16), cond_on_text_encodings=False)
    dec = VideoDecoder(unet=(u1, u2), frame_sizes=(64, 128), frame_numbers=(args.frames, args.frames),
                       timesteps=1000, learned_variance=False)
    for un in dec.unets:
        deterministic_fill_(un)
    dec = dec.to(device)
    tr = VideoDecoderTrainer(dec, lr=3e-4, wd=1e-2, use_ema=False, amp=True, use_graphs=True)
    g = torch.Generator(device=device).manual_seed(99)
    video = torch.rand(args.batch, 3, args.frames, 224, 224, device=device, generator=g)
    emb = torch.randn(args.batch, 512, device=device, generator=g)
    t_unet = [0.0, 0.0]

    def pair(timed=False):
        for un in (1, 2):
            if timed:
                torch.cuda.synchronize()
                t0 = time.perf_counter()
            tr(video_embed=emb, video=video, unet_number=un)
            tr.update(un)
            if timed:
                torch.cuda.synchronize()
                t_unet[un - 1] += time.perf_counter() - t0

    for _ in range(12):  # every graph (unet1, unet2 x 2 blur decisions) captured
        pair()
    torch.cuda.synchronize()
    n = 20
    t0 = time.perf_counter()
    for _ in range(n):
        pair()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    for _ in range(5):  # per-unet split (synchronised calls)
        pair(timed=True)
    n_graphs = len(tr._graphs)
    fl1 = STEP_TFLOP * 1e12
    fl2 = 3.0 * forward_flops(dec.unets[1], (args.batch, 3, args.frames, 128, 128), device, lowres=True)
    rate = n / dt
    achieved = (fl1 + fl2) * rate / 1e12
    out = {"config": "BASELINE config 3 (1 GPU): alternating unet1 (64^2) + update(1), unet2 (128^2, low-res "
                     f"conditioned, blur p=0.5) + update(2); {args.batch}x3x{args.frames}x224x224 synthetic clips, "
                     "bf16, HIP-graph replay",
           "value": round(rate, 3), "unit": "alternating steps/s (one unet1 + one unet2 training step each)",
           "ms_per_pair": round(1e3 / rate, 3), "pairs": n, "graphs_captured": n_graphs,
           "unet1_ms": round(t_unet[0] / 5 * 1e3, 3), "unet2_ms": round(t_unet[1] / 5 * 1e3, 3),
           "roofline": {"bound": "mfma", "achieved": round(achieved, 1), "peak": PEAK_BF16_TFLOPS,
                        "unit": "TFLOP/s", "frac": round(achieved / PEAK_BF16_TFLOPS, 4),
                        "flop_per_pair": f"{(fl1 + fl2) / 1e12:.4f}e12 (unet1 {STEP_TFLOP} + unet2 3 x timed "
                                         f"forward contractions {fl2 / 3e12:.4f})"}}
    del tr, dec
    return out


def sampling_leg(args, device):
    """DDPM sampling (p_sample_loop_ddpm, dalle2_video.py:1667-1755): every
    denoise step is one Unet3D forward + the posterior update, replayed from
    one captured HIP graph.  Times whole sample() calls (including the two
    eager steps and the capture), bf16 autocast."""
    from dalle2_video.dalle2_video import Unet3D, VideoDecoder
    from dalle2_video.utils import deterministic_fill_

    T = args.sample_steps
    out = {"steps_per_loop": T, "dtype": "bf16", "unit": "denoise-steps/s",
           "step": "one Unet3D forward + p_sample update (HIP-graph replay)"}
    u = Unet3D(64, video_embed_dim=512, channels=3, dim_mults=(1, 2, 4, 8))
    dec = VideoDecoder(unet=(u,), frame_sizes=(args.size,), frame_numbers=(args.frames,),
                       timesteps=T, learned_variance=False)
    deterministic_fill_(dec.unets[0])
    dec = dec.to(device)
    for bs in (args.batch, 1):
        emb = torch.randn(bs, 512, device=device)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            dec.sample(video_embed=emb, one_unet_in_gpu_at_time=False)  # warm-up loop
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            vid = dec.sample(video_embed=emb, one_unet_in_gpu_at_time=False)
            torch.cuda.synchronize()
            dt = time.perf_counter() - t0
        assert torch.isfinite(vid).all(), "non-finite sample"
        sps = T / dt
        log(f"sampling bs={bs}: {sps:.1f} steps/s ({dt:.2f} s per {T}-step loop)")
        fl = FWD_TFLOP * bs / 4
        out[f"bs{bs}"] = {"value": round(sps, 2), "loop_s": round(dt, 3),
                          "clip": [args.frames, args.size, args.size],
                          "roofline": {"bound": "mfma", "achieved": round(fl * sps, 1),
                                       "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s",
                                       "frac": round(fl * sps / PEAK_BF16_TFLOPS, 4),
                                       "flop_per_step": f"{fl:.4f}e12 (Cfg2 forward x bs/4)"}}
    del dec, u
    # config 5 shape: unet1 on a 32-frame 128x128 clip, bs=2 — the mid attention
    # runs over 32 x 16 x 16 = 8,192 tokens (K/V-streamed flash kernel).  The
    # per-step rate is differential — two sample() calls of T5A and T5B steps,
    # (T5B - T5A) / (t_B - t_A) — so the per-call constant (the denoise-step
    # graph capture and the weight images of a fresh sampling cache) is not
    # spread over a short loop; est_1000_step_s adds it back once.
    T5A, T5B = 8, 24
    u = Unet3D(64, video_embed_dim=512, channels=3, dim_mults=(1, 2, 4, 8))
    # VideoDecoder rebuilds the unet it is given (cast_model_parameters, quirk
    # Q3: a fresh instance, as the reference's Decoder): the first decoder's unet
    # is the one filled and timed, and the second decoder is pointed at it
    d0 = VideoDecoder(unet=(u,), frame_sizes=(128,), frame_numbers=(32,), timesteps=T5A,
                      learned_variance=False)
    u = d0.unets[0]
    deterministic_fill_(u)
    d1 = VideoDecoder(unet=(u,), frame_sizes=(128,), frame_numbers=(32,), timesteps=T5B,
                      learned_variance=False)
    d1.unets[0] = u
    decs = [d0.to(device), d1.to(device)]
    assert next(u.parameters()).is_cuda
    emb = torch.randn(2, 512, device=device)
    from dalle2_video import ops

    def loop_rate():
        ts = []
        with torch.autocast("cuda", dtype=torch.bfloat16):
            for dec in decs:
                dec.sample(video_embed=emb, one_unet_in_gpu_at_time=False)
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                vid = dec.sample(video_embed=emb, one_unet_in_gpu_at_time=False)
                torch.cuda.synchronize()
                ts.append(time.perf_counter() - t0)
                assert torch.isfinite(vid).all()
        step = (ts[1] - ts[0]) / (T5B - T5A)
        return step, ts[0] + (1000 - T5A) * step, ts

    def timed_forward(fp8_attention=False):
        u.fp8_attention = fp8_attention
        ops.TIMER = ops.KernelTimer()
        with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16), ops.private_pack_cache():
            xin = torch.randn(2, 3, 32, 128, 128, device=device)
            tin = torch.full((2,), 500, device=device, dtype=torch.long)
            u(xin, tin)  # packs the weight images of this cache
            ops.TIMER.records.clear()
            u(xin, tin)
        summ = ops.TIMER.summary()
        ops.TIMER = None
        u.fp8_attention = False
        return summ

    step16, est16, ts16 = loop_rate()
    summ = timed_forward()
    att = summ.get("attn:mqa_fwd")
    fl5 = FWD_TFLOP * (2 * 32 * 128 * 128) / (4 * 16 * 64 * 64)
    out["config5_bf16"] = {
        "config": "BASELINE config 5 shape, bf16 (not fp8): unet1 sampling, 32x128x128 clip, bs=2; "
                  f"per-step rate from {T5A}- and {T5B}-step DDPM loops (per-step cost is schedule-independent)",
        "value": round(1 / step16, 2), "unit": "denoise-steps/s",
        "est_1000_step_s": round(est16, 1), "loops_s": [round(t, 3) for t in ts16],
        "roofline": {"bound": "mfma", "achieved": round(fl5 / step16, 1), "peak": PEAK_BF16_TFLOPS,
                     "unit": "TFLOP/s", "frac": round(fl5 / step16 / PEAK_BF16_TFLOPS, 4),
                     "flop_per_step": f"{fl5:.3f}e12 (Cfg2 forward x 4 pixels ratio)"},
        "mid_attention": None if att is None else {
            "tokens": 8192, "us": round(att["ms"] / att["count"] * 1e3, 1),
            "tflops": round(att["flops"] / (att["ms"] * 1e-3) / 1e12, 1),
            "frac": round(att["flops"] / (att["ms"] * 1e-3) / 1e12 / PEAK_BF16_TFLOPS, 4)},
    }
    log(f"config5 bf16: {1 / step16:.2f} steps/s")
    # the same loops with the MX-fp8 convs (Unet3D.fp8: e4m3 operands with a
    # power-of-two scale per 32 channels on v_mfma_scale_f32_32x32x64_f8f6f4);
    # the mid attention stays on the bf16 bounded-score kernel (the fp8-PV
    # kernel measured slower: its opt-in A/B is `mid_attention_fp8` below)
    u.fp8 = True
    step8, est8, ts8 = loop_rate()
    summ8 = timed_forward()
    summ8a = timed_forward(fp8_attention=True)
    u.fp8 = False
    mx = {k: v for k, v in summ8.items() if k.startswith("conv_fwd_mx8")}
    kname, kd = max(mx.items(), key=lambda kv: kv[1]["ms"])
    k_tf = kd["flops"] / (kd["ms"] * 1e-3) / 1e12
    # the mid attention with PV in MX-fp8 (dv_mqa_fwd_fp8) against the bf16
    # streamed kernel of the bf16 leg, same process / box; half its FLOPs (QK^T)
    # stay bf16, so the peak is the harmonic blend of the two MFMA peaks
    att8 = summ8a.get("attn:mqa_fwd8")
    mid8 = None
    if att8 is not None:
        a8_us = att8["ms"] / att8["count"] * 1e3
        a8_tf = att8["flops"] / (att8["ms"] * 1e-3) / 1e12
        blend = 2.0 / (1.0 / PEAK_BF16_TFLOPS + 1.0 / PEAK_FP8_TFLOPS)
        mid8 = {"tokens": 8192, "us": round(a8_us, 1), "tflops": round(a8_tf, 1),
                "bf16_us": None if att is None else round(att["ms"] / att["count"] * 1e3, 1),
                "speedup_vs_bf16": None if att is None else round(att["ms"] / att["count"] * 1e3 / a8_us, 3),
                "roofline": {"bound": "mfma", "achieved": round(a8_tf, 1), "peak": round(blend, 1),
                             "unit": "TFLOP/s", "frac": round(a8_tf / blend, 4),
                             "frac_of_fp8_peak": round(a8_tf / PEAK_FP8_TFLOPS, 4),
                             "note": "QK^T bf16 + PV MX-fp8 (v_mfma_scale_f32_32x32x64_f8f6f4); peak = harmonic "
                                     "blend of the dense bf16 and fp8 peaks (half the FLOPs each)"}}
    out["config5_fp8"] = {
        "config": "BASELINE config 5: unet1 sampling, 32x128x128 clip, bs=2, every 3x3 conv with cin, cout % 64 == 0 "
                  "in MX-fp8 (e4m3 + e8m0 per 32 channels), the mid attention bf16 (its fp8-PV form is "
                  "an opt-in A/B: mid_attention_fp8); "
                  f"per-step rate from {T5A}- and {T5B}-step DDPM loops",
        "value": round(1 / step8, 2), "unit": "denoise-steps/s", "speedup_vs_bf16": round(step16 / step8, 3),
        "est_1000_step_s": round(est8, 1), "loops_s": [round(t, 3) for t in ts8],
        "fp8_convs_per_step": sum(v["count"] for v in mx.values()),
        "roofline": {"bound": "mfma", "kernel": kname, "achieved": round(k_tf, 1), "peak": PEAK_FP8_TFLOPS,
                     "unit": "TFLOP/s", "frac": round(k_tf / PEAK_FP8_TFLOPS, 4),
                     "avg_launch_us": round(kd["ms"] / kd["count"] * 1e3, 2),
                     "note": "dominant MX-fp8 conv kernel, HIP events per launch; peak = dense MX-fp8 MFMA"},
        "kernels_ms_per_step": {k: round(v["ms"], 3) for k, v in sorted(mx.items(), key=lambda kv: -kv[1]["ms"])},
        "mid_attention_fp8": mid8,  # Unet3D.fp8_attention (opt-in, not in `value`)
    }
    log(f"config5 fp8: {1 / step8:.2f} steps/s")
    del decs, u
    # config 4: two-stage cascade, base 16x64x64 + spatial-SR unet2 (dim 8, mults 1..16) to 256x256
    u1 = Unet3D(64, video_embed_dim=512, channels=3, dim_mults=(1, 2, 4, 8))
    u2 = Unet3D(8, video_embed_dim=512, channels=3, dim_mults=(1, 2, 4, 8, 16))
    dec = VideoDecoder(unet=(u1, u2), frame_sizes=(args.size, 256), frame_numbers=(args.frames, args.frames),
                       timesteps=T, learned_variance=False)
    for un in dec.unets:
        deterministic_fill_(un)
    dec = dec.to(device)
    emb = torch.randn(1, 512, device=device)
    log("cascade sampling ...")
    with torch.autocast("cuda", dtype=torch.bfloat16):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        vid = dec.sample(video_embed=emb)  # reference defaults: one unet on the GPU at a time
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
    assert vid.shape == (1, 3, args.frames, 256, 256) and torch.isfinite(vid).all()
    # per-step contraction FLOPs of each stage's forward (bs 1), both stages' loops
    dec.to(device)
    fc1 = forward_flops(dec.unets[0], (1, 3, args.frames, args.size, args.size), device)
    fc2 = forward_flops(dec.unets[1], (1, 3, args.frames, 256, 256), device, lowres=True)
    casc_tf = T * (fc1 + fc2) / dt / 1e12
    out["cascade"] = {"config": f"BASELINE config 4: base {args.frames}x{args.size}x{args.size} + SR to "
                                f"{args.frames}x256x256, bs=1, {T}-step DDPM per stage, one unet on the GPU "
                                "at a time (the reference's sample() default)",
                      "seconds": round(dt, 3), "value": round(2 * T / dt, 2),
                      "unit": "denoise-steps/s (both stages)",
                      "roofline": {"bound": "mfma", "achieved": round(casc_tf, 1), "peak": PEAK_BF16_TFLOPS,
                                   "unit": "TFLOP/s", "frac": round(casc_tf / PEAK_BF16_TFLOPS, 4),
                                   "flop_per_step": f"base {fc1 / 1e12:.4f}e12, SR {fc2 / 1e12:.4f}e12 (timed "
                                                    "forward contractions, bs 1)",
                                   "note": "whole sample() call incl. one-unet-at-a-time host moves and the "
                                           "per-stage graph captures"}}
    del dec
    return out


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # DV_DIST_BACKEND=gloo + DV_SHARE_GPU=1: rehearse the N-rank path with every
    # rank on the same GPU (a one-GPU box cannot run RCCL ranks); the driver's
    # multi-GPU runs use the defaults (RCCL, one GPU per rank)
    backend = os.environ.get("DV_DIST_BACKEND", "nccl")
    if os.environ.get("DV_SHARE_GPU") == "1":
        local = local % torch.cuda.device_count()
    # DV_BENCH_PG=1 (+ DV_FORCE_ALLREDUCE=1): a one-rank process group, so the
    # N > 1 step (bucketed RCCL all-reduce captured with the backward) runs on
    # a one-GPU box
    if world > 1 or os.environ.get("DV_BENCH_PG") == "1":
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    device = torch.device("cuda", local)
    torch.manual_seed(1234 + rank)

    dec, trainer = build(args, device)
    g = torch.Generator(device=device).manual_seed(1234 + rank)
    video = torch.rand(args.batch, 3, args.frames, args.size, args.size, device=device, generator=g)
    embed = torch.randn(args.batch, 512, device=device, generator=g)

    def step():
        trainer(video_embed=embed, video=video, unet_number=1)
        trainer.update(1)

    # the trainer captures its HIP graph on the 4th call (the first update()
    # builds the flat gradient buffers, then two eager calls warm the pass):
    # with fewer warm-up steps the capture lands in the timed region
    if args.warmup < 4 and not args.no_graphs:
        log(f"warning: --warmup {args.warmup} < 4 times the graph capture (the 4th call) as a step")
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

    exposed = None
    if world > 1 and trainer.overlap is not None:
        # the all-reduce time the backward does not hide: eager steps (the same
        # bucket schedule the captured graph replays), from the end of the
        # backward's compute to the join of every bucket, max over ranks
        graphs, trainer.use_graphs = trainer.use_graphs, False
        trainer.comm_probe = []
        for _ in range(3):
            step()
        torch.cuda.synchronize()
        ex = [p[1].elapsed_time(p[2]) for p in trainer.comm_probe if p[0] == "exposed"]
        trainer.comm_probe, trainer.use_graphs = None, graphs
        t = torch.tensor([sorted(ex)[len(ex) // 2] if ex else -1.0], device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        exposed = round(t.item(), 3)

    roof = None
    kernels = None
    conv_shapes = None
    attention = None
    if not args.no_roofline:
        # live per-launch HIP-event timing of every conv kernel over K more steps
        from dalle2_video import ops
        ops.TIMER = ops.KernelTimer()
        for _ in range(max(2, min(args.steps, 5))):
            step()
        summ = ops.TIMER.summary()
        event_ovh_us = ops.TIMER.event_overhead_ms * 1e3
        name, d = max(summ.items(), key=lambda kv: kv[1]["ms"])
        peak = PEAK_BF16_TFLOPS if args.dtype == "bf16" else PEAK_F32_TFLOPS
        nrep = max(2, min(args.steps, 5))
        lps = d["count"] // nrep
        # frac: one step's launches of the dominant kernel replayed back to back
        # from a HIP graph (no event brackets; the kernel boundaries included),
        # the way the rocprofv3 kernel trace sees them
        rep_ms = ops.TIMER.replay_ms(name, lps)
        fl_launch = d["flops"] / d["count"]
        achieved = fl_launch / (rep_ms * 1e-3) / 1e12
        traffic = pmc_traffic(name)
        roof = {"bound": "mfma", "kernel": name, "achieved": round(achieved, 1), "peak": peak,
                "unit": "TFLOP/s", "frac": round(achieved / peak, 4),
                "method": "graph replay of one step's launches of the kernel, back to back, per launch",
                "avg_launch_us": round(rep_ms * 1e3, 2),
                "traffic": None if traffic is None else round(traffic),
                "traffic_unit": "bytes/launch (2*FETCH_SIZE + WRITE_SIZE, PMC)",
                "algorithmic_bytes_per_launch": round(d["bytes"] / d["count"]),
                "launches_per_step": lps,
                # per-launch HIP-event brackets (a device spin before each): the raw
                # bracket is an upper bound on the kernel (a lower-bound frac); minus
                # the empty-bracket cost it reads high (r04: 0.219 / 0.268 vs rocprof 0.253)
                "frac_events_raw": round(d["flops"] / (d["ms_raw"] * 1e-3) / 1e12 / peak, 4),
                "frac_events_minus_bracket": round(d["flops"] / (d["ms"] * 1e-3) / 1e12 / peak, 4),
                "event_bracket_us": round(event_ovh_us, 2),
                "algorithmic_flop_per_launch": round(fl_launch)}
        nrep = max(2, min(args.steps, 5))
        kernels = {k: {"ms_per_step": round(v["ms"] / nrep, 3),
                       "tflops": round(v["flops"] / (v["ms"] * 1e-3) / 1e12, 1)}
                   for k, v in sorted(summ.items(), key=lambda kv: -kv[1]["ms"])}
        # per (kernel, pass, M, N, K) rows: the roofline of every conv GEMM shape
        conv_shapes = []
        for (k, shp), v in sorted(ops.TIMER.summary(by_shape=True).items(), key=lambda kv: -kv[1]["ms"]):
            if shp is None:
                continue
            tf = v["flops"] / (v["ms"] * 1e-3) / 1e12
            tbs = v["bytes"] / (v["ms"] * 1e-3) / 1e12
            # bound by arithmetic intensity (algorithmic FLOP per algorithmic
            # byte: input read once, output written once) vs the ridge point
            hbm = v["flops"] / max(v["bytes"], 1.0) < peak / PEAK_HBM_TBS
            conv_shapes.append({"kernel": k, "pass": shp[0], "M": shp[1], "N": shp[2], "K": shp[3],
                                "launches_per_step": v["count"] // nrep,
                                "us_per_launch": round(v["ms"] / v["count"] * 1e3, 2),
                                "ms_per_step": round(v["ms"] / nrep, 3), "tflops": round(tf, 1),
                                "tbytes_per_s": round(tbs, 2), "bound": "hbm" if hbm else "mfma",
                                "frac": round(tbs / PEAK_HBM_TBS if hbm else tf / peak, 4)})
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
        ops.TIMER = None
        del summ

    log(f"train: {args.steps / elapsed:.2f} steps/s per GPU")
    fp32 = None
    if not args.no_fp32 and args.dtype == "bf16" and world == 1:
        # hand the cached blocks of the bf16 legs back first: on a cache the
        # bf16 step and the timer's closures have carved up, the f32 step ran
        # at 12.7-13.1 steps/s instead of 17.7-18.1 (r05, same box, same tree)
        import gc
        gc.collect()
        torch.cuda.empty_cache()
        fp32 = fp32_leg(args, device)
        log("fp32:", fp32["value"], "steps/s")
    sampling = None
    if not args.no_sampling and world == 1:
        sampling = sampling_leg(args, device)
    config3 = None
    if not args.no_config3 and world == 1:
        import gc
        gc.collect()
        torch.cuda.empty_cache()
        config3 = config3_leg(args, device)
        log(f"config3: {config3['value']} alternating steps/s")

    base = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        log("cpu baseline on", args.cpu_threads or torch.get_num_threads(), "threads")
        base = cpu_baseline(args)
        log("cpu baseline:", base["value"], "steps/s")

    if rank == 0:
        sps = args.steps / elapsed  # per GPU
        value = world * sps
        out = {
            "metric": METRIC, "value": round(value, 3), "unit": "denoise-steps/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(1e3 / sps, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": args.dtype, "data": "synthetic",
            "config": {"workload": f"BASELINE config 2: unet1 (dim 64, mults 1/2/4/8) train step on a "
                                   f"{args.frames}x{args.size}x{args.size} clip, bs={args.batch} per GPU: "
                                   "p_losses fwd+bwd + RCCL grad all-reduce + fused AdamW",
                       "clip": [args.frames, args.size, args.size], "batch_per_gpu": args.batch,
                       "global_batch": args.batch * world, "parallelism": f"dp{world}"},
            "step_tflops_algorithmic": round(STEP_TFLOP * sps, 1),
            # N > 1: median over 3 eager steps of the gradient all-reduce time left after the
            # backward's compute (overlapped buckets; max over ranks), ms
            "allreduce_exposed_ms": exposed,
            "roofline": roof, "cpu_baseline": base,
            # the bulky per-kernel tables first, the headline sub-results LAST:
            # the driver keeps the tail of stdout
            "kernels": kernels, "conv_shapes": conv_shapes[:24] if conv_shapes else None,
            "fp32": fp32, "sampling": sampling, "config3": config3, "attention": attention,
        }
        # one write (line and newline together): another rank's stderr merged
        # into the same pipe cannot land inside the line
        sys.stdout.write(json.dumps(out) + "\n")
        sys.stdout.flush()
    if dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
