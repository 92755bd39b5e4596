"""One rank of tests/test_dp_trainer_gpu.py: the real VideoDecoderTrainer
(__call__ + update, HIP-graph capture on) under torch.distributed (gloo, every
rank on cuda:0), training on its rank-strided share of one fixed global batch.

  python tests/dp_trainer_worker.py OUT_DIR WORLD RANK PORT [BACKEND]

BACKEND gloo (default) or nccl (one rank only on the one-GPU box: with
DV_FORCE_ALLREDUCE=1 the trainer's overlapped all-reduce then runs on a
one-rank RCCL communicator, captured into the HIP graph).
DV_TEST_ACCUM=2: two trainer calls per update (gradient accumulation; the
second call uses the next step's data).  DV_TEST_GRAPHS=0: no graph capture
(every call eager, so every call after the first two overlaps its buckets).

The decoder's two random draws — `times` (torch.randint, reference
dalle2_video.py:2229) and `noise` (torch.randn_like in p_losses, :1946) — are
injected: this rank's slice of one global (times, noise) pair, so the world-N
run and the world-1 run see the same per-sample inputs.  Writes per-step
losses, the step-0 local gradient, the flat parameters after the last update,
and the parameters after the init broadcast to OUT_DIR/w{WORLD}_r{RANK}.pt.
"""
import os

import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "dalle2-video_amd"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

GLOBAL_B, T, S, STEPS = 4, 4, 32, 5


def main():
    out_dir, world, rank, port = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
    backend = sys.argv[5] if len(sys.argv) > 5 else "gloo"
    torch.cuda.set_device(0)
    if world > 1 or backend == "nccl":
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = port
        if backend == "nccl":
            dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", 0))
        else:
            dist.init_process_group("gloo", rank=rank, world_size=world)
    from dalle2_video.dalle2_video import Unet3D, VideoDecoder
    from dalle2_video.trainer import VideoDecoderTrainer
    from dalle2_video.utils import deterministic_fill_

    u = Unet3D(16, video_embed_dim=512, channels=3, dim_mults=(1, 2, 4, 8))
    dec = VideoDecoder(unet=(u,), frame_sizes=(S,), frame_numbers=(T,), timesteps=1000, learned_variance=False)
    deterministic_fill_(dec.unets[0])
    if rank > 0:  # different local init: the trainer's init broadcast must replace it
        with torch.no_grad():
            for p in dec.unets[0].parameters():
                p.mul_(1.5)
    dec = dec.cuda()
    accum = int(os.environ.get("DV_TEST_ACCUM", "1"))
    tr = VideoDecoderTrainer(dec, lr=3e-4, wd=1e-2, use_ema=False,
                             use_graphs=os.environ.get("DV_TEST_GRAPHS", "1") == "1")
    init = torch.cat([p.detach().reshape(-1) for p in dec.unets[0].parameters()]).cpu()

    g = torch.Generator().manual_seed(2024)
    per = GLOBAL_B // world
    sl = slice(rank * per, (rank + 1) * per)
    video_all = torch.rand(STEPS, GLOBAL_B, 3, T, S, S, generator=g)
    times_all = torch.randint(0, 1000, (STEPS, GLOBAL_B), generator=g)
    noise_all = torch.randn(STEPS, GLOBAL_B, 3, T, S, S, generator=g)
    # fixed device buffers (a captured graph reads them at their addresses)
    video_d = video_all[0, sl].cuda()
    times_d = times_all[0, sl].cuda()
    noise_d = noise_all[0, sl].cuda()
    real_randint, real_randn_like = torch.randint, torch.randn_like

    def randint(low, high, size, *a, **k):
        if tuple(size) == (per,) and high == 1000:
            return times_d
        return real_randint(low, high, size, *a, **k)

    def randn_like(x, *a, **k):
        if x.shape == noise_d.shape:
            return noise_d
        return real_randn_like(x, *a, **k)

    torch.randint, torch.randn_like = randint, randn_like
    losses, grad0 = [], None
    opt = tr.optim0
    for s in range(STEPS):
        for a in range(accum):
            src = (s + a) % STEPS
            video_d.copy_(video_all[src, sl])
            times_d.copy_(times_all[src, sl])
            noise_d.copy_(noise_all[src, sl])
            losses.append(tr(video=video_d, unet_number=1))
        if s == 0:
            grad0 = torch.cat([p.grad.detach().reshape(-1) for p in dec.unets[0].parameters()
                               if p.grad is not None]).cpu()
        tr.update(1)
    torch.cuda.synchronize()
    graphed = any("graph" in v for v in tr._graphs.values())
    overlapped = any(v.get("overlapped", False) for v in tr._graphs.values())
    params = torch.cat([p.detach().reshape(-1) for p in dec.unets[0].parameters()]).cpu()
    torch.save(dict(losses=losses, grad0=grad0, params=params, init=init, graphed=graphed, per=per,
                    overlapped=overlapped, buckets=0 if tr.overlap is None else len(tr.overlap[0]._buckets())),
               os.path.join(out_dir, f"w{world}_r{rank}_{backend}_a{accum}.pt"))
    if dist.is_initialized():
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
