"""Host-side logic of the drop-in package that runs without a GPU: module
wiring and state-dict layout identical to the oracle's (which is pinned to the
reference's, G2), the deterministic weight fill shared with the oracle, loud
failure of the compute path on CPU tensors (no fallback), and the trainer's
pure-Python helpers (optimizer grouping, warmup, EMA schedule, batch split).
"""
import math

import pytest
import torch

from oracle import dv_ref as R


def _both(dim, mults, lowres):
    from dalle2_video import dalle2_video as D

    out = []
    for mod in (R, D):
        u = mod.Unet3D(dim, video_embed_dim=512, channels=3, dim_mults=mults,
                       cond_on_text_encodings=False)
        out.append(u.cast_model_parameters(lowres_cond=lowres, lowres_noise_cond=False, channels=3,
                                           channels_out=3, cond_on_image_embeds=not lowres,
                                           cond_on_text_encodings=False))
    return out


@pytest.mark.parametrize("dim,mults,lowres,nkeys,nparams", [
    (64, (1, 2, 4, 8), False, 439, 49_967_171),
    (8, (1, 2, 4, 8, 16), True, 539, 4_203_412),
])
def test_state_dict_layout_matches_oracle(dim, mults, lowres, nkeys, nparams):
    o, p = _both(dim, mults, lowres)
    so, sp = o.state_dict(), p.state_dict()
    assert list(so.keys()) == list(sp.keys())
    assert len(sp) == nkeys
    assert all(so[k].shape == sp[k].shape for k in so)
    assert sum(t.numel() for t in p.parameters()) == nparams
    assert p.cond_on_video_embeds is False  # cast quirk: embed conditioning off
    p.load_state_dict(so, strict=True)


def test_deterministic_fill_identical_to_oracle():
    from dalle2_video.utils import deterministic_fill_

    o, p = _both(16, (1, 2, 4, 8), False)
    R.deterministic_fill_(o)
    deterministic_fill_(p)
    for (n, a), (_, b) in zip(o.named_parameters(), p.named_parameters()):
        assert torch.equal(a, b), n


def test_compute_path_fails_loudly_on_cpu():
    from dalle2_video import dalle2_video as D
    from dalle2_video._lib import DVError

    u = D.Unet3D(16, video_embed_dim=512, channels=3, dim_mults=(1, 2, 4, 8))
    x, t = torch.randn(1, 3, 4, 32, 32), torch.tensor([5])
    with pytest.raises(DVError, match="GPU only"):
        u(x, t)
    dec = D.VideoDecoder(u, frame_sizes=(32,), frame_numbers=(4,), timesteps=1000,
                         learned_variance=False)
    with pytest.raises(DVError):
        dec(x, unet_number=1)


def test_out_of_path_features_raise():
    from dalle2_video import dalle2_video as D

    u = D.Unet3D(16, video_embed_dim=512, channels=3, dim_mults=(1, 2, 4, 8))
    with pytest.raises(NotImplementedError):
        D.VideoDecoder(u, frame_sizes=(32,), frame_numbers=(4,), learned_variance=True)


def test_get_optimizer_groups_match_reference_rule():
    from dalle2_video.trainer import FusedAdamW, get_optimizer

    _, p = _both(16, (1, 2, 4, 8), False)
    opt = get_optimizer(p.parameters(), lr=3e-4, wd=1e-2)
    assert isinstance(opt, FusedAdamW)
    g0, g1 = opt.param_groups
    assert all(t.ndim >= 2 for t in g0["params"]) and g0["weight_decay"] == 1e-2
    assert all(t.ndim < 2 for t in g1["params"]) and g1["weight_decay"] == 0.0
    assert g0["betas"] == (0.9, 0.99) and g0["eps"] == 1e-8
    assert len(g0["params"]) + len(g1["params"]) == len(list(p.parameters()))
    opt0 = get_optimizer(p.parameters(), lr=1e-4, wd=0)
    assert len(opt0.param_groups) == 1 and opt0.param_groups[0]["weight_decay"] == 0.0


def test_linear_warmup_dampening():
    """pytorch_warmup.LinearWarmup semantics: step 0 is dampened at
    construction; each dampening() restores the undamped lr for the wrapped
    scheduler step and dampens the next step by min(1, (step+1)/period)."""
    from dalle2_video.trainer import _LinearWarmup

    opt = torch.optim.SGD([torch.nn.Parameter(torch.zeros(1))], lr=1.0)
    sched = torch.optim.lr_scheduler.LambdaLR(opt, lr_lambda=lambda s: 1.0)
    w = _LinearWarmup(opt, 4)
    lrs = [opt.param_groups[0]["lr"]]
    for _ in range(5):
        with w.dampening():
            sched.step()
        lrs.append(opt.param_groups[0]["lr"])
    assert lrs == [0.25, 0.5, 0.75, 1.0, 1.0, 1.0]


def test_linear_warmup_with_cosine_decay_does_not_compound():
    """Warmup composed with CosineAnnealingLR (trainer.py:75-87): the lr seen
    by each optimizer step is cosine(step) * warmup(step), never compounded."""
    from dalle2_video.trainer import _LinearWarmup

    base, period, tmax = 1e-4, 10, 100
    opt = torch.optim.SGD([torch.nn.Parameter(torch.zeros(1))], lr=base)
    sched = torch.optim.lr_scheduler.CosineAnnealingLR(opt, T_max=tmax)
    w = _LinearWarmup(opt, period)
    for step in range(40):
        want = base * 0.5 * (1 + math.cos(math.pi * step / tmax)) * min(1.0, (step + 1) / period)
        assert opt.param_groups[0]["lr"] == pytest.approx(want, rel=1e-9), step
        with w.dampening():
            sched.step()


def test_trainer_lr_follows_warmup_and_cosine_host_side():
    """VideoDecoderTrainer wires the same warmup/scheduler pair per unet."""
    from dalle2_video import dalle2_video as D
    from dalle2_video.trainer import VideoDecoderTrainer

    u = D.Unet3D(16, video_embed_dim=512, channels=3, dim_mults=(1, 2, 4, 8))
    dec = D.VideoDecoder(u, frame_sizes=(32,), frame_numbers=(4,), timesteps=1000, learned_variance=False)
    tr = VideoDecoderTrainer(dec, lr=3e-4, use_ema=False, warmup_steps=4, cosine_decay_max_steps=50)
    assert tr.optim0.param_groups[0]["lr"] == pytest.approx(3e-4 / 4)
    w, s = tr.warmup_schedulers[0], tr.sched0
    for _ in range(6):
        with w.dampening():
            s.step()
    want = 3e-4 * 0.5 * (1 + math.cos(math.pi * 6 / 50))
    assert tr.optim0.param_groups[0]["lr"] == pytest.approx(want, rel=1e-9)


def test_shard_loader_rank_strided_and_disjoint():
    """accelerate.prepare's per-rank split of the loaders (trainer.py:117-124):
    two ranks see disjoint samples that together cover the dataset, shuffled
    the same way on both ranks, reshuffled per epoch."""
    from torch.utils.data import DataLoader, TensorDataset

    from dalle2_video.trainer import ShardedLoader

    ds = TensorDataset(torch.arange(20))
    for shuffle in (False, True):
        dl = DataLoader(ds, batch_size=3, shuffle=shuffle)
        shards = [ShardedLoader(dl, 2, r, seed=7) for r in range(2)]
        seen = [[int(v) for (b,) in s for v in b] for s in shards]
        assert not set(seen[0]) & set(seen[1])
        assert sorted(seen[0] + seen[1]) == list(range(20))
        assert len(shards[0]) == 4 and shards[0].batch_size == 3
        again = [int(v) for (b,) in shards[0] for v in b]
        assert (again != seen[0]) == shuffle  # set_epoch advances the shuffle order


def test_ema_schedule():
    from dalle2_video.trainer import EMA

    m = torch.nn.Linear(2, 2)
    ema = EMA(m, beta=0.9999, update_after_step=100, update_every=10)
    ema.step.fill_(111)
    epoch = 111 - 100 - 1
    assert math.isclose(ema._decay(), 1 - (1 + epoch) ** (-2 / 3), rel_tol=1e-12)
    ema.step.fill_(50)
    assert ema._decay() == 0.0
    with torch.no_grad():
        m.weight.fill_(3.0)
    ema.step.fill_(0)
    ema.update()  # first update copies the online weights
    assert torch.equal(ema.ema_model.weight, m.weight)


def test_split_args_and_kwargs():
    from dalle2_video.trainer import split_args_and_kwargs

    x = torch.arange(10).reshape(5, 2)
    chunks = list(split_args_and_kwargs(x, split_size=2, video_embed=torch.zeros(5, 3), flag=True))
    assert [round(f, 6) for f, _ in chunks] == [0.4, 0.4, 0.2]
    assert sum(f for f, _ in chunks) == pytest.approx(1.0)
    (a,), kw = chunks[-1][1]
    assert a.shape == (1, 2) and kw["video_embed"].shape == (1, 3) and kw["flag"] is True
    assert list(split_args_and_kwargs(x, split_size=None))[0][0] == 1.0


def test_sinusoid_freqs_match_torch_expression():
    from dalle2_video import ops

    for dim in (16, 64, 128):
        half = dim // 2
        ref = torch.exp(torch.arange(half) * -(math.log(10000) / (half - 1)))
        assert torch.equal(ops.sinusoid_freqs(dim, "cpu"), ref.float())


def test_shard_loader_keeps_custom_batch_sampler_batches():
    """a DataLoader built with a custom batch_sampler (batch_size
    None) is sharded by batches — rank r of N gets batches r, r+N, ... as the
    sampler made them — instead of being rebuilt with automatic batching off."""
    from torch.utils.data import DataLoader, TensorDataset

    from dalle2_video.trainer import shard_loader

    ds = TensorDataset(torch.arange(20))
    batches = [[0, 1, 2], [3, 4, 5], [6, 7, 8], [9, 10, 11], [12, 13]]
    loader = DataLoader(ds, batch_sampler=batches)
    assert loader.batch_size is None
    got = []
    for r in range(2):
        sh = shard_loader(loader, 2, r)
        got.append([b[0].tolist() for b in sh])
        assert len(sh) == len(got[-1])
    assert got[0] == [batches[0], batches[2], batches[4]]
    assert got[1] == [batches[1], batches[3]]


def test_shard_loader_leaves_the_callers_sampler_unseeded():
    """sharding a loader whose batch sampler draws from an
    unseeded RandomSampler seeds a COPY (every rank draws the broadcast-seeded
    order); the caller's DataLoader keeps its own sampler, unseeded."""
    from torch.utils.data import BatchSampler, DataLoader, RandomSampler, TensorDataset

    from dalle2_video.trainer import shard_loader

    ds = TensorDataset(torch.arange(32))
    rs = RandomSampler(ds)
    loader = DataLoader(ds, batch_sampler=BatchSampler(rs, 4, drop_last=False))
    orders = []
    for r in range(2):
        sh = shard_loader(loader, 2, r)
        orders.append([b[0].tolist() for b in sh])
    assert rs.generator is None and loader.batch_sampler.sampler is rs
    flat = sorted(v for o in orders for b in o for v in b)
    assert flat == list(range(32))  # the two ranks' batches partition one seeded order


def test_decoder_state_dict_keys_match_the_reference_layout():
    """VideoDecoder's checkpoint keys (what train_decoder.py:177-184 saves):
    the reference module tree (dalle2_video.py:1169-1506) registers, per unet
    i, `unets.i.*` (the Unet3D keys, pinned to the reference by golden G2),
    `noise_schedulers.i.*` (NoiseScheduler's persistent buffers — restated
    from dalle2-pytorch 1.14.2, so this part is pinned to the oracle's
    restatement, not to the package), nothing for `vaes` (NullVQGanVAE) or
    `lowres_conds` (LowresVideoConditioner without noising), and `_dummy` is
    non-persistent.  Values of the schedule buffers match the oracle's."""
    from dalle2_video import dalle2_video as D

    u1 = D.Unet3D(16, video_embed_dim=512, channels=3, dim_mults=(1, 2, 4, 8))
    u2 = D.Unet3D(8, video_embed_dim=512, channels=3, dim_mults=(1, 2, 4, 8, 16))
    dec = D.VideoDecoder((u1, u2), frame_sizes=(64, 128), frame_numbers=(16, 16), timesteps=1000,
                         learned_variance=False)
    sd = dec.state_dict()
    want = set()
    for i, u in enumerate(dec.unets):
        want |= {f"unets.{i}.{k}" for k in u.state_dict()}
    scheds = [R.NoiseScheduler(beta_schedule=b, timesteps=1000, loss_type="l2") for b in ("cosine", "linear")]
    for i, s in enumerate(scheds):
        want |= {f"noise_schedulers.{i}.{k}" for k in s.state_dict()}
    assert set(sd) == want, (sorted(set(sd) - want)[:5], sorted(want - set(sd))[:5])
    for i, s in enumerate(scheds):
        for k, v in s.state_dict().items():
            assert torch.allclose(sd[f"noise_schedulers.{i}.{k}"], v, rtol=1e-6, atol=0), (i, k)
