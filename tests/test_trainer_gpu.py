"""VideoDecoderTrainer (fused HIP AdamW + HIP grad-norm clip) vs the golden
3-step training trace G4 (torch AdamW + clip_grad_norm_ on the CPU oracle)."""
import contextlib
import os

import numpy as np
import pytest
import torch

from oracle import dv_ref as R

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


def test_three_step_trace_matches_golden():
    from dalle2_video import dalle2_video as D
    from dalle2_video.trainer import VideoDecoderTrainer

    g = np.load(os.path.join(GOLD, "g4_plosses.npz"))
    ou = R.deterministic_fill_(R.Unet3D(16, video_embed_dim=512, channels=3, dim_mults=(1, 2, 4, 8))
                               .cast_model_parameters(lowres_cond=False, lowres_noise_cond=False, channels=3,
                                                      channels_out=3, cond_on_image_embeds=True,
                                                      cond_on_text_encodings=False))
    u = D.Unet3D(16, video_embed_dim=512, channels=3, dim_mults=(1, 2, 4, 8))
    dec = D.VideoDecoder(u, frame_sizes=(32,), frame_numbers=(4,), timesteps=1000, learned_variance=False)
    dec.unets[0].load_state_dict(ou.state_dict(), strict=True)
    dec = dec.cuda()
    tr = VideoDecoderTrainer(dec, lr=3e-4, wd=1e-2, use_ema=False)
    x = torch.from_numpy(g["x"]).cuda()
    times = torch.from_numpy(g["times"]).cuda()
    noise = torch.from_numpy(g["noise"]).cuda()
    losses = []
    for _ in range(3):
        loss = dec.p_losses(dec.unets[0], x, times, video_embed=None,
                            noise_scheduler=dec.noise_schedulers[0], noise=noise)
        losses.append(loss.item())
        loss.backward()
        tr.update(1)
    ref = g["losses"]
    print("losses", losses, "ref", ref.tolist())
    assert np.allclose(losses, ref, rtol=1e-4)
    psum = sum(p.double().sum().item() for p in dec.unets[0].parameters())
    assert abs(psum - g["param_sum"][0]) / abs(g["param_sum"][0]) < 1e-5
    w = dec.unets[0].to_out.weight.detach().cpu().flatten().numpy()
    assert np.allclose(w, g["to_out_w"], rtol=1e-3, atol=1e-6)
    assert tr.num_steps_taken(1) == 3
    sd = tr.optim0.state_dict()
    assert len(sd["state"]) > 0 and all(float(s["step"]) == 3.0 for s in sd["state"].values())


def test_trainer_call_api_and_checkpoint(tmp_path):
    from dalle2_video import dalle2_video as D
    from dalle2_video.trainer import VideoDecoderTrainer

    u1 = D.Unet3D(16, video_embed_dim=512, channels=3, dim_mults=(1, 2, 4, 8))
    u2 = D.Unet3D(8, video_embed_dim=512, channels=3, dim_mults=(1, 2, 4, 8, 16))
    dec = D.VideoDecoder(unet=(u1, u2), frame_sizes=(32, 64), frame_numbers=(4, 4), timesteps=1000,
                         learned_variance=False).cuda()
    tr = VideoDecoderTrainer(dec, lr=3e-4, wd=1e-2, use_ema=False, amp=True)
    video = torch.rand(2, 3, 4, 64, 64, device="cuda")
    emb = torch.randn(2, 512, device="cuda")
    for un in (1, 2):
        l = tr(video_embed=emb, video=video, unet_number=un)
        assert isinstance(l, float) and np.isfinite(l)
        tr.update(un)
    assert tr.optim0.param_groups[0]["lr"] == 3e-4 and tr.optim1.param_groups[0]["lr"] == 3e-4
    path = tmp_path / "ck.pt"
    tr.save(str(path))
    flat_before = [t.clone() for t in tr.optim0._flat[:4]]  # P, G, M, V
    u1b = D.Unet3D(16, video_embed_dim=512, channels=3, dim_mults=(1, 2, 4, 8))
    u2b = D.Unet3D(8, video_embed_dim=512, channels=3, dim_mults=(1, 2, 4, 8, 16))
    dec2 = D.VideoDecoder(unet=(u1b, u2b), frame_sizes=(32, 64), frame_numbers=(4, 4), timesteps=1000,
                          learned_variance=False).cuda()
    tr2 = VideoDecoderTrainer(dec2, lr=3e-4, wd=1e-2, use_ema=False)
    tr2.load(str(path))
    assert tr2.steps.tolist() == [1, 1]
    # weights and AdamW moments restored: one more identical step on both
    # trainers gives identical flat buffers
    g = torch.Generator(device="cuda").manual_seed(5)
    x = torch.rand(2, 3, 4, 32, 32, device="cuda", generator=g)
    t = torch.tensor([3, 700], device="cuda")
    nz = torch.randn(x.shape, device="cuda", generator=g)
    for d, t_ in ((dec, tr), (dec2, tr2)):
        d.p_losses(d.unets[0], x, t, video_embed=None, noise_scheduler=d.noise_schedulers[0],
                   noise=nz).backward()
        t_.update(1)
    P1, _, M1, V1 = tr.optim0._flat[:4]
    P2, _, M2, V2 = tr2.optim0._flat[:4]
    assert not torch.equal(flat_before[0], P1)  # the extra step moved the weights
    for a, b in ((P1, P2), (M1, M2), (V1, V2)):
        assert ((a - b).norm() / a.norm()).item() < 1e-5
    st = tr2.optim0.state_dict()["state"]
    assert len(st) > 0 and all(float(v["step"]) == 2.0 for v in st.values())


@pytest.mark.parametrize("use_ema", [False, True])
def test_train_sample_train_keeps_training(use_ema):
    """trainer.sample between updates (reference trainer.py:276-300) must not
    detach the parameters from the fused optimizer's flat buffers: train ->
    sample -> train ends on the same weights as train -> train (to 1e-4: the
    f32 atomics of GroupNorm / split-K reductions reorder sums run to run)."""
    from dalle2_video import dalle2_video as D
    from dalle2_video.trainer import VideoDecoderTrainer
    from dalle2_video.utils import deterministic_fill_

    def make():
        u = D.Unet3D(16, video_embed_dim=512, channels=3, dim_mults=(1, 2, 4, 8))
        dec = D.VideoDecoder(u, frame_sizes=(32,), frame_numbers=(2,), timesteps=4, learned_variance=False)
        deterministic_fill_(dec.unets[0])
        dec = dec.cuda()
        return dec, VideoDecoderTrainer(dec, lr=3e-4, use_ema=use_ema, ema_update_every=1,
                                        ema_update_after_step=0)

    g = torch.Generator(device="cuda").manual_seed(9)
    x = torch.rand(1, 3, 2, 32, 32, device="cuda", generator=g)
    nz = torch.randn(x.shape, device="cuda", generator=g)
    t = torch.tensor([2], device="cuda")  # within the 4-step schedule

    def train(dec, tr):
        dec.p_losses(dec.unets[0], x, t, video_embed=None, noise_scheduler=dec.noise_schedulers[0],
                     noise=nz).backward()
        tr.update(1)

    decA, trA = make()
    decB, trB = make()
    train(decA, trA)
    train(decB, trB)
    w0 = decB.unets[0].to_out.weight.detach().clone()
    vid = trB.sample(video_embed=torch.randn(1, 512, device="cuda"))
    assert vid.shape == (1, 3, 2, 32, 32) and torch.isfinite(vid).all()
    train(decA, trA)
    train(decB, trB)
    wA, wB = decA.unets[0].to_out.weight.detach(), decB.unets[0].to_out.weight.detach()
    assert not torch.equal(wB, w0), "the update after sampling did not change the weights"
    for (n, pa), pb in zip(decA.unets[0].named_parameters(), decB.unets[0].parameters()):
        assert ((pa - pb).norm() / pa.norm().clamp_min(1e-30)).item() < 1e-4, n


@pytest.mark.parametrize("streamed", [True, False])
def test_deferred_wgrad_sum_matches_per_conv_sum(streamed):
    """ops.defer_wgrad (the trainer's forward+backward): the row-window wgrad
    partials of every conv are summed either on a side stream right after
    each wgrad (streamed, the default) or in ONE dv_wgrad_reduce_batched
    launch at the end of the pass, instead of one reduce per conv on the main
    stream.  Same split count and summation order -> bit-identical weight and
    bias gradients, also when a gradient accumulates (a second pass, or one
    weight read by two convs: streamed sums stay ordered on their stream,
    pending batched sums are flushed before the second target write)."""
    from dalle2_video import ops

    g = torch.Generator(device="cuda").manual_seed(11)
    shapes = [(16, 32, 32, 64, 64, 3), (64, 8, 8, 128, 256, 3), (8, 64, 64, 64, 128, 1)]
    xs, ws, bs, dys = [], [], [], []
    for nf, h, w, cin, cout, k in shapes:
        xs.append(torch.randn(nf, h, w, cin, device="cuda", generator=g).bfloat16())
        ws.append(torch.randn(cout, cin, 1, k, k, device="cuda", generator=g).div_((cin * k * k) ** 0.5)
                  .requires_grad_())
        bs.append(torch.randn(cout, device="cuda", generator=g).requires_grad_())
        dys.append(torch.randn(nf, h, w, cout, device="cuda", generator=g).bfloat16())

    def run(defer, passes):
        for p in ws + bs:
            p.grad = None
        n_pending = []
        for _ in range(passes):
            with (ops.defer_wgrad() if defer else contextlib.nullcontext()):
                outs = [ops.conv(x, w_, b_) for x, w_, b_ in zip(xs, ws, bs)]
                outs.append(ops.conv(xs[0], ws[0], bs[0]))  # the same weight read twice
                torch.autograd.backward(outs, dys + [dys[0]])
                n_pending.append(ops.WGRAD_DEFER.added)
        torch.cuda.synchronize()
        return [p.grad.clone() for p in ws + bs], n_pending

    saved = ops.WGRAD_DEFER.STREAM
    ops.WGRAD_DEFER.STREAM = streamed
    try:
        for passes in (1, 2):
            ref, _ = run(False, passes)
            got, n_pending = run(True, passes)
            assert all(n >= 1 for n in n_pending), n_pending
            assert not ops.WGRAD_DEFER.pending and ops.WGRAD_DEFER.streamed is None
            for i, (a, b) in enumerate(zip(ref, got)):
                assert torch.equal(a, b), (passes, i, ((a - b).norm() / a.norm()).item())
    finally:
        ops.WGRAD_DEFER.STREAM = saved


def test_graph_replay_matches_eager():
    """HIP-graph capture/replay of forward+backward (use_graphs=True) reproduces
    the eager call: same seed -> same sampled times/noise -> same loss and
    gradients (atomics reorder f32 sums: tolerance 1e-5)."""
    from dalle2_video import dalle2_video as D
    from dalle2_video.trainer import VideoDecoderTrainer
    from dalle2_video.utils import deterministic_fill_

    u = D.Unet3D(16, video_embed_dim=512, channels=3, dim_mults=(1, 2, 4, 8))
    dec = D.VideoDecoder(u, frame_sizes=(32,), frame_numbers=(4,), timesteps=1000, learned_variance=False)
    deterministic_fill_(dec.unets[0])
    dec = dec.cuda()
    tr = VideoDecoderTrainer(dec, lr=3e-4, use_ema=False, use_graphs=True)
    g = torch.Generator(device="cuda").manual_seed(3)
    video = torch.rand(2, 3, 4, 32, 32, device="cuda", generator=g)
    torch.cuda.manual_seed(1)
    tr(video=video, unet_number=1)
    tr.update(1)  # builds the flat gradient buffer
    opt = tr.optim0
    res = {}
    for tag, seed in (("A", 7), ("B", 8), ("C", 7), ("D", 8)):  # A, B eager warm-up; C captures
        opt.zero_grad()
        torch.cuda.manual_seed(seed)
        loss = tr(video=video, unet_number=1)
        torch.cuda.synchronize()
        res[tag] = (loss, opt.flat_grad.clone())
    assert len(tr._graphs) == 1 and "graph" in next(iter(tr._graphs.values()))
    G = opt.flat_grad
    views = [(n, (p.grad.data_ptr() - G.data_ptr()) // 4, p.numel()) for n, p in dec.named_parameters()
             if p.grad is not None]
    for e, gph in (("A", "C"), ("B", "D")):
        le, ge = res[e]
        lg, gg = res[gph]
        assert abs(le - lg) <= 1e-5 * abs(le), (e, le, lg)
        err = ((ge - gg).norm() / ge.norm()).item()
        if err >= 1e-5:
            worst = sorted(((((ge[o:o + k] - gg[o:o + k]).norm() / ge[o:o + k].norm().clamp_min(1e-30)).item(), n)
                            for n, o, k in views), reverse=True)[:8]
            raise AssertionError(f"{e} vs {gph}: rel {err:.3e}; worst params {worst}")


def test_graph_replay_sees_inputs_modified_in_place():
    """The replay skips copying an input that is the previous call's very
    tensor, unmodified (its version counter): an in-place change of that
    tensor, or another tensor, must be copied in.  Replays with modified /
    new inputs equal the eager calls on the same data."""
    from dalle2_video import dalle2_video as D
    from dalle2_video.trainer import VideoDecoderTrainer
    from dalle2_video.utils import deterministic_fill_

    u = D.Unet3D(16, video_embed_dim=512, channels=3, dim_mults=(1, 2, 4, 8))
    dec = D.VideoDecoder(u, frame_sizes=(32,), frame_numbers=(4,), timesteps=1000, learned_variance=False)
    deterministic_fill_(dec.unets[0])
    dec = dec.cuda()

    def run(graphs):
        tr = VideoDecoderTrainer(dec, lr=0.0, use_ema=False, use_graphs=graphs)
        g = torch.Generator(device="cuda").manual_seed(3)
        video = torch.rand(2, 3, 4, 32, 32, device="cuda", generator=g)
        other = torch.rand(2, 3, 4, 32, 32, device="cuda", generator=g)
        torch.cuda.manual_seed(1)
        tr(video=video, unet_number=1)
        tr.update(1)
        out = []
        for step in range(7):  # calls 3.. replay when graphs=True
            if step == 4:
                video.mul_(0.5)  # in place: same object, new version
            x = other if step == 6 else video
            torch.cuda.manual_seed(11)
            out.append(tr(video=x, unet_number=1))
        return out

    eager, graph = run(False), run(True)
    for a, b in zip(eager, graph):
        assert abs(a - b) <= 1e-5 * abs(a), (eager, graph)
    assert abs(eager[3] - eager[4]) > 1e-4 * abs(eager[3])  # the in-place change mattered


def test_graph_replay_after_checkpoint_load(tmp_path):
    """A captured graph keeps writing the live gradient buffer after
    trainer.save/load (the flat buffers are kept): replayed calls
    after the load give the same gradients as eager calls."""
    from dalle2_video import dalle2_video as D
    from dalle2_video.trainer import VideoDecoderTrainer
    from dalle2_video.utils import deterministic_fill_

    u = D.Unet3D(16, video_embed_dim=512, channels=3, dim_mults=(1, 2, 4, 8))
    dec = D.VideoDecoder(u, frame_sizes=(32,), frame_numbers=(4,), timesteps=1000, learned_variance=False)
    deterministic_fill_(dec.unets[0])
    dec = dec.cuda()
    tr = VideoDecoderTrainer(dec, lr=3e-4, use_ema=False, use_graphs=True)
    video = torch.rand(2, 3, 4, 32, 32, device="cuda")
    for _ in range(4):  # update, eager, eager, capture+replay
        tr(video=video, unet_number=1)
        tr.update(1)
    assert any("graph" in v for v in tr._graphs.values())
    path = tmp_path / "ck.pt"
    tr.save(str(path))
    G = tr.optim0.flat_grad
    tr.load(str(path))
    assert tr.optim0.flat_grad is G
    opt = tr.optim0
    opt.zero_grad()
    torch.cuda.manual_seed(11)
    l_graph = tr(video=video, unet_number=1)  # replay
    g_graph = opt.flat_grad.clone()
    assert g_graph.abs().max() > 0, "replay after load wrote no gradient into the live buffer"
    opt.zero_grad()
    tr.use_graphs = False
    torch.cuda.manual_seed(11)
    l_eager = tr(video=video, unet_number=1)
    assert abs(l_graph - l_eager) <= 1e-5 * abs(l_eager)
    assert ((g_graph - opt.flat_grad).norm() / opt.flat_grad.norm()).item() < 1e-5


def test_graphs_survive_sampling_the_trainable_unet():
    """trainer.sample with use_ema=False samples the
    trainable unet, and one_unet_in_gpu moves its parameters through host
    memory (new storage for every p.data / p.grad).  The next training call
    must not replay the graph captured on the old storage: the trainer
    re-points the unet into fresh flat buffers first and drops its graphs, so
    the gradients of the call after sampling land in the live buffer and
    equal an eager call's."""
    from dalle2_video import dalle2_video as D
    from dalle2_video.trainer import VideoDecoderTrainer
    from dalle2_video.utils import deterministic_fill_

    u = D.Unet3D(16, video_embed_dim=512, channels=3, dim_mults=(1, 2, 4, 8))
    dec = D.VideoDecoder(u, frame_sizes=(32,), frame_numbers=(2,), timesteps=4, learned_variance=False)
    deterministic_fill_(dec.unets[0])
    dec = dec.cuda()
    tr = VideoDecoderTrainer(dec, lr=3e-4, use_ema=False, use_graphs=True)
    video = torch.rand(2, 3, 2, 32, 32, device="cuda")
    for _ in range(5):  # update, eager, eager, capture, replay
        tr(video=video, unet_number=1)
        tr.update(1)
    assert any("graph" in v for v in tr._graphs.values())
    opt = tr.optim0
    G_old = opt.flat_grad
    vid = tr.sample(video_embed=torch.randn(2, 512, device="cuda"))
    assert torch.isfinite(vid).all()
    opt.zero_grad()
    torch.cuda.manual_seed(21)
    l1 = tr(video=video, unet_number=1)
    torch.cuda.synchronize()
    assert opt._aliased(), "parameters are not views of the optimizer's flat buffers after sampling"
    assert opt.flat_grad is not G_old
    g1 = opt.flat_grad.clone()
    assert g1.abs().max() > 0, "the call after sampling wrote no gradient into the live buffer"
    opt.zero_grad()
    tr.use_graphs = False
    torch.cuda.manual_seed(21)
    l2 = tr(video=video, unet_number=1)
    assert abs(l1 - l2) <= 1e-5 * abs(l2)
    assert ((g1 - opt.flat_grad).norm() / opt.flat_grad.norm()).item() < 1e-5
    w0 = dec.unets[0].to_out.weight.detach().clone()
    tr.update(1)
    assert not torch.equal(dec.unets[0].to_out.weight.detach(), w0), "the update did not move the weights"
