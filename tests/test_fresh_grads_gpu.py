"""The deferred gradient zeros (ops.FRESH: update() fills only the gradients
no conv backward writes whole, the conv backward's first write overwrites the
rest) against the plain full fill, on the benchmarked trainer at BASELINE
config 2: two identically initialised trainers stepped in lockstep with the
same seeds, one with the deferral (ops.GRAD_OVERWRITE) and one without.
Covers the eager calls, the captured / replayed pass (its own graph per
deferral state), and an accumulating second call before an update (which
must add, not overwrite).  Reference: trainer.py:322-365 (the call and
update(): optimizer.zero_grad after the step).

After every update the deferred trainer's weights and moments are copied into
the other (and the packed images refreshed), so each step starts both from
the same state and the errors stay at the eager-vs-eager floor instead of
compounding.

Tolerances (norm-wise relative): loss and whole gradient f32 1e-5 (the
eager-vs-replay bound of tests/test_cfg2_trainer_gpu.py), bf16 1e-3 (its
eager-vs-eager floor is ~1e-4: f32 atomics in arrival order); per parameter
f32 1e-3, bf16 5e-2.  A stale gradient (the previous step's added in) shows
as an O(1) error of its parameter."""
import pytest
import torch

pytestmark = pytest.mark.gpu

B, T, S = 4, 16, 64


def rel(a, b):
    a, b = a.detach().double(), b.detach().double()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


@pytest.mark.parametrize("amp,graphs,tol,ptol", [(False, False, 1e-5, 1e-3), (False, True, 1e-5, 1e-3),
                                                  (True, True, 1e-3, 5e-2)])
def test_deferred_zero_matches_full_fill(parity_log, amp, graphs, tol, ptol):
    from dalle2_video import dalle2_video as D
    from dalle2_video import ops
    from dalle2_video.trainer import VideoDecoderTrainer
    from dalle2_video.utils import deterministic_fill_

    def make():
        u = D.Unet3D(64, video_embed_dim=512, channels=3, dim_mults=(1, 2, 4, 8), cond_on_text_encodings=False)
        dec = D.VideoDecoder(unet=(u,), frame_sizes=(S,), frame_numbers=(T,), timesteps=1000,
                             learned_variance=False)
        deterministic_fill_(dec.unets[0])
        return VideoDecoderTrainer(dec.cuda(), lr=3e-4, wd=1e-2, use_ema=False, amp=amp, use_graphs=graphs)

    g = torch.Generator(device="cuda").manual_seed(99)
    video = torch.rand(B, 3, T, S, S, device="cuda", generator=g)
    trs = {True: make(), False: make()}
    old = ops.GRAD_OVERWRITE
    worst = {"loss": 0.0, "grad": 0.0, "param": 0.0, "param_name": ""}
    names = [n for n, _ in trs[True].decoder.unets[0].named_parameters()]
    try:
        # step 0: eager, its update builds the flat buffers and arms the
        # deferral; 1-2 eager warm-ups of the deferred pass, 3 captures it,
        # 4-6 replay; step 5 also accumulates a second call (its own,
        # non-deferred pass) before the update
        for step in range(7):
            res = {}
            for flag, tr in trs.items():
                ops.GRAD_OVERWRITE = flag
                torch.cuda.manual_seed(10 + step)
                loss = tr(video=video, unet_number=1)
                if step == 5:
                    torch.cuda.manual_seed(50 + step)
                    loss += tr(video=video, unet_number=1)
                torch.cuda.synchronize()
                res[flag] = (loss, [None if p.grad is None else p.grad.detach().clone()
                                    for p in tr.decoder.unets[0].parameters()])
                tr.update(1)
            oa, ob = trs[True].optim0, trs[False].optim0
            for i in (0, 2, 3):  # P, M, V: the next step starts both from one state
                ob._flat[i].copy_(oa._flat[i])
            ops.PACK.refresh()
            el = abs(res[True][0] - res[False][0]) / abs(res[False][0])
            ga, gb = res[True][1], res[False][1]
            assert [g is None for g in ga] == [g is None for g in gb]
            live = [(n, a, b) for n, a, b in zip(names, ga, gb) if a is not None]
            eg = rel(torch.cat([a.reshape(-1) for _, a, _ in live]), torch.cat([b.reshape(-1) for _, _, b in live]))
            ep, en = max((rel(a, b), n) for n, a, b in live if b.norm() > 0)
            worst["loss"], worst["grad"] = max(worst["loss"], el), max(worst["grad"], eg)
            if ep > worst["param"]:
                worst["param"], worst["param_name"] = ep, en
            assert el <= tol and eg <= tol and ep <= ptol, (step, el, eg, en, ep)
        if graphs:
            sig_tokens = [k[3] for k in trs[True]._graphs]
            assert any(t is not None for t in sig_tokens), "the deferred pass was never captured"
            assert all("graph" in e for k, e in trs[True]._graphs.items() if k[3] is not None)
        assert all(k[3] is None for k in trs[False]._graphs)
    finally:
        ops.GRAD_OVERWRITE = old
        for tr in trs.values():  # leave no deferred zeros behind for later tests
            ops.FRESH.drop(list(tr.decoder.unets[0].parameters()))
    parity_log(config=f"cfg2 trainer deferred zero_grad amp={amp} graphs={graphs}", **worst)
