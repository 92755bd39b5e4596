"""BASELINE config 3's training step as bench.py times it (the `config3` leg):
VideoDecoderTrainer(use_graphs=True) on the two-unet decoder — unet1 (dim 64,
64^2) and the low-res conditioned SR unet2 (dim 8, mults 1..16, 128^2) —
alternating trainer(unet k) + update(k) on 224^2 clips (reference
train_decoder.py:127-138; VideoDecoder.forward dalle2_video.py:2188-2299; the
LowresVideoConditioner's per-call kornia blur draw `:1139`).

unet2's call is captured too: the trainer draws the conditioner's blur
decision on the host (the same one random.random() per call the eager path
makes inside the conditioner) and replays the graph of that decision.

  * per decision (blur_prob forced to 1 and to 0): the two eager warm-up calls
    vs captured replays of the same device seeds — loss and flat gradient;
    f32 <= 1e-5 (the captured machinery is exact), bf16 loss <= 1e-4 and
    gradient <= 5e-4 (the eager-vs-eager floor of the f32-atomic sums, see
    tests/test_cfg2_trainer_gpu.py)
  * the alternating loop with blur_prob 0.5: graphs on vs graphs off from the
    same python / device seeds take the same blur decisions and give the same
    losses (bf16 <= 2e-3 relative per call over 8 calls)
"""
import random

import pytest
import torch

pytestmark = pytest.mark.gpu

B, T = 4, 16


def rel(a, b):
    a, b = a.detach().double().cpu(), b.detach().double().cpu()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def _trainer(amp, graphs):
    from dalle2_video import dalle2_video as D
    from dalle2_video.trainer import VideoDecoderTrainer
    from dalle2_video.utils import deterministic_fill_

    u1 = D.Unet3D(64, video_embed_dim=512, channels=3, dim_mults=(1, 2, 4, 8), cond_on_text_encodings=False)
    u2 = D.Unet3D(8, video_embed_dim=512, channels=3, dim_mults=(1, 2, 4, 8, 16), cond_on_text_encodings=False)
    dec = D.VideoDecoder(unet=(u1, u2), frame_sizes=(64, 128), frame_numbers=(T, T), timesteps=1000,
                         learned_variance=False)
    for u in dec.unets:
        deterministic_fill_(u)
    dec = dec.cuda()
    return dec, VideoDecoderTrainer(dec, lr=3e-4, wd=1e-2, use_ema=False, amp=amp, use_graphs=graphs)


def _clip():
    g = torch.Generator(device="cuda").manual_seed(99)
    return torch.rand(B, 3, T, 224, 224, device="cuda", generator=g)


@pytest.mark.parametrize("amp,gtol,ltol", [(True, 5e-4, 1e-4), (False, 1e-5, 1e-5)])
def test_unet2_graph_replay_per_blur_decision(parity_log, amp, gtol, ltol):
    dec, tr = _trainer(amp, True)
    video = _clip()
    torch.cuda.manual_seed(1)
    tr(video=video, unet_number=2)
    tr.update(2)  # builds unet2's flat buffers (the first call is never captured)
    lc = dec.lowres_conds[1]
    assert lc is not None
    opt = tr.optim1
    errs = {}
    for blur in (True, False):
        lc.blur_prob = 1.0 if blur else 0.0
        res = {}
        for tag, seed in (("A", 7), ("B", 8), ("C", 7), ("D", 8)):
            opt.zero_grad()
            torch.cuda.manual_seed(seed)
            loss = tr(video=video, unet_number=2)
            torch.cuda.synchronize()
            res[tag] = (loss, opt.flat_grad.clone())
        for e, r in (("A", "C"), ("B", "D")):
            errs[f"blur{int(blur)}_loss_{e}{r}"] = abs(res[e][0] - res[r][0]) / abs(res[e][0])
            errs[f"blur{int(blur)}_grad_{e}{r}"] = rel(res[r][1], res[e][1])
    caps = [k for k, v in tr._graphs.items() if k[0] == 2 and "graph" in v]
    assert sorted(k[2] for k in caps) == [False, True], "one captured unet2 graph per blur decision"
    parity_log(config=f"cfg3 unet2 trainer graph replay vs eager amp={amp} 4x3x16x224^2 -> 128^2", **errs)
    for k, v in errs.items():
        assert v <= (ltol if "_loss_" in k else gtol), (k, v)


def test_alternating_step_graphs_match_eager(parity_log):
    losses = {}
    for graphs in (False, True):
        dec, tr = _trainer(True, graphs)
        video = _clip()
        random.seed(5)
        out = []
        for i in range(8):  # calls 4.. of each unet replay captured graphs when graphs=True
            for un in (1, 2):
                torch.cuda.manual_seed(100 + 2 * i + un)
                out.append(tr(video=video, unet_number=un))
                tr.update(un)
        torch.cuda.synchronize()
        losses[graphs] = out
        if graphs:
            assert any(k[0] == 2 and "graph" in v for k, v in tr._graphs.items())
        del tr, dec
    errs = [abs(a - b) / abs(a) for a, b in zip(losses[False], losses[True])]
    parity_log(config="cfg3 alternating step graphs vs eager (blur p=0.5)", worst=max(errs),
               losses_eager=losses[False], losses_graphs=losses[True])
    assert max(errs) <= 2e-3, errs
