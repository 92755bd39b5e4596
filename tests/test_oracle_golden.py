"""Pin the CPU oracle (oracle/dv_ref.py) to the golden fixtures generated from
the reference's own Unet3D / block classes (tests/golden/gen_golden.py).

G1 (block outputs), G2 (full Unet3D forward at Cfg1 + the cascade unet2),
G3 (NoiseScheduler tables) and G4 (p_losses + a 3-step torch-AdamW training
trace) are all recomputed here from deterministically filled weights
(crc32(name)-seeded, identical on both sides) and compared in fp32.
"""
import os

import numpy as np
import pytest
import torch

from oracle import dv_ref as R

GOLD = os.path.join(os.path.dirname(__file__), "golden")


def gold(name):
    return np.load(os.path.join(GOLD, name + ".npz"))


def rel(a, b):
    a = torch.as_tensor(a).double()
    b = torch.as_tensor(b).double()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def unet(dim, mults, lowres):
    u = R.Unet3D(dim, video_embed_dim=512, channels=3, dim_mults=mults, cond_on_text_encodings=False)
    u = u.cast_model_parameters(lowres_cond=lowres, lowres_noise_cond=False, channels=3,
                                channels_out=3, cond_on_image_embeds=not lowres,
                                cond_on_text_encodings=False)
    return R.deterministic_fill_(u)


@pytest.fixture(autouse=True)
def _threads():
    n = torch.get_num_threads()
    torch.set_num_threads(min(8, os.cpu_count() or 1))
    yield
    torch.set_num_threads(n)


def test_g1_blocks():
    g = gold("g1_blocks")
    x, x3 = torch.from_numpy(g["x"]), torch.from_numpy(g["x3"])
    temb, cond = torch.from_numpy(g["temb"]), torch.from_numpy(g["cond"])
    cases = {
        "block": (lambda: R.Block3D(32, 48), lambda m: m(x)),
        "block_ss": (lambda: R.Block3D(32, 48),
                     lambda m: m(x, scale_shift=(0.1 * temb[:, :48, None, None, None],
                                                 0.1 * temb[:, 48:96, None, None, None]))),
        "resnet": (lambda: R.ResnetBlock3D(32, 64, time_cond_dim=128), lambda m: m(x, temb)),
        "resnet_xattn": (lambda: R.ResnetBlock3D(32, 64, cond_dim=32, time_cond_dim=128),
                         lambda m: m(x, temb, cond)),
        "crossembed": (lambda: R.CrossEmbedLayer3D(3, dim_out=32, kernel_sizes=(3, 7, 15), stride=1),
                       lambda m: m(x3)),
        "downsample": (lambda: R.Downsample3D(32, 64), lambda m: m(x)),
        "pixelshuffle": (lambda: R.PixelShuffleUpsample3D(32, 16), lambda m: m(x)),
    }
    for name, (mk, run) in cases.items():
        m = R.deterministic_fill_(mk())
        with torch.no_grad():
            y = run(m)
        assert rel(y, g[f"y_{name}"]) < 1e-6, name


def test_g2_unet1_cfg1_and_intermediates():
    g = gold("g2_unet_cfg1")
    u = unet(64, (1, 2, 4, 8), False)
    assert sum(p.numel() for p in u.parameters()) == 49_967_171
    with torch.no_grad():
        y, inter = u(torch.from_numpy(g["x"]), torch.from_numpy(g["times"]), return_intermediates=True)
    assert rel(y, g["y"]) < 1e-6
    for k, v in inter.items():
        assert rel(v.double().sum().reshape(1), g[f"sum_{k}"]) < 1e-6, k
        assert rel(v.flatten()[:256], g[f"head_{k}"]) < 1e-6, k


def test_g2_unet2_lowres():
    g = gold("g2_unet_cfg1")
    u = unet(8, (1, 2, 4, 8, 16), True)
    with torch.no_grad():
        y = u(torch.from_numpy(g["x2"]), torch.from_numpy(g["times2"]),
              lowres_cond_video=torch.from_numpy(g["lowres2"]))
    assert rel(y, g["y2"]) < 1e-6


@pytest.mark.parametrize("sched", ["cosine", "linear"])
def test_g3_scheduler_tables_oracle_and_product(sched):
    from dalle2_video import dalle2_video as D

    g = gold("g3_sched")
    so = R.NoiseScheduler(beta_schedule=sched, timesteps=1000, loss_type="l2")
    sp = D.NoiseScheduler(beta_schedule=sched, timesteps=1000, loss_type="l2")
    for b in R.NoiseScheduler.BUFFERS:
        ref = g[f"{sched}_{b}"]
        assert np.allclose(getattr(so, b).numpy(), ref, rtol=1e-6, atol=1e-7), b
        assert np.allclose(getattr(sp, b).cpu().numpy(), ref, rtol=1e-6, atol=1e-7), b


def test_g4_p_losses_and_training_trace():
    g = gold("g4_plosses")
    u = unet(16, (1, 2, 4, 8), False)
    sched = R.NoiseScheduler(beta_schedule="cosine", timesteps=1000, loss_type="l2")
    x, times, noise = (torch.from_numpy(g[k]) for k in ("x", "times", "noise"))
    loss0 = R.p_losses(u, sched, x, times, noise, video_cond_drop_prob=0.0, text_cond_drop_prob=0.0)
    assert abs(loss0.item() - g["loss0"][0]) < 1e-5 * abs(g["loss0"][0])
    opt = R.get_optimizer(u.parameters(), lr=3e-4, wd=1e-2)
    losses = [R.train_step(u, sched, opt, x, times, noise, video_cond_drop_prob=0.0,
                           text_cond_drop_prob=0.0) for _ in range(3)]
    assert np.allclose(losses, g["losses"], rtol=1e-5)
    psum = sum(p.double().sum() for p in u.parameters()).item()
    assert abs(psum - g["param_sum"][0]) < 1e-6 * abs(g["param_sum"][0])
    assert rel(u.to_out.weight.detach().flatten(), g["to_out_w"]) < 1e-5
