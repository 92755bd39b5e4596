"""Host -> HBM hand-off of training batches (datasets.DeviceLoader, what the
reference's accelerate-prepared loaders do) and the 224x224 clip path of
VideoDecoder.forward (per-frame nearest resize on the GPU, reference
dalle2_video.py:2257)."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def test_device_loader_delivers_identical_batches_on_gpu():
    from dalle2_video.datasets import DeviceLoader

    vids = torch.randn(10, 3, 4, 32, 32)
    emb = torch.randn(10, 512)
    ds = torch.utils.data.TensorDataset(emb, vids)
    dl = torch.utils.data.DataLoader(ds, batch_size=4)
    dev = DeviceLoader(dl, "cuda")
    for epoch in range(2):
        n = 0
        for (e0, v0), (e1, v1) in zip(dl, dev):
            assert e1.is_cuda and v1.is_cuda
            v1 = v1 * 1.0  # consume on the current stream
            assert torch.equal(e1.cpu(), e0) and torch.equal(v1.cpu(), v0)
            n += 1
        assert n == 3


def test_device_loader_passes_device_batches_through():
    from dalle2_video.datasets import DeviceLoader

    batches = [(torch.randn(2, 3, device="cuda"), torch.arange(2))]
    out = list(DeviceLoader(batches, "cuda"))
    assert len(out) == 1 and torch.equal(out[0][0], batches[0][0]) and out[0][1].is_cuda


def test_trainer_loader_on_device_and_224_clip_path():
    from dalle2_video import dalle2_video as D
    from dalle2_video.trainer import VideoDecoderTrainer
    from dalle2_video.utils import deterministic_fill_

    u = D.Unet3D(16, video_embed_dim=512, channels=3, dim_mults=(1, 2, 4, 8))
    dec = D.VideoDecoder(u, frame_sizes=(32,), frame_numbers=(4,), timesteps=1000, learned_variance=False)
    deterministic_fill_(dec.unets[0])
    dec = dec.cuda()
    g = torch.Generator().manual_seed(0)
    clips = torch.rand(4, 3, 4, 224, 224, generator=g)
    ds = torch.utils.data.TensorDataset(torch.randn(4, 512, generator=g), clips)
    dl = torch.utils.data.DataLoader(ds, batch_size=2)
    tr = VideoDecoderTrainer(dec, lr=3e-4, use_ema=False, dataloaders={"train": dl, "val": dl})
    losses = []
    for emb, video in tr.train_loader:
        assert video.is_cuda and video.shape == (2, 3, 4, 224, 224)
        torch.cuda.manual_seed(7)
        l224 = tr(video_embed=emb, video=video, unet_number=1)
        small = torch.stack([F.interpolate(video[:, :, t], size=(32, 32), mode="nearest")
                             for t in range(video.shape[2])], 2)
        torch.cuda.manual_seed(7)
        l32 = tr(video_embed=emb, video=small, unet_number=1)
        losses.append((l224, l32))
    assert len(losses) == 2
    for a, b in losses:
        assert np.isfinite(a) and abs(a - b) <= 1e-5 * abs(b), (a, b)
