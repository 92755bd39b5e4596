"""Data path (reference dalle2_video/datasets.py:23-114): the CelebV-Text
dataset stages, the collator's video fetch and the CPU pass-through of the
device loader.  Videos come from a memory-mapped .npy of preprocess.py's clip
layout (3, T, H, W) float32 — h5py is not in the image."""
import numpy as np
import pytest
import torch


@pytest.fixture()
def files(tmp_path):
    rng = np.random.default_rng(0)
    vids = rng.standard_normal((6, 3, 4, 16, 16)).astype(np.float32)
    np.save(tmp_path / "videos.npy", vids)
    torch.save(torch.randn(6, 512), tmp_path / "video_embeds.pt")
    torch.save(torch.randn(6, 512), tmp_path / "text_embeds.pt")
    torch.save(torch.randint(0, 100, (6, 77)), tmp_path / "texts.pt")
    return tmp_path, vids


def test_decoder_stage_items_and_collate(files):
    from dalle2_video.datasets import CelebVTextDataset

    d, vids = files
    ds = CelebVTextDataset(videos_path=str(d / "videos.npy"), video_embeds_path=str(d / "video_embeds.pt"))
    assert ds.stage == "decoder" and len(ds) == 6
    emb, idx = ds[4]
    assert emb.shape == (512,) and int(idx) == 4
    dl = torch.utils.data.DataLoader(ds, batch_size=4, shuffle=True, collate_fn=ds.collate_fn,
                                     generator=torch.Generator().manual_seed(3))
    seen = []
    for x, v in dl:
        assert v.dtype == torch.float32 and v.shape[1:] == (3, 4, 16, 16)
        for e, clip in zip(x, v):
            i = int(torch.nonzero((ds.video_embeds == e).all(1))[0])
            seen.append(i)
            assert np.array_equal(clip.numpy(), vids[i])  # the collator fetched the right rows, in batch order
    assert sorted(seen) == list(range(6))


def test_stage_detection(files):
    from dalle2_video.datasets import CelebVTextDataset

    d, _ = files
    assert CelebVTextDataset(text_embeds_path=str(d / "text_embeds.pt"),
                             video_embeds_path=str(d / "video_embeds.pt")).stage == "prior"
    clip = CelebVTextDataset(texts_path=str(d / "texts.pt"), videos_path=str(d / "videos.npy"))
    assert clip.stage == "CLIP" and clip[2][0].shape == (77,)
    with pytest.raises(ValueError):
        CelebVTextDataset(video_embeds_path=str(d / "video_embeds.pt"))
    with pytest.raises(AssertionError):
        CelebVTextDataset(texts_path=str(d / "texts.pt"), videos_path=str(d / "videos.npy"),
                          video_embeds_path=str(d / "video_embeds.pt"))


def test_h5_needs_h5py(tmp_path):
    from dalle2_video.datasets import open_videos

    try:
        import h5py  # noqa: F401
        pytest.skip("h5py present")
    except ImportError:
        pass
    with pytest.raises(ImportError, match="h5py"):
        open_videos(str(tmp_path / "preprocessed_20subsets.h5"))


def test_device_loader_cpu_passthrough(files):
    from dalle2_video.datasets import CelebVTextDataset, DeviceLoader

    d, _ = files
    ds = CelebVTextDataset(videos_path=str(d / "videos.npy"), video_embeds_path=str(d / "video_embeds.pt"))
    dl = torch.utils.data.DataLoader(ds, batch_size=3, collate_fn=ds.collate_fn)
    wrapped = DeviceLoader(dl, "cpu")
    assert len(wrapped) == 2 and wrapped.batch_size == 3 and wrapped.dataset is ds
    for (a, b), (c, e) in zip(dl, wrapped):
        assert torch.equal(a, c) and torch.equal(b, e)
