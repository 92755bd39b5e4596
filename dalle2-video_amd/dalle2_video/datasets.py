"""Data path of decoder training (reference dalle2_video/datasets.py:23-114,
train_decoder.py:45-60, 127-128): the CelebV-Text dataset / collator API, and
the host -> HBM hand-off the reference gets from `accelerator.prepare`'s
device placement, done MI355X-side: pinned host batches copied on a
dedicated HIP stream one batch ahead of the step that consumes them.

Clip layout is the reference's: preprocess.py stores (3, T, 224, 224) float32
CLIP-normalised frames per video in an HDF5 dataset "videos"; the collator
stacks the selected videos into (b, 3, T, 224, 224).  The per-frame nearest
resize to the unet's frame size happens on the GPU inside VideoDecoder.forward
(dv_resize_nearest, reference dalle2_video.py:2257).

h5py / natsort / clip are not dependencies of the hot path: an .h5 path needs
h5py (imported on use); a .npy path (np.load(mmap_mode="r")) or any array-like
indexable by video id works the same way.
"""
from __future__ import annotations

import os
from typing import Any, List, Optional, Tuple

import numpy as np
import torch
import torch.nn as nn


def exists(val: Any) -> bool:
    return val is not None


def open_videos(videos_path):
    """The "videos" dataset of preprocess.py's HDF5 file, or a .npy array
    (memory-mapped), or an array-like passed through."""
    if not isinstance(videos_path, (str, os.PathLike)):
        return videos_path
    path = os.fspath(videos_path)
    if path.endswith(".npy"):
        return np.load(path, mmap_mode="r")
    try:
        import h5py
    except ImportError as e:  # the image has no h5py: say what would be needed
        raise ImportError(f"reading {path} needs h5py (or convert the 'videos' dataset to .npy)") from e
    return h5py.File(path, "r")["videos"]


def _load_tensor(path):
    return torch.load(path, map_location="cpu", weights_only=True).cpu()


class CelebVTextCollator(nn.Module):
    """Stacks (x, index) items and fetches the indexed videos
    (reference datasets.py:23-45): returns (x, videos (b, c, t, h, w))."""

    def __init__(self, videos_ref) -> None:
        super().__init__()
        self.videos_ref = videos_ref

    def forward(self, batch: List[Tuple[torch.Tensor, torch.Tensor]]) -> Tuple[torch.Tensor, torch.Tensor]:
        x = torch.stack([item[0] for item in batch])
        idx = [int(item[1]) for item in batch]
        # one sorted read per batch (HDF5 chunk order), then back to batch order
        order = sorted(range(len(idx)), key=idx.__getitem__)
        rows = {idx[i]: np.asarray(self.videos_ref[idx[i]]) for i in order}
        videos = np.stack([rows[i] for i in idx])
        return x, torch.from_numpy(videos)


class CelebVTextDataset(torch.utils.data.Dataset):
    """Stage-dependent items (reference datasets.py:47-114):
    CLIP (texts, video ids), prior (text embeds, video embeds) or decoder
    (video embeds, video ids); the videos themselves are loaded by
    `collate_fn` (a CelebVTextCollator) when a videos path is given."""

    def __init__(self, texts_path: Optional[str] = None, videos_path=None,
                 text_embeds_path: Optional[str] = None, video_embeds_path: Optional[str] = None) -> None:
        self.texts = _load_tensor(texts_path) if exists(texts_path) else None
        self.videos_ref = open_videos(videos_path) if exists(videos_path) else None
        self.videos = (torch.arange(len(self.videos_ref), dtype=torch.int64)
                       if exists(self.videos_ref) else None)
        self.text_embeds = _load_tensor(text_embeds_path) if exists(text_embeds_path) else None
        self.video_embeds = _load_tensor(video_embeds_path) if exists(video_embeds_path) else None

        if exists(self.texts) and exists(self.videos):
            assert self.text_embeds is None and self.video_embeds is None, \
                "Embeddings are not needed for CLIP training."
            self.stage = "CLIP"
            assert len(self.texts) == len(self.videos)
        elif exists(self.text_embeds) and exists(self.video_embeds):
            assert self.texts is None and self.videos is None, \
                "Texts and videos are not needed for prior training."
            self.stage = "prior"
            assert len(self.text_embeds) == len(self.video_embeds)
        elif exists(self.video_embeds) and exists(self.videos):
            assert self.texts is None and self.text_embeds is None, \
                "Texts and text embeddings are not needed for decoder training."
            self.stage = "decoder"
            assert len(self.video_embeds) == len(self.videos)
        else:
            raise ValueError("No matching training stage for the given paths.")
        self.collate_fn = CelebVTextCollator(self.videos_ref) if exists(self.videos) else None

    def __len__(self):
        return len(self.texts) if self.stage == "CLIP" else len(self.video_embeds)

    def __getitem__(self, i: int):
        if self.stage == "CLIP":
            return self.texts[i], self.videos[i]
        if self.stage == "prior":
            return self.text_embeds[i], self.video_embeds[i]
        return self.video_embeds[i], self.videos[i]


# ---------------------------------------------------------------------------
# host -> device hand-off
# ---------------------------------------------------------------------------
def _map(obj, fn):
    if torch.is_tensor(obj):
        return fn(obj)
    if isinstance(obj, (list, tuple)):
        out = [_map(o, fn) for o in obj]
        return type(obj)(out) if isinstance(obj, list) else tuple(out)
    if isinstance(obj, dict):
        return {k: _map(v, fn) for k, v in obj.items()}
    return obj


class DeviceLoader:
    """Batches of `loader` delivered on `device` (what accelerate's prepared
    loaders do for the reference, trainer.py:117-124): batch i+1's pinned host
    tensors are copied on a dedicated stream while batch i is consumed; a
    batch is handed out only after the consumer's stream waits for its copy,
    and its memory is not reused before the consumer's work on it is queued
    (record_stream).  CPU devices pass batches through unchanged."""

    def __init__(self, loader, device):
        self.loader = loader
        self.device = torch.device(device)
        self._stream = None

    def __len__(self):
        return len(self.loader)

    def __getattr__(self, name):  # dataset, batch_size, sampler, ... of the wrapped loader
        if name in ("loader", "device", "_stream"):
            raise AttributeError(name)
        return getattr(self.loader, name)

    def _to_device(self, batch):
        def move(t):
            if t.device.type != "cpu":  # already on a device: a plain (stream-ordered) move
                return t.to(self.device, non_blocking=True)
            if not t.is_pinned():
                t = t.pin_memory()
            return t.to(self.device, non_blocking=True)

        with torch.cuda.stream(self._stream):
            out = _map(batch, move)
            ev = torch.cuda.Event()
            ev.record(self._stream)
        return out, ev

    def __iter__(self):
        if self.device.type != "cuda":
            yield from self.loader
            return
        if self._stream is None:
            self._stream = torch.cuda.Stream(device=self.device)
        it = iter(self.loader)
        try:
            nxt = self._to_device(next(it))
        except StopIteration:
            return
        while nxt is not None:
            cur, ev = nxt
            try:
                nxt = self._to_device(next(it))  # copy of the next batch overlaps this one's step
            except StopIteration:
                nxt = None
            consumer = torch.cuda.current_stream(self.device)
            consumer.wait_event(ev)
            _map(cur, lambda t: t.record_stream(consumer))
            yield cur
