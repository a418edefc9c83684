"""GPU-resident synthetic dataset + loader: no DataLoader, collate or host->device copy per step.

The reference decodes and resizes every Carvana JPEG on the CPU inside the training loop
(``utils/dataloading.py:54-73``, ``num_workers`` 0-1: SURVEY K15).  On an MI355X the whole synthetic
dataset fits in HBM many times over (5,088 images at 512x512: 16 GB fp32 of 288 GB), so it is
rendered ONCE on the device and every step only gathers its batch there:

* :class:`DeviceSyntheticSegmentation` - item ``i`` is a pure function of ``(seed, i)``: the same
  ellipse masks, colours and shading as :class:`.synthetic.SyntheticSegmentation` item ``i`` (their
  parameters come from the same per-item CPU generator, drawn in the same order); only the +/-0.05
  pixel noise differs (a counter-based integer hash of (seed, i, c, y, x) evaluated on the device
  instead of the CPU generator's stream).  Images are STORED as uint8 (k/255: what a decoded JPEG
  divided by 255 is, reference ``dataloading.py:40``) -- 4x less HBM than float32, so the 5,088-image
  set is 4 GB at 512x512 and ranks sharing a device in a rehearsal stay small -- and served as float32
  ``[3,H,W]`` in [0,1] (reference item format, ``dataloading.py:70-73``); masks ``uint8``.
* :class:`DeviceLoader` - batches of indices from any sampler (the epoch-seeded shuffle or
  ``DistributedSampler``; ``random_split`` subsets are resolved to base indices), gathered with one
  ``index_select`` each into ``(images float32[B,3,H,W], targets float32[B,1,H,W])``.
"""
from __future__ import annotations

import math
from typing import Iterator, Optional, Sequence

import torch
from torch.utils.data import BatchSampler, Dataset, Subset


def _hash_noise(seed: int, idx: torch.Tensor, c: int, h: int, w: int) -> torch.Tensor:
    """Uniform [0,1) noise of shape [n, c, h, w] from a 32-bit integer hash (lowbias32) of the
    element coordinates: deterministic per (seed, item index), independent of batch composition."""
    dev = idx.device
    n = idx.numel()
    k = (torch.arange(c * h * w, device=dev, dtype=torch.int64).view(1, -1)
         + idx.view(-1, 1).to(torch.int64) * (c * h * w) + (seed & 0x7FFFFFFF) * 0x9E3779B1)
    x = k & 0xFFFFFFFF
    x = x ^ (x >> 16)
    x = (x * 0x7FEB352D) & 0xFFFFFFFF
    x = x ^ (x >> 15)
    x = (x * 0x846CA68B) & 0xFFFFFFFF
    x = x ^ (x >> 16)
    return (x.to(torch.float32) * (1.0 / 4294967296.0)).view(n, c, h, w)


def _item_params(seed: int, idx: int, channels: int):
    """The per-item random draws of ``synthetic._render`` (same generator, same order)."""
    g = torch.Generator().manual_seed(seed * 1_000_003 + idx)
    k = 3
    cy = torch.rand(1, k, generator=g) * 1.2 - 0.6
    cx = torch.rand(1, k, generator=g) * 1.2 - 0.6
    ry = torch.rand(1, k, generator=g) * 0.35 + 0.1
    rx = torch.rand(1, k, generator=g) * 0.35 + 0.1
    fg = torch.rand(1, channels, 1, 1, generator=g) * 0.5 + 0.5
    bg = torch.rand(1, channels, 1, 1, generator=g) * 0.5
    ph = torch.rand(1, 1, 1, 1, generator=g) * 2 * math.pi
    return cy, cx, ry, rx, fg, bg, ph


@torch.no_grad()
def render_items(seed: int, indices: Sequence[int], h: int, w: int, channels: int, device):
    """Render items ``indices`` on ``device``: (images float32 [n,C,h,w], masks uint8 [n,h,w])."""
    ps = [_item_params(seed, int(i), channels) for i in indices]
    cy, cx, ry, rx, fg, bg, ph = (torch.cat([p[j] for p in ps]).to(device) for j in range(7))
    yy = torch.linspace(-1, 1, h, device=device).view(1, h, 1)
    xx = torch.linspace(-1, 1, w, device=device).view(1, 1, w)
    masks = torch.zeros(len(ps), h, w, device=device, dtype=torch.bool)
    for j in range(cy.shape[1]):
        e = ((yy - cy[:, j, None, None]) / ry[:, j, None, None]) ** 2 + \
            ((xx - cx[:, j, None, None]) / rx[:, j, None, None]) ** 2
        masks |= e <= 1.0
    m = masks.unsqueeze(1).float()
    img = m * fg + (1 - m) * bg
    img = img + 0.1 * torch.sin(3 * xx.unsqueeze(0) + 2 * yy.unsqueeze(0) + ph)
    idx = torch.as_tensor(list(indices), device=device)
    img = (img + 0.1 * (_hash_noise(seed, idx, channels, h, w) - 0.5)).clamp_(0, 1)
    return img, masks.to(torch.uint8)


class DeviceSyntheticSegmentation(Dataset):
    """The whole synthetic dataset rendered into device memory (see module docstring)."""

    def __init__(self, length: int, size=(512, 512), channels: int = 3, seed: int = 0, device="cuda",
                 chunk: int = 64):
        self.length = int(length)
        self.h, self.w = int(size[0]), int(size[1])
        self.channels, self.seed = channels, seed
        self.device = torch.device(device)
        import logging
        logging.getLogger(__name__).info(
            "rendering %d synthetic %dx%d images into %s: %.2f GiB (uint8 images + masks)", self.length, self.h,
            self.w, self.device, self.length * (channels + 1) * self.h * self.w / 2 ** 30)
        self.images = torch.empty(self.length, channels, self.h, self.w, dtype=torch.uint8, device=self.device)
        self.masks = torch.empty(self.length, self.h, self.w, dtype=torch.uint8, device=self.device)
        for s in range(0, self.length, chunk):
            e = min(self.length, s + chunk)
            img, self.masks[s:e] = render_items(seed, range(s, e), self.h, self.w, channels, self.device)
            self.images[s:e] = img.mul_(255.0).round_().to(torch.uint8)

    @property
    def nbytes(self) -> int:
        return self.images.numel() + self.masks.numel()

    def __len__(self):
        return self.length

    @staticmethod
    def to_float(img_u8: torch.Tensor) -> torch.Tensor:
        return img_u8.to(torch.float32).mul_(1.0 / 255.0)

    def __getitem__(self, idx):
        return {"image": self.to_float(self.images[idx]), "mask": self.masks[idx].long()}


def _base(ds):
    """(device dataset, index map) through nested ``Subset`` wrappers (``random_split``)."""
    idx = None
    while isinstance(ds, Subset):
        sub = torch.as_tensor(ds.indices, dtype=torch.int64)
        idx = sub if idx is None else sub[idx]
        ds = ds.dataset
    assert isinstance(ds, DeviceSyntheticSegmentation), type(ds)
    return ds, idx


class DeviceLoader:
    """Batches gathered on the device; yields ``(images, targets)`` like ``loaders.DeviceBatcher``."""

    def __init__(self, dataset, batch_size: int, sampler=None, drop_last: bool = False):
        self.base, idx = _base(dataset)
        self.n = len(dataset)
        self.index_map = None if idx is None else idx.to(self.base.device)
        self.sampler = sampler if sampler is not None else range(self.n)
        self.batches = BatchSampler(self.sampler, batch_size, drop_last)

    def __len__(self):
        return len(self.batches)

    def __iter__(self) -> Iterator:
        dev = self.base.device
        for b in self.batches:
            i = torch.as_tensor(b, dtype=torch.int64).to(dev, non_blocking=True)
            if self.index_map is not None:
                i = self.index_map.index_select(0, i)
            img = self.base.to_float(self.base.images.index_select(0, i))
            tgt = self.base.masks.index_select(0, i).to(torch.float32).unsqueeze(1)
            yield img, tgt


def device_loaders(train_set, val_set, batch_size: int, *, rank: int = 0, world_size: int = 1, seed: int = 0,
                   drop_last: bool = False):
    """``loaders.build_loaders`` for a device-resident dataset (same samplers, same batches)."""
    from torch.utils.data.distributed import DistributedSampler
    from .loaders import EpochShuffleSampler
    val_sampler: Optional[object] = None
    if world_size > 1:
        train_sampler = DistributedSampler(train_set, num_replicas=world_size, rank=rank, shuffle=True, seed=seed,
                                           drop_last=drop_last)
        if len(val_set) >= world_size:
            val_sampler = DistributedSampler(val_set, num_replicas=world_size, rank=rank, shuffle=False,
                                             drop_last=True)
    else:
        train_sampler = EpochShuffleSampler(len(train_set), seed)
    return (DeviceLoader(train_set, batch_size, train_sampler, drop_last),
            DeviceLoader(val_set, batch_size, val_sampler, False), train_sampler)
