"""Synthetic segmentation data: random smooth images with learnable binary masks.

The reference needs the Carvana download (README.md:18).  Every benchmark/test config here runs
on synthetic data of the same shape instead (BASELINE.json: "synthetic masks / random-init
weights").  Masks are unions of random ellipses and the image is a noisy, colour-shifted render
of the mask, so the segmentation task is learnable and Dice is a meaningful parity metric.

Items follow the reference item format (dataloading.py:70-73):
``{'image': float32[3,H,W] in [0,1], 'mask': int64[H,W] in {0,1}}``.
"""
from __future__ import annotations

import math

import torch
from torch.utils.data import Dataset


def _render(gen: torch.Generator, n: int, h: int, w: int, channels: int, device="cpu"):
    yy = torch.linspace(-1, 1, h, device=device).view(1, h, 1)
    xx = torch.linspace(-1, 1, w, device=device).view(1, 1, w)
    masks = torch.zeros(n, h, w, device=device, dtype=torch.bool)
    k = 3
    cy = torch.rand(n, k, generator=gen, device="cpu").to(device) * 1.2 - 0.6
    cx = torch.rand(n, k, generator=gen, device="cpu").to(device) * 1.2 - 0.6
    ry = torch.rand(n, k, generator=gen, device="cpu").to(device) * 0.35 + 0.1
    rx = torch.rand(n, k, generator=gen, device="cpu").to(device) * 0.35 + 0.1
    for j in range(k):
        e = ((yy - cy[:, j, None, None]) / ry[:, j, None, None]) ** 2 + \
            ((xx - cx[:, j, None, None]) / rx[:, j, None, None]) ** 2
        masks |= e <= 1.0
    fg = torch.rand(n, channels, 1, 1, generator=gen).to(device) * 0.5 + 0.5
    bg = torch.rand(n, channels, 1, 1, generator=gen).to(device) * 0.5
    m = masks.unsqueeze(1).float()
    img = m * fg + (1 - m) * bg
    # low-frequency shading + pixel noise
    ph = torch.rand(n, 1, 1, 1, generator=gen).to(device) * 2 * math.pi
    img = img + 0.1 * torch.sin(3 * xx.unsqueeze(0) + 2 * yy.unsqueeze(0) + ph)
    noise = torch.rand(img.shape, generator=gen).to(device) if device == "cpu" else \
        torch.rand(img.shape, device=device)
    img = (img + 0.1 * (noise - 0.5)).clamp_(0, 1)
    return img.float(), masks.long()


def synthetic_batch(n: int, h: int, w: int, channels: int = 3, seed: int = 0, device="cpu"):
    """One batch ``(images float32[n,C,h,w], masks int64[n,h,w])`` generated directly on ``device``."""
    gen = torch.Generator().manual_seed(seed)
    return _render(gen, n, h, w, channels, device=device)


class SyntheticSegmentation(Dataset):
    """Deterministic per-index synthetic dataset (item ``i`` depends only on ``(seed, i)``)."""

    def __init__(self, length: int = 64, size=(128, 128), channels: int = 3, seed: int = 0):
        self.length = int(length)
        # reference newsize is (W, H) (utils/train_utils.py:26); we take (H, W)
        self.h, self.w = int(size[0]), int(size[1])
        self.channels = channels
        self.seed = seed

    def __len__(self):
        return self.length

    def __getitem__(self, idx):
        if idx < 0:
            idx += self.length
        if not 0 <= idx < self.length:
            raise IndexError(idx)
        gen = torch.Generator().manual_seed(self.seed * 1_000_003 + idx)
        img, mask = _render(gen, 1, self.h, self.w, self.channels)
        return {"image": img[0].contiguous(), "mask": mask[0].contiguous()}
