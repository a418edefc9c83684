"""Split + loaders + device prefetch.

Reference: ``utils/train_utils.py:35-42`` (single/MP), ``:110-116`` (DP), ``:186-191`` (DDP).
Fixes: one seeded split everywhere (A8), ``DistributedSampler`` driven with ``set_epoch`` (A7),
validation sharded across ranks and averaged (instead of rank-0-only, A5).

``DeviceBatcher`` overlaps the host->device copy of batch i+1 with compute on batch i using a
dedicated HIP copy stream and pinned memory, and converts the mask to the float ``[B,1,H,W]``
target the loss wants (reference does ``.to(float32).unsqueeze(1)`` on the compute stream).
"""
from __future__ import annotations

from typing import Iterator, Optional

import torch
from torch.utils.data import DataLoader, Dataset, random_split
from torch.utils.data.distributed import DistributedSampler


def split_dataset(dataset: Dataset, val_percent: float, seed: int = 0):
    n_val = int(len(dataset) * val_percent / 100)
    n_train = len(dataset) - n_val
    return random_split(dataset, [n_train, n_val], generator=torch.Generator().manual_seed(seed))


def build_loaders(train_set, val_set, batch_size: int, *, rank: int = 0, world_size: int = 1,
                  num_workers: int = 0, pin_memory: bool = False, seed: int = 0, drop_last: bool = False):
    train_sampler = None
    val_sampler = None
    if world_size > 1:
        train_sampler = DistributedSampler(train_set, num_replicas=world_size, rank=rank, shuffle=True,
                                           seed=seed, drop_last=drop_last)
        if len(val_set) >= world_size:
            val_sampler = DistributedSampler(val_set, num_replicas=world_size, rank=rank, shuffle=False,
                                             drop_last=True)
    train_loader = DataLoader(train_set, batch_size=batch_size, shuffle=train_sampler is None,
                              sampler=train_sampler, num_workers=num_workers, pin_memory=pin_memory,
                              drop_last=drop_last, persistent_workers=num_workers > 0)
    val_loader = DataLoader(val_set, batch_size=batch_size, shuffle=False, sampler=val_sampler,
                            num_workers=num_workers, pin_memory=pin_memory, drop_last=False)
    return train_loader, val_loader, train_sampler


def to_target(mask: torch.Tensor) -> torch.Tensor:
    """int64 ``[B,H,W]`` mask -> float32 ``[B,1,H,W]`` target (train_utils.py:61)."""
    return mask.to(torch.float32).unsqueeze(1)


class DeviceBatcher:
    """Iterate ``(images, targets)`` on ``device``, prefetching one batch ahead on a side stream."""

    def __init__(self, loader, device: torch.device, image_dtype=torch.float32):
        self.loader = loader
        self.device = torch.device(device)
        self.image_dtype = image_dtype
        self.cuda = self.device.type == "cuda"

    def __len__(self):
        return len(self.loader)

    def _move(self, batch):
        img = batch["image"].to(self.device, non_blocking=True).to(self.image_dtype)
        tgt = to_target(batch["mask"].to(self.device, non_blocking=True))
        return img, tgt

    def __iter__(self) -> Iterator:
        if not self.cuda:
            for batch in self.loader:
                yield self._move(batch)
            return
        stream = torch.cuda.Stream(device=self.device)
        it = iter(self.loader)
        nxt: Optional[tuple] = None

        def prefetch():
            try:
                b = next(it)
            except StopIteration:
                return None
            with torch.cuda.stream(stream):
                return self._move(b)

        nxt = prefetch()
        while nxt is not None:
            torch.cuda.current_stream(self.device).wait_stream(stream)
            cur = nxt
            for t in cur:
                t.record_stream(torch.cuda.current_stream(self.device))
            nxt = prefetch()
            yield cur
