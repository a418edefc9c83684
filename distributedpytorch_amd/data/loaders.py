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
from torch.utils.data import DataLoader, Dataset, Sampler, random_split
from torch.utils.data.distributed import DistributedSampler


def split_dataset(dataset: Dataset, val_percent: float, seed: int = 0):
    n_val = int(len(dataset) * val_percent / 100)
    n_train = len(dataset) - n_val
    return random_split(dataset, [n_train, n_val], generator=torch.Generator().manual_seed(seed))


class EpochShuffleSampler(Sampler):
    """Shuffled order that is a pure function of ``(seed, epoch)``.

    Used instead of ``shuffle=True`` (which draws from the process-global torch RNG): every rank
    of a multi-process pipeline iterates its own loader - stage 0 takes the images, the last stage
    the masks - and they pair up only if both see the same order; resuming at epoch ``e``
    replays exactly the order an uninterrupted run would have used (reference shuffled with the
    global RNG, ``utils/train_utils.py:41``)."""

    def __init__(self, n: int, seed: int = 0):
        self.n, self.seed, self.epoch = int(n), int(seed), 0

    def set_epoch(self, epoch: int):
        self.epoch = int(epoch)

    def __len__(self):
        return self.n

    def __iter__(self):
        g = torch.Generator().manual_seed(self.seed * 1_000_003 + self.epoch)
        return iter(torch.randperm(self.n, generator=g).tolist())


def build_loaders(train_set, val_set, batch_size: int, *, rank: int = 0, world_size: int = 1,
                  num_workers: int = 0, pin_memory: bool = False, seed: int = 0, drop_last: bool = False):
    val_sampler = None
    if world_size > 1:
        train_sampler = DistributedSampler(train_set, num_replicas=world_size, rank=rank, shuffle=True,
                                           seed=seed, drop_last=drop_last)
        if len(val_set) >= world_size:
            val_sampler = DistributedSampler(val_set, num_replicas=world_size, rank=rank, shuffle=False,
                                             drop_last=True)
    else:
        train_sampler = EpochShuffleSampler(len(train_set), seed)
    train_loader = DataLoader(train_set, batch_size=batch_size, shuffle=False,
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
