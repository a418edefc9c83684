"""Metrics: reference loss-curve pickles + JSONL perf log + throughput meter.

Reference: every 10 steps append ``[step, wallclock_s, mean(last 10 losses)]``,
per epoch ``[step, wallclock_s, val_loss]``; written at the end as pandas pickles
``loss/<method>/{train,val}_loss.pkl`` with columns ``Step, Time, Loss``
(``utils/train_utils.py:75-92``).  The directory is created (defect A4).

Additions: a JSONL log (``logs/<method>.jsonl``) with img/s, step time, Dice, peak HBM; and a
throughput meter that excludes warm-up steps.  Loss values are kept as device tensors and only
synchronised every ``log_every`` steps (defect A17: the reference called ``loss.item()`` every step).
"""
from __future__ import annotations

import json
import os
import time
from typing import List, Optional

import torch


class LossCurves:
    def __init__(self):
        self.train: List[list] = []
        self.val: List[list] = []

    def add_train(self, step: int, t: float, loss: float):
        self.train.append([step, t, loss])

    def add_val(self, step: int, t: float, loss: float):
        self.val.append([step, t, loss])

    def save(self, out_dir: str, method: str):
        import pandas as pd

        d = os.path.join(out_dir, "loss", method)
        os.makedirs(d, exist_ok=True)
        pd.DataFrame(self.train, columns=["Step", "Time", "Loss"]).to_pickle(os.path.join(d, "train_loss.pkl"))
        pd.DataFrame(self.val, columns=["Step", "Time", "Loss"]).to_pickle(os.path.join(d, "val_loss.pkl"))
        return d


class MetricsLogger:
    def __init__(self, path: Optional[str], enabled: bool = True):
        self.path = path
        self.enabled = enabled and path is not None
        if self.enabled:
            os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)

    def log(self, **kw):
        if not self.enabled:
            return
        kw.setdefault("ts", time.time())
        with open(self.path, "a") as f:
            f.write(json.dumps(kw) + "\n")


class Throughput:
    """Images/s over steps after ``warmup`` (device-synchronised at the edges only)."""

    def __init__(self, warmup: int = 2, device=None):
        self.warmup = warmup
        self.device = device
        self.n = 0
        self.images = 0
        self.t0 = None

    def _sync(self):
        if self.device is not None and torch.device(self.device).type == "cuda":
            torch.cuda.synchronize(self.device)

    def step(self, images: int):
        self.n += 1
        if self.n == self.warmup:
            self._sync()
            self.t0 = time.perf_counter()
        elif self.n > self.warmup:
            self.images += images

    def rate(self) -> float:
        if self.t0 is None or self.images == 0:
            return 0.0
        self._sync()
        return self.images / (time.perf_counter() - self.t0)
