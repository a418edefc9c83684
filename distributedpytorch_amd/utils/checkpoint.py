"""Checkpoints with the reference's file names and key layout, plus full training state.

Reference: ``torch.save(model.state_dict())`` once at the end to
``checkpoints/{singleGPU,DP,DDP}.pth`` (DP/DDP keys prefixed ``module.``; MP wrote singleGPU.pth,
A9), loaded with ``torch.load(f"checkpoints\\{name}.pth")`` (Windows path, A3).

Here:
* ``save_model`` writes ``checkpoints/<method>.pth`` with plain NCHW/OIHW fp32 tensors on CPU.
  ``module_prefix=True`` reproduces the ``module.`` prefix of DP/DDP checkpoints for layout parity.
* ``load_model_state`` accepts either layout (prefix-tolerant) and maps to CPU first.
* ``save_training_state``/``load_training_state`` add optimizer, scheduler, epoch, step and RNG state
  for resume (``checkpoints/<method>_last.pt``), written atomically (tmp + rename).
Everything is loaded with ``weights_only=True``.
"""
from __future__ import annotations

import os
import random
from typing import Dict

import numpy as np
import torch


def strip_prefix(sd: Dict[str, torch.Tensor], prefix: str = "module.") -> Dict[str, torch.Tensor]:
    if sd and all(k.startswith(prefix) for k in sd):
        return {k[len(prefix):]: v for k, v in sd.items()}
    return sd


def _atomic_save(obj, path: str):
    os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    tmp = path + ".tmp"
    torch.save(obj, tmp)
    os.replace(tmp, path)


def save_model(model: torch.nn.Module, path: str, module_prefix: bool = False):
    sd = {k: v.detach().to("cpu", torch.float32) if v.is_floating_point() else v.detach().cpu()
          for k, v in model.state_dict().items()}
    if module_prefix:
        sd = {"module." + k: v for k, v in sd.items()}
    _atomic_save(sd, path)
    return path


def load_model_state(model: torch.nn.Module, path: str, strict: bool = True):
    sd = torch.load(path, map_location="cpu", weights_only=True)
    sd = strip_prefix(sd)
    with torch.no_grad():
        missing, unexpected = model.load_state_dict(sd, strict=strict)
    return missing, unexpected


def save_training_state(path: str, *, model, optimizer=None, scheduler=None, epoch: int = 0, step: int = 0,
                        extra=None):
    state = {
        "model": {k: v.detach().cpu() for k, v in model.state_dict().items()},
        "optimizer": None if optimizer is None else _cpu(optimizer.state_dict()),
        "scheduler": None if scheduler is None else scheduler.state_dict(),
        "epoch": epoch, "step": step,
        "rng": {"torch": torch.get_rng_state(), "numpy": _np_state(), "python": repr(random.getstate())},
        "extra": extra or {},
    }
    _atomic_save(state, path)


def load_training_state(path: str, *, model, optimizer=None, scheduler=None):
    state = torch.load(path, map_location="cpu", weights_only=True)
    with torch.no_grad():
        model.load_state_dict(strip_prefix(state["model"]))
    if optimizer is not None and state.get("optimizer") is not None:
        optimizer.load_state_dict(state["optimizer"])
    if scheduler is not None and state.get("scheduler") is not None:
        scheduler.load_state_dict(state["scheduler"])
    torch.set_rng_state(state["rng"]["torch"])
    return state["epoch"], state["step"]


def _cpu(obj):
    if isinstance(obj, torch.Tensor):
        return obj.detach().cpu()
    if isinstance(obj, dict):
        return {k: _cpu(v) for k, v in obj.items()}
    if isinstance(obj, (list, tuple)):
        return type(obj)(_cpu(v) for v in obj)
    return obj


def _np_state():
    s = np.random.get_state()
    return {"name": s[0], "keys": torch.from_numpy(s[1].astype(np.int64)), "pos": s[2]}
