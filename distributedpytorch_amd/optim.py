"""Optimiser + LR schedule.

Reference: ``Adam(lr, weight_decay=1e-8)`` + ``ReduceLROnPlateau('min', patience=2)``
(``utils/train_utils.py:45-46,120-121,199-200``).  Adam's weight decay there is the
classic L2 form (added to the gradient, not decoupled), which is what we implement.

MI355X design:
* :class:`FlatParameterSpace` re-homes every parameter and gradient of a module into ONE contiguous
  fp32 buffer each, laid out in *backward order* (last layer first).  Gradient buckets for the
  data-parallel all-reduce are then plain contiguous slices (no pack/unpack copies, no per-tensor
  launches), and the optimiser update is a single kernel over the whole buffer.
* :class:`FusedAdam` runs one HIP launch (``ops.adam_step``) over the flat buffer on GPU and the
  same math on CPU via torch ops.  It keeps ``param_groups`` so torch schedulers work unchanged.
* :func:`plateau_step` makes the ReduceLROnPlateau decision identical on every rank (fix for
  reference defect A5: there only rank 0 stepped the scheduler and replicas diverged).
"""
from __future__ import annotations

import math
from typing import Iterable, List, Optional

import torch
import torch.distributed as dist
import torch.nn as nn


def _hip_available() -> bool:
    from .ops import _lib
    return _lib.available()


class FlatParameterSpace:
    """Make every parameter/grad of ``module`` a view into one flat fp32 buffer (backward order)."""

    def __init__(self, module, device=None, order: str = "backward"):
        if isinstance(module, nn.Module):
            named = [(n, p) for n, p in module.named_parameters() if p.requires_grad]
        else:  # iterable of (name, param)
            named = [(n, p) for n, p in module if p.requires_grad]
        if order == "backward":
            if isinstance(module, nn.Module) and hasattr(module, "cfg") and hasattr(module, "decoder"):
                from .models.unet import backward_param_order
                rank = {n: i for i, n in enumerate(backward_param_order(module))}
                named = sorted(named, key=lambda kv: rank.get(kv[0], len(rank)))
            else:
                named = list(reversed(named))
        self.names = [n for n, _ in named]
        self.params: List[nn.Parameter] = [p for _, p in named]
        device = torch.device(device) if device is not None else self.params[0].device
        self.numels = [p.numel() for p in self.params]
        self.offsets = [0]
        for n in self.numels:
            self.offsets.append(self.offsets[-1] + n)
        total = self.offsets[-1]
        self.data = torch.empty(total, dtype=torch.float32, device=device)
        self.grad = torch.zeros(total, dtype=torch.float32, device=device)
        for p, o, n in zip(self.params, self.offsets, self.numels):
            self.data[o:o + n].copy_(p.detach().reshape(-1))
            p.data = self.data[o:o + n].view_as(p)
            p.grad = self.grad[o:o + n].view_as(p)
        self._index = {id(p): i for i, p in enumerate(self.params)}
        for p in self.params:
            p._dpa_space = self          # lets kernel engines find the space owning a parameter
        self.version = 0                 # bumped whenever parameter values change (optimizer, sync, load)
        self._ready_listeners = []       # called with param indices whose gradient is final
        if isinstance(module, nn.Module):
            module._flat_space = self

    def touch(self):
        """Record that parameter values changed (kernels that cache packed weights re-pack)."""
        self.version += 1

    def add_ready_listener(self, fn):
        self._ready_listeners.append(fn)

    def notify_ready(self, params):
        """Explicit-backward engines announce finished gradients (replaces autograd hooks)."""
        if not self._ready_listeners:
            return
        idx = [self._index[id(p)] for p in params if id(p) in self._index]
        for fn in self._ready_listeners:
            for i in idx:
                fn(i)

    @property
    def numel(self) -> int:
        return self.offsets[-1]

    def index_of(self, p: torch.Tensor) -> int:
        return self._index[id(p)]

    def slice_of(self, i: int):
        return self.offsets[i], self.offsets[i + 1]

    def zero_grad(self):
        if self.grad.is_cuda and _hip_available():
            from .ops.kernels import zero_
            zero_(self.grad)                 # a DMA memset: no compute kernel in the step
        else:
            self.grad.zero_()
        # autograd may have replaced .grad with a fresh tensor (e.g. after set_to_none); re-bind
        for p, o, n in zip(self.params, self.offsets, self.numels):
            if p.grad is None or p.grad.data_ptr() != self.grad[o:o + n].data_ptr():
                p.grad = self.grad[o:o + n].view_as(p)

    def rebind(self):
        for p, o, n in zip(self.params, self.offsets, self.numels):
            if p.data.data_ptr() != self.data[o:o + n].data_ptr():
                self.data[o:o + n].copy_(p.data.reshape(-1))
                p.data = self.data[o:o + n].view_as(p)
        self.touch()


def spaces_by_device(module: nn.Module) -> List[FlatParameterSpace]:
    """One flat space per device holding the module's parameters (multi-device single process)."""
    groups = {}
    for n, p in module.named_parameters():
        if p.requires_grad:
            groups.setdefault(p.device, []).append((n, p))
    return [FlatParameterSpace(v, device=d) for d, v in groups.items()]


class FusedAdam(torch.optim.Optimizer):
    """Adam with L2 weight decay over one or more :class:`FlatParameterSpace` (one launch per space).

    Several spaces occur when a single process owns parameters on several devices (``-t DP``
    replicas, single-process ``-t MP`` stages); each device then runs its own fused update.
    """

    def __init__(self, spaces, lr=1e-4, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.0,
                 use_kernel: Optional[bool] = None):
        if isinstance(spaces, FlatParameterSpace):
            spaces = [spaces]
        self.spaces: List[FlatParameterSpace] = list(spaces)
        params = [p for s in self.spaces for p in s.params]
        defaults = dict(lr=lr, betas=betas, eps=eps, weight_decay=weight_decay)
        super().__init__(params, defaults)
        self.exp_avg = [torch.zeros_like(s.data) for s in self.spaces]
        self.exp_avg_sq = [torch.zeros_like(s.data) for s in self.spaces]
        self.step_count = 0
        self.use_kernel = use_kernel
        self.device_state = False
        self._dev_state: List[torch.Tensor] = []
        self._dev_lr = None

    def enable_device_state(self):
        """Keep (step, lr, bias corrections) in a per-space fp64 device block that the step kernel
        updates itself: the launch sequence is then identical every step and can be captured once in
        a HIP graph.  The host mirror ``step_count`` is kept by the caller of the replay."""
        if not self.device_state:
            self.device_state = True
            self._dev_state = [torch.zeros(4, dtype=torch.float64, device=s.data.device) for s in self.spaces]
        self.sync_device_state()

    def sync_device_state(self):
        """Upload the host step count and lr (after a restore, a resume or an LR plateau cut)."""
        lr = float(self.param_groups[0]["lr"])
        for st in self._dev_state:
            st.copy_(torch.tensor([float(self.step_count), lr, 0.0, 0.0], dtype=torch.float64))
        self._dev_lr = lr

    @property
    def space(self) -> FlatParameterSpace:
        return self.spaces[0]

    def zero_grad(self, set_to_none: bool = False):  # keep the flat views alive
        for s in self.spaces:
            s.zero_grad()

    @torch.no_grad()
    def step(self, closure=None):
        loss = closure() if closure is not None else None
        g = self.param_groups[0]
        self.step_count += 1
        b1, b2 = g["betas"]
        lr, eps, wd = g["lr"], g["eps"], g["weight_decay"]
        bc1 = 1 - b1 ** self.step_count
        bc2 = 1 - b2 ** self.step_count
        if self.device_state:
            from . import ops
            if lr != self._dev_lr and not _capturing(self.spaces[0].data):
                self.step_count -= 1
                self.sync_device_state()
                self.step_count += 1
            for s, m, v, st in zip(self.spaces, self.exp_avg, self.exp_avg_sq, self._dev_state):
                s.touch()
                ops.adam_step_dev(s.data, s.grad, m, v, st, beta1=b1, beta2=b2, eps=eps, weight_decay=wd)
            return loss
        for s, m, v in zip(self.spaces, self.exp_avg, self.exp_avg_sq):
            s.touch()
            use_k = s.data.is_cuda if self.use_kernel is None else self.use_kernel
            if use_k:
                from . import ops
                ops.adam_step(s.data, s.grad, m, v, lr=lr, beta1=b1, beta2=b2, eps=eps,
                              weight_decay=wd, bc1=bc1, bc2=bc2)
            else:
                adam_reference(s.data, s.grad, m, v, lr, b1, b2, eps, wd, bc1, bc2)
        return loss

    def state_dict(self):
        return {"step": self.step_count,
                "exp_avg": [m.detach().cpu() for m in self.exp_avg],
                "exp_avg_sq": [v.detach().cpu() for v in self.exp_avg_sq],
                "names": [s.names for s in self.spaces],
                "param_groups": [{k: v for k, v in g.items() if k != "params"} for g in self.param_groups]}

    def load_state_dict(self, sd):
        # the moments are flat buffers matched by position: refuse a state whose parameter layout
        # differs (another --mp-cut / --stages, another model) instead of loading foreign moments
        mine = [list(s.names) for s in self.spaces]
        saved = sd.get("names")
        if saved is not None and [list(n) for n in saved] != mine:
            def brief(nn):
                return [f"{len(n)} params ({n[0]} .. {n[-1]})" if n else "0 params" for n in nn]
            raise ValueError(f"optimizer state was saved for a different parameter layout: saved {brief(saved)}, "
                             f"this run {brief(mine)} (same --mp-cut/--stages/model needed to resume)")
        if len(sd["exp_avg"]) != len(self.exp_avg) or any(
                tuple(a.shape) != tuple(b.shape) for a, b in zip(self.exp_avg, sd["exp_avg"])):
            raise ValueError("optimizer state buffers do not match this run's flat parameter spaces")
        self.step_count = int(sd["step"])
        for m, src in zip(self.exp_avg, sd["exp_avg"]):
            m.copy_(src)
        for v, src in zip(self.exp_avg_sq, sd["exp_avg_sq"]):
            v.copy_(src)
        for g, s in zip(self.param_groups, sd["param_groups"]):
            g.update(s)
        if self.device_state:
            self.sync_device_state()


def _capturing(t: torch.Tensor) -> bool:
    return t.is_cuda and torch.cuda.is_current_stream_capturing()


@torch.no_grad()
def adam_reference(p, g, m, v, lr, b1, b2, eps, wd, bc1, bc2):
    """torch.optim.Adam (non-amsgrad, L2 decay) math, in place on flat tensors."""
    grad = g.add(p, alpha=wd) if wd != 0 else g
    m.mul_(b1).add_(grad, alpha=1 - b1)
    v.mul_(b2).addcmul_(grad, grad, value=1 - b2)
    denom = (v.sqrt() / math.sqrt(bc2)).add_(eps)
    p.addcdiv_(m, denom, value=-lr / bc1)


def make_plateau(optimizer, patience: int = 2):
    return torch.optim.lr_scheduler.ReduceLROnPlateau(optimizer, "min", patience=patience)


def plateau_step(scheduler, val_loss: float):
    """Step ``scheduler`` with the same value on every rank (all ranks pass the global val loss)."""
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        t = torch.tensor([float(val_loss)], dtype=torch.float64)
        if dist.get_backend() == "nccl":
            t = t.cuda()
        dist.broadcast(t, src=0)
        val_loss = float(t.item())
    scheduler.step(val_loss)
