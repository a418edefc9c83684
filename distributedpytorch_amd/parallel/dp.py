"""Single-process multi-GPU data parallelism (``-t DP``).

Reference: ``torch.nn.DataParallel`` (``utils/train_utils.py:95-167``), which
broadcasts all parameters from cuda:0 every forward, scatters the batch, runs one thread per
GPU, gathers outputs to cuda:0 and reduces gradients back to cuda:0.  As written it crashed (A1:
CPU model, A2: mask shape) - we implement the intended behaviour.

MI355X design (same semantics, less traffic):
* one persistent replica per device, each with its own flat fp32 param/grad buffer and its own
  fused Adam -> no per-step parameter broadcast (N6 disappears); replicas stay bit-identical
  because they apply the same update to the same data with a deterministic kernel.
* the loss keeps the reference's *global-batch* semantics without gathering outputs (N8): each
  device produces the 4 partial loss sums of its shard, they are added on device 0 and the scalar
  loss is back-propagated through those tiny copies into every replica.
* gradients are summed across devices with one single-process RCCL all-reduce over the flat
  buffers: the native clique of :mod:`.dp_comm` (csrc/dp_comm.cpp: ncclCommInitAll once, then one
  grouped ncclAllReduce per step on each device's compute stream), each device riding its own
  xGMI links; fallbacks: ``torch.cuda.nccl.all_reduce``, then ``torch.cuda.comm`` reduce+broadcast.
  The initial replicas are made identical with one grouped ncclBroadcast of the flat parameters.
* per-device forward runs on one host thread per device (kernel launch cost overlaps).

On CPU (tests) "devices" may repeat ``cpu``; the all-reduce is then a plain sum.
"""
from __future__ import annotations

import copy
import os
import threading
from typing import List, Sequence

import torch

from ..compute import loss_from_partials, make_compute
from ..optim import FlatParameterSpace


class ReplicatedDataParallel:
    def __init__(self, model: torch.nn.Module, devices: Sequence, backend: str = "auto", dtype: str = "bf16"):
        self.devices = [torch.device(d) for d in devices]
        assert len(self.devices) >= 1
        self.replicas: List[torch.nn.Module] = []
        for i, d in enumerate(self.devices):
            r = model if i == 0 else copy.deepcopy(model)
            self.replicas.append(r.to(d))
        self.spaces = [FlatParameterSpace(r, device=d) for r, d in zip(self.replicas, self.devices)]
        self.computes = [make_compute(r, backend, dtype) for r in self.replicas]
        self.module = self.replicas[0]
        self._nccl = all(d.type == "cuda" for d in self.devices) and len(self.devices) > 1 and \
            len({d.index for d in self.devices}) == len(self.devices)
        self.comm = None
        if self._nccl and os.environ.get("DPA_DP_NATIVE_COMM", "1") == "1":
            from . import dp_comm
            if dp_comm.available():
                self.comm = dp_comm.DPComm(self.devices)
                self.comm.broadcast([s.data for s in self.spaces], root=0)
                for s in self.spaces:
                    s.touch()

    # ------------------------------------------------------------------ forward
    def _parallel(self, fn, args_per_dev):
        if len(self.devices) == 1 or not self.devices[0].type == "cuda":
            return [fn(i, *a) for i, a in enumerate(args_per_dev)]
        out = [None] * len(self.devices)
        err = [None] * len(self.devices)

        def run(i, a):
            try:
                with torch.cuda.device(self.devices[i]):
                    out[i] = fn(i, *a)
            except BaseException as e:  # propagate to the caller thread
                err[i] = e

        th = [threading.Thread(target=run, args=(i, a)) for i, a in enumerate(args_per_dev)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        for e in err:
            if e is not None:
                raise e
        return out

    def scatter(self, x: torch.Tensor) -> List[torch.Tensor]:
        chunks = x.chunk(len(self.devices), dim=0)
        assert len(chunks) == len(self.devices), "batch smaller than the number of devices"
        return [c.to(d, non_blocking=True) for c, d in zip(chunks, self.devices)]

    def forward_loss(self, images: torch.Tensor, targets: torch.Tensor, dice: bool = True):
        xs, ts = self.scatter(images), self.scatter(targets)
        parts = self._parallel(lambda i, x, t: self.computes[i].forward_partials(x, t), list(zip(xs, ts)))
        d0 = self.devices[0]
        S = sum(p.to(d0) for p in parts)
        return loss_from_partials(S, targets.numel(), dice)

    @torch.no_grad()
    def probs(self, images: torch.Tensor) -> torch.Tensor:
        xs = self.scatter(images)
        outs = self._parallel(lambda i, x: self.computes[i].probs(x), [(x,) for x in xs])
        return torch.cat([o.to(self.devices[0]) for o in outs])

    # ------------------------------------------------------------------ grads
    def zero_grad(self):
        for s in self.spaces:
            s.zero_grad()

    def all_reduce_grads(self):
        grads = [s.grad for s in self.spaces]
        if len(grads) == 1:
            return
        if self.comm is not None:
            self.comm.all_reduce(grads, "sum")
            return
        if self._nccl:
            try:
                import torch.cuda.nccl as nccl
                if nccl.is_available(grads):
                    nccl.all_reduce(grads)
                    return
            except (RuntimeError, ImportError):
                pass
            total = torch.cuda.comm.reduce_add(grads, destination=self.devices[0].index)
            outs = torch.cuda.comm.broadcast(total, devices=[d.index for d in self.devices])
            for g, o in zip(grads, outs):
                g.copy_(o)
            return
        total = grads[0].clone()
        for g in grads[1:]:
            total += g.to(total.device)
        for g in grads:
            g.copy_(total.to(g.device))

    @torch.no_grad()
    def sync_buffers(self):
        """Replica 0's floating-point buffers (BatchNorm running statistics) to every replica."""
        src = [b for b in self.replicas[0].buffers()]
        for r in self.replicas[1:]:
            for b, s in zip(r.buffers(), src):
                b.copy_(s.to(b.device))

    @torch.no_grad()
    def sync_from_replica0(self):
        """After replica 0's parameters were overwritten (resume): replicate them and its buffers."""
        if self.comm is not None:
            self.comm.broadcast([s.data for s in self.spaces], root=0)
        else:
            for s in self.spaces[1:]:
                s.data.copy_(self.spaces[0].data.to(s.data.device))
        for s in self.spaces:
            s.touch()
        self.sync_buffers()

    def state_dict(self):
        return self.module.state_dict()
