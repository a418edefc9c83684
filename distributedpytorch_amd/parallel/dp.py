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
* gradients are summed across devices by bucketed single-process RCCL all-reduces overlapped with
  the backward (:class:`DPBucketReducer`): the flat gradient buffers are cut into the same
  contiguous buckets as DDP's (``ddp.bucket_plan``); the HIP backward announces finished
  gradients block by block on every replica (``space.notify_ready``, autograd hooks for the torch
  backend) and as soon as a bucket is final on ALL replicas one grouped ncclAllReduce over that
  slice runs on per-device comm streams (the native clique of :mod:`.dp_comm`, csrc/dp_comm.cpp:
  ncclCommInitAll once), each device riding its own xGMI links while the earlier (full-resolution)
  layers' backward still computes.  The initial replicas are made identical with one grouped
  ncclBroadcast of the flat parameters.  Without the native clique (CPU tests, same-device
  rehearsal) the same bucket schedule sums the slices directly.
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
from ..utils.tracing import trace_range
from .ddp import bucket_plan


class ReplicatedDataParallel:
    def __init__(self, model: torch.nn.Module, devices: Sequence, backend: str = "auto", dtype: str = "bf16",
                 bucket_mb: float = 8.0, overlap: bool = True):
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
        self.reducer = DPBucketReducer(self.spaces, self.devices, self.comm, bucket_mb, overlap=overlap) \
            if len(self.devices) > 1 else None

    # ------------------------------------------------------------------ forward
    def _parallel(self, fn, args_per_dev):
        if len(self.devices) == 1 or not self.devices[0].type == "cuda":
            return [fn(i, *a) for i, a in enumerate(args_per_dev)]
        out = [None] * len(args_per_dev)
        err = [None] * len(args_per_dev)

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
        """torch.nn.DataParallel's split: ceil(B / n) images per replica, so a batch smaller than the
        replica count (a short last or validation batch) feeds only the first replicas."""
        chunks = x.chunk(len(self.devices), dim=0)
        return [c.to(d, non_blocking=True) for c, d in zip(chunks, self.devices)]

    def forward_loss(self, images: torch.Tensor, targets: torch.Tensor, dice: bool = True):
        xs, ts = self.scatter(images), self.scatter(targets)
        if len(xs) < len(self.devices) and self.reducer is not None and torch.is_grad_enabled():
            # replicas without images this step: their (zeroed) gradients are final now
            for k in range(len(xs), len(self.devices)):
                for i in range(len(self.spaces[k].numels)):
                    self.reducer.mark_ready(i, k)
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
        """End of the backward: launch the buckets not started yet, then every compute stream
        waits for its comm stream (the optimizer reads summed gradients)."""
        if self.reducer is not None:
            self.reducer.finish()

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


class DPBucketReducer:
    """Bucketed, backward-overlapped gradient sum across the replicas of one process.

    Readiness arrives from several threads (the autograd engine runs one worker thread per device;
    each replica's backward calls its flat space's ``notify_ready``), so the per-bucket counters
    are guarded by a lock; the thread that completes a bucket on the last replica launches it.
    Buckets launch strictly in index order.  On GPUs with the native clique each bucket is one
    grouped ncclAllReduce (sum) over the slices, issued on per-device comm streams that first wait
    for their device's compute stream; :meth:`finish` makes every compute stream wait for its comm
    stream and records the exposed (un-overlapped) wait on device 0."""

    def __init__(self, spaces, devices, comm=None, bucket_mb: float = 8.0, first_bucket_mb: float = 1.0,
                 overlap: bool = True):
        self.spaces, self.devices, self.comm = list(spaces), list(devices), comm
        # overlap=False (``--no-comm-overlap``): ONE reduction of the whole gradient buffer after the
        # backward (no bucket launches from the autograd device threads)
        self.overlap = bool(overlap)
        if self.overlap:
            self.buckets, self.bucket_of = bucket_plan(self.spaces[0], bucket_mb, first_bucket_mb)
        else:
            n = len(self.spaces[0].numels)
            self.buckets, self.bucket_of = [(0, self.spaces[0].offsets[-1], 0, n)], [0] * n
        for sp in self.spaces[1:]:
            assert sp.offsets == self.spaces[0].offsets, "replicas must share one flat layout"
        self.expected = [(b[3] - b[2]) * len(self.spaces) for b in self.buckets]
        self.lock = threading.Lock()
        self.streams = ([torch.cuda.Stream(device=d) for d in self.devices] if comm is not None else None)
        self._exposed = None
        self._hooks = []
        for k, sp in enumerate(self.spaces):
            sp.add_ready_listener(lambda i, k=k: self.mark_ready(i, k))
            for i, p in enumerate(sp.params):       # torch-op backend: autograd accumulation hooks
                self._hooks.append(p.register_post_accumulate_grad_hook(lambda _p, i=i, k=k: self.mark_ready(i, k)))
        self.reset()

    def reset(self):
        if getattr(self, "launch_log", None):
            self.last_launch_log = self.launch_log
        self.pending = list(self.expected)
        self.seen = [[False] * len(self.bucket_of) for _ in self.spaces]
        self.n_ready = 0
        self.next_launch = 0
        self.launch_log = []     # (bucket, announcements so far, launched by finish())

    def mark_ready(self, param_index: int, replica: int = 0):
        with self.lock:
            assert not self.seen[replica][param_index], \
                f"replica {replica}: gradient of parameter {param_index} announced twice in one step"
            self.seen[replica][param_index] = True
            self.n_ready += 1
            self.pending[self.bucket_of[param_index]] -= 1
            while (self.overlap and self.next_launch < len(self.buckets)
                   and self.pending[self.next_launch] == 0):
                self._launch(self.next_launch)
                self.next_launch += 1

    def _launch(self, b: int, in_finish: bool = False):
        self.launch_log.append((b, self.n_ready, in_finish))
        s, e = self.buckets[b][:2]
        grads = [sp.grad[s:e] for sp in self.spaces]
        with trace_range(f"dp_allreduce_bucket{b}"):
            if self.comm is not None:
                for d, st in zip(self.devices, self.streams):
                    st.wait_stream(torch.cuda.current_stream(d))   # the slice's gradients are enqueued
                self.comm.all_reduce(grads, "sum", streams=self.streams)
                return
            total = grads[0].clone()
            for g in grads[1:]:
                total += g.to(total.device)
            for g in grads:
                g.copy_(total.to(g.device))

    def finish(self):
        with self.lock:
            while self.next_launch < len(self.buckets):
                self._launch(self.next_launch, in_finish=True)
                self.next_launch += 1
            if self.streams is not None:
                cur0 = torch.cuda.current_stream(self.devices[0])
                ev0 = torch.cuda.Event(enable_timing=True)
                ev0.record(cur0)
                for d, st in zip(self.devices, self.streams):
                    torch.cuda.current_stream(d).wait_stream(st)
                ev1 = torch.cuda.Event(enable_timing=True)
                ev1.record(cur0)
                self._exposed = (ev0, ev1)
            self.reset()

    def exposed_comm_ms(self):
        if self._exposed is None:
            return None
        self._exposed[1].synchronize()
        return float(self._exposed[0].elapsed_time(self._exposed[1]))
