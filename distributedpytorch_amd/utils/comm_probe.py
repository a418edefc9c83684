"""Does an RCCL gradient bucket get CUs while the backward runs?  A one-GPU measurement (VERDICT r5 #3c).

DDP's bucketed all-reduce (:mod:`..parallel.ddp`, reference ``utils/train_utils.py:195-224`` / SURVEY N4)
launches a bucket the moment its gradients are final, while the rest of the backward still computes.  The
backward's GEMMs run one 512-thread workgroup per CU holding 131-149 KB of LDS, so a collective's kernel
may find no CU with room for its workgroups until a GEMM workgroup retires.  Without a second GPU no RCCL
kernel runs, so this module measures the proxy: at every bucket-ready point of a single-device step it
launches a bucket-sized copy with RCCL's geometry (``blocks`` workgroups of 256 threads,
``ops.kernels.comm_probe``) on a stream of its own that first waits for the compute stream's work so far
(exactly the dependency ``ProcessGroupNCCL`` gives its stream) and records

* ``total_us``: the probe stream's event pair around the kernel (wait for CUs + run),
* ``run_us``: first workgroup start to last workgroup end (the kernel's own constant-clock stamps),
* ``spread_us``: first to last workgroup START (how long until all its workgroups had a CU),

next to the same kernel on the idle GPU.  ``total_us - run_us`` minus its idle value is the launch-to-start
delay a bucket pays; ``run_us`` over its idle value is the slowdown from sharing CUs with the GEMMs.
"""
from __future__ import annotations

from typing import Dict

import torch

from ..parallel.ddp import bucket_plan

_TICK_US = 0.01          # s_memrealtime: 100 MHz


class CommProbe:
    def __init__(self, space, bucket_mb: float = 8.0, first_bucket_mb: float = 1.0, blocks: int = 32):
        self.space = space
        self.blocks = int(blocks)
        self.buckets, self.bucket_of = bucket_plan(space, bucket_mb, first_bucket_mb)
        self.expected = [b[3] - b[2] for b in self.buckets]
        dev = space.grad.device
        self.device = dev
        self.stream = torch.cuda.Stream(device=dev)
        nmax = max(e - s for s, e, _, _ in self.buckets)
        self.src = torch.zeros(nmax, dtype=torch.float32, device=dev)
        self.dst = torch.empty_like(self.src)
        k = len(self.buckets)      # slots 0..k-1: in the backward; k..2k-1: the same buckets on the idle GPU
        self.stamp = torch.zeros(2 * k, 2 * self.blocks, dtype=torch.int64, device=dev)
        self.ev = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(2 * k)]
        self.ev_step = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        space.add_ready_listener(self.mark_ready)
        self.reset()

    def reset(self):
        self.pending = list(self.expected)
        self.next_launch = 0

    def start_step(self):
        self.ev_step[0].record(torch.cuda.current_stream(self.device))

    def mark_ready(self, i: int):
        self.pending[self.bucket_of[i]] -= 1
        while self.next_launch < len(self.buckets) and self.pending[self.next_launch] == 0:
            self._launch(self.next_launch)
            self.next_launch += 1

    def _launch(self, b: int, slot: int = None):
        slot = b if slot is None else slot
        s, e = self.buckets[b][:2]
        n = (e - s) // 4 * 4
        ev_ready, ev0, ev1 = self.ev[slot]
        ev_ready.record(torch.cuda.current_stream(self.device))
        self.stream.wait_event(ev_ready)
        from ..ops import kernels as K
        with torch.cuda.stream(self.stream):
            ev0.record(self.stream)
            K.comm_probe(self.src[:n], self.dst[:n], self.stamp[slot], blocks=self.blocks)
            ev1.record(self.stream)

    def finish_step(self) -> Dict:
        """After the step: each bucket's numbers next to the same bucket's probe on the idle GPU."""
        self.ev_step[1].record(torch.cuda.current_stream(self.device))
        torch.cuda.synchronize(self.device)
        k = len(self.buckets)
        launched = self.next_launch
        for b in range(launched):
            for _ in range(2):              # the second run is the baseline (the first pays launch warm-up)
                self._launch(b, slot=k + b)
                torch.cuda.synchronize(self.device)
        st = self.stamp.cpu()
        step_us = self.ev_step[0].elapsed_time(self.ev_step[1]) * 1e3

        def row(slot):
            _, e0, e1 = self.ev[slot]
            t0, t1 = st[slot, 0::2], st[slot, 1::2]
            return {"total_us": round(e0.elapsed_time(e1) * 1e3, 1),
                    "run_us": round(float(t1.max() - t0.min()) * _TICK_US, 1),
                    "spread_us": round(float(t0.max() - t0.min()) * _TICK_US, 1)}

        rows = []
        for b in range(launched):
            r, idle = row(b), row(k + b)
            r.update(bucket=b, mb=round((self.buckets[b][1] - self.buckets[b][0]) * 4 / 2 ** 20, 3),
                     ready_at_us=round(self.ev_step[0].elapsed_time(self.ev[b][0]) * 1e3, 1),
                     idle=idle,
                     delay_us=round((r["total_us"] - r["run_us"]) - (idle["total_us"] - idle["run_us"]), 1))
            rows.append(r)
        self.reset()
        return {"step_us": round(step_us, 1), "blocks": self.blocks, "buckets": rows,
                "unlaunched": k - launched}
