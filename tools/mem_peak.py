#!/usr/bin/env python3
"""Where a training step's peak HBM goes: records one step's allocator trace
(torch.cuda.memory._record_memory_history), replays it, and prints the tensors live at the peak
grouped by the first engine frame (file:line function) that allocated them.

    python tools/mem_peak.py --model unet-bn --batch 256 > gpurun_out/mem_peak.txt
"""
import argparse
import os
import sys
from collections import defaultdict

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def site(frames, prefer=("distributedpytorch_amd",)):
    """The first frame inside the engine (innermost first), else the innermost frame."""
    for f in frames:
        fn = f.get("filename", "")
        if any(p in fn for p in prefer) and "ops/kernels.py" not in fn:
            return f"{os.path.basename(fn)}:{f.get('line')} {f.get('name')}"
    if frames:
        f = frames[0]
        return f"{os.path.basename(f.get('filename', '?'))}:{f.get('line')} {f.get('name')}"
    return "?"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="unet-bn")
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--img", type=int, default=512)
    ap.add_argument("--top", type=int, default=30)
    a = ap.parse_args()

    from distributedpytorch_amd.config import TrainConfig
    from distributedpytorch_amd.data.synthetic import synthetic_batch
    from distributedpytorch_amd.models.unet import build_model
    from distributedpytorch_amd.trainer import SingleDevice

    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    cfg = TrainConfig(train_method="singleGPU", batch_size=a.batch, img_size=(a.img, a.img), dtype="bf16",
                      backend="hip", model=a.model, lr=1e-4)
    strat = SingleDevice(cfg, build_model(a.model), dev)
    x, m = synthetic_batch(a.batch, a.img, a.img, 3, seed=1, device=dev)
    t = m.float().unsqueeze(1)
    for _ in range(2):
        strat.train_step(x, t)
    torch.cuda.synchronize()
    torch.cuda.reset_peak_memory_stats(dev)
    base = torch.cuda.memory_allocated(dev)
    torch.cuda.memory._record_memory_history(enabled="all", stacks="python", max_entries=200000)
    strat.train_step(x, t)
    torch.cuda.synchronize()
    snap = torch.cuda.memory._snapshot()
    torch.cuda.memory._record_memory_history(enabled=None)
    peak_alloc = torch.cuda.max_memory_allocated(dev)

    trace = snap["device_traces"][dev.index]
    live, cur, best, best_i, best_live = {}, 0, -1, -1, None
    for i, ev in enumerate(trace):
        act = ev["action"]
        if act == "alloc":
            live[ev["addr"]] = (ev["size"], ev.get("frames", []))
            cur += ev["size"]
            if cur > best:
                best, best_i, best_live = cur, i, dict(live)
        elif act in ("free_requested",):
            e = live.pop(ev["addr"], None)
            if e is not None:
                cur -= e[0]
    gb = 2 ** 30
    print(f"model {a.model} batch {a.batch} {a.img}^2: allocated before the step {base / gb:.2f} GB, "
          f"max_memory_allocated {peak_alloc / gb:.2f} GB, traced peak {base / gb:.2f} + {best / gb:.2f} GB "
          f"at event {best_i} of {len(trace)}")
    if best_i >= 0:
        print(f"peak reached allocating at: {site(trace[best_i].get('frames', []))}")
        groups = defaultdict(lambda: [0, 0])
        for size, frames in best_live.values():
            g = groups[site(frames)]
            g[0] += size
            g[1] += 1
        print(f"{'GB':>7s} {'n':>4s}  allocation site (tensors live at the peak, allocated during the step)")
        for k, (s, n) in sorted(groups.items(), key=lambda kv: -kv[1][0])[:a.top]:
            print(f"{s / gb:7.2f} {n:4d}  {k}")


if __name__ == "__main__":
    main()
