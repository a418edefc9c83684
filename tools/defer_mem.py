#!/usr/bin/env python3
"""Peak HBM of a pipeline step with the merged (deferred) weight gradients on / off and the deferral
cap (deferred wgrad operands stay alive until the merged launch).  One-GPU rehearsal:
every stage on cuda:0 (GPipeLocal), so the figure is the WHOLE pipeline's peak -- an upper bound
on any one stage of the multi-GPU run.

    python tools/defer_mem.py --model unet --img 512 --stages 2 --microbatches 8 --batch 256
"""
import argparse
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="unet")
    ap.add_argument("--img", type=int, default=512)
    ap.add_argument("--stages", type=int, default=2)
    ap.add_argument("--microbatches", type=int, default=8)
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--cap-gb", type=float, nargs="*", default=[8.0])
    a = ap.parse_args()

    from distributedpytorch_amd.config import TrainConfig
    from distributedpytorch_amd.data.synthetic import synthetic_batch
    from distributedpytorch_amd.models.unet import build_model
    from distributedpytorch_amd.trainer import PipelineLocalStrategy

    dev = torch.device("cuda:0")
    rows = []
    for mode, cap in [("off", None)] + [("on", c) for c in a.cap_gb]:
        torch.manual_seed(0)
        cfg = TrainConfig(train_method="MP", batch_size=a.batch, img_size=(a.img, a.img), dtype="bf16", backend="hip",
                          model=a.model, lr=1e-4, microbatches=a.microbatches, stages=a.stages, mp_cut="balanced")
        strat = PipelineLocalStrategy(cfg, build_model(a.model).to(dev), [dev] * a.stages)
        for b in strat.pipe.stage_blocks:
            if hasattr(b, "defer_wgrad"):
                b.defer_wgrad = a.microbatches if mode == "on" else 0
                if cap is not None:
                    b.defer_cap_bytes = int(cap * 2 ** 30)
        x, m = synthetic_batch(a.batch, a.img, a.img, 3, seed=1, device=dev)
        t = m.float().unsqueeze(1)
        strat.train_step(x, t)
        torch.cuda.synchronize()
        torch.cuda.reset_peak_memory_stats(dev)
        t0 = time.perf_counter()
        for _ in range(a.steps):
            loss = strat.train_step(x, t)
        torch.cuda.synchronize()
        ms = (time.perf_counter() - t0) * 1000 / a.steps
        r = {"model": a.model, "img": a.img, "stages": a.stages, "microbatches": a.microbatches, "batch": a.batch,
             "defer": mode, "cap_gb": cap, "peak_gb": round(torch.cuda.max_memory_allocated(dev) / 2 ** 30, 2),
             "ms_per_step": round(ms, 2), "loss": round(float(loss), 5)}
        print(json.dumps(r), flush=True)
        rows.append(r)
        del strat, x, m, t
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
