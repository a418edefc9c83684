#!/usr/bin/env python3
"""Headline benchmark: UNet 512x512 bf16 training throughput (images/s, whole job).

Metric/config from BASELINE.json: "images/sec (whole node) UNet 512x512 bf16 at 1/2/4/8 MI355X".
Model: the reference 4-level UNet (base 32, 7,760,097 params, random init), full training step
(forward, BCE - log Dice loss, backward, RCCL gradient all-reduce for N>1, fused Adam step) through
the framework's own strategy classes.  Data: synthetic images/masks generated on the GPU (a pool
of distinct batches cycled every step; the reference's CPU JPEG decode is not part of the step).

    python bench.py                                  # N=1, defaults finish in ~1-2 min
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 --master-port P \
        bench.py --gpus N --steps K --warmup W      # one rank per GPU over RCCL (DDP)

Timing: W untimed warm-up steps; then barrier + device sync, K timed steps, barrier + device sync;
elapsed = MAX over ranks.  value = N * per_gpu_batch * K / elapsed (weak scaling).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

BASELINE_METRIC = "images/sec (whole node) UNet 512x512 bf16 at 1/2/4/8 MI355X; Dice parity"
# measured stock PyTorch-ROCm (MIOpen convs, bf16 autocast, channels_last) img/s per GPU on MI355X for
# this model at 512x512 and the LARGEST per-GPU batch it could be measured at: batch 32 (909.6 img/s,
# profiles/stock_torch_b32_r02.log; batch 8: 758).  At the bench's batch 256 its first iteration
# (MIOpen kernel compilation + find) did not finish within 1080 s (profiles/stock_torch_b256_attempt_r02.log),
# so vs_baseline compares against the batch-32 rate; the reference publishes no number.
STOCK_BASELINE_PER_GPU = 909.62
STOCK_BASELINE_BATCH = 32


def _hw(s: str):
    p = [int(v) for v in str(s).lower().split("x")]
    return (p[0], p[0]) if len(p) == 1 else (p[0], p[1])


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=256,
                    help="images per GPU per step (HBM: ~58 GB of 288 at 256; 128 -> ~29 GB, ~1%% lower img/s)")
    ap.add_argument("--img", type=_hw, default=(512, 512),
                    help="image size: S (square) or HxW, e.g. 640x960 (the reference's default, utils/train_utils.py:26)")
    ap.add_argument("--backend", choices=["hip", "torch", "auto"], default="auto")
    ap.add_argument("--dtype", choices=["bf16", "fp32"], default="bf16",
                    help="compute / storage precision (fp32: the reference's precision, on the fp32 HIP engine)")
    ap.add_argument("--model", default="unet")
    ap.add_argument("--bucket-mb", type=float, default=8.0)
    ap.add_argument("--grad-comm-dtype", choices=["fp32", "bf16"], default="fp32",
                    help="N>1: gradient all-reduce wire dtype")
    ap.add_argument("--no-comm-overlap", dest="comm_overlap", action="store_false",
                    help="N>1 DDP: all-reduce the gradients after the backward (one collective) instead of "
                         "bucket by bucket during it")
    ap.add_argument("--pool", type=int, default=2, help="distinct synthetic batches cycled")
    ap.add_argument("--out", default=None, help="also append the JSON line to this file")
    ap.add_argument("--graph", action="store_true",
                    help="N=1: replay the step from a captured HIP graph; dp1proc: each replica's forward and "
                         "backward from HIP graphs (trainer.GraphedDP)")
    ap.add_argument("--parallelism", choices=["dp", "mp", "dp1proc"], default="dp",
                    help="dp: one replica per GPU, RCCL all-reduce (weak scaling); mp: GPipe over the N ranks "
                         "(one batch of --batch images split into --microbatches, strong scaling); with one "
                         "process, mp runs --stages stages on cuda:0 (pipeline rehearsal); dp1proc: -t DP, one "
                         "process driving --replicas replicas (one host thread each, native RCCL clique, "
                         "--batch images per replica; replicas beyond the visible GPUs share them: a host-"
                         "issue rehearsal)")
    ap.add_argument("--replicas", type=int, default=0,
                    help="dp1proc: replicas (0: one per visible GPU)")
    ap.add_argument("--reserve-cus", type=int, default=0,
                    help="run the step's compute (and the engine's side streams) on CU-masked streams that leave this "
                         "many CUs free for communication kernels (RCCL buckets; measured with --comm-probe)")
    ap.add_argument("--comm-probe", action="store_true",
                    help="N=1 dp: after the timed steps, run steps that launch an RCCL-bucket stand-in at each "
                         "DDP bucket-ready point and report how long it waited for CUs (utils/comm_probe.py)")
    ap.add_argument("--microbatches", type=int, default=0,
                    help="mp microbatches (0: the pipeline plan's count for this model / image / stages / batch, "
                         "parallel/plans.json; without one 2 for the reference cut, 8 otherwise)")
    ap.add_argument("--stages", type=int, default=2, help="mp with one process: stages on the local device")
    ap.add_argument("--mp-replicas", type=int, default=1,
                    help="mp over N ranks: R pipelines of N/R stages, data-parallel across them (each pipeline "
                         "trains its own --batch images)")
    ap.add_argument("--mp-cut", choices=["auto", "reference", "balanced", "v", "time", "spatial"], default="auto",
                    help="mp stage placement (auto: the link-aware plan from measured block times when "
                         "parallel/plans.json has one for this configuration, else the skip-local mirrored "
                         "V placement; reference: the reference's encoder|decoder cut)")
    ap.add_argument("--timing-ablation", default="",
                    help="MEASUREMENT ONLY, numerically wrong: skip these kernel families (comma list of "
                         "stream,halo,glds,wgrad,wgrad_deep,bwd,deconv) to see what they cost; the JSON line is "
                         "marked invalid")
    ap.add_argument("--infer", action="store_true",
                    help="inference throughput instead of training: eval-mode forward to the probability map "
                         "(BatchNorm folded into the convs), no loss/backward/optimizer")
    return ap.parse_args()


def _heartbeat(period: float = 60.0):
    """Print a line every ``period`` s (first-iteration kernel compilation in stock MIOpen can take
    minutes; a silent process looks hung to job supervisors)."""
    import threading

    t0 = time.time()
    stop = threading.Event()

    def run():
        while not stop.wait(period):
            print(f"[bench] alive {time.time() - t0:.0f}s", file=sys.stderr, flush=True)

    threading.Thread(target=run, daemon=True).start()
    return stop


def main():
    a = parse()
    hb = _heartbeat()
    import torch
    import torch.distributed as dist

    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != a.gpus and rank == 0:
        print(f"[bench] note: WORLD_SIZE={world} but --gpus={a.gpus}", file=sys.stderr)
    # DPA_SAME_DEVICE=1 + DPA_DIST_BACKEND=gloo rehearse the multi-rank path on a one-GPU box
    if os.environ.get("DPA_SAME_DEVICE", "0") == "1":
        local = 0
    torch.cuda.set_device(local)
    device = torch.device(f"cuda:{local}")
    if world > 1:
        backend = os.environ.get("DPA_DIST_BACKEND", "nccl")
        # a collective that never completes (a rank lost, a link down) errors out after 10 minutes
        # instead of hanging the job; no step of this bench legitimately waits that long
        import datetime
        tmo = datetime.timedelta(seconds=600)
        if backend == "nccl":
            dist.init_process_group("nccl", init_method="env://", device_id=device, timeout=tmo)
        else:
            dist.init_process_group(backend, init_method="env://", timeout=tmo)

    from distributedpytorch_amd.config import TrainConfig
    from distributedpytorch_amd.data.synthetic import synthetic_batch
    from distributedpytorch_amd.models.summary import layer_table
    from distributedpytorch_amd.models.unet import PRESETS, build_model, count_params
    from distributedpytorch_amd.trainer import (DDPStrategy, DPStrategy, PipelineDistStrategy, PipelineLocalStrategy,
                                                SingleDevice)
    from distributedpytorch_amd.compute import resolve_backend
    from distributedpytorch_amd.utils import set_seed

    set_seed(1234)
    from distributedpytorch_amd.ops import kernels as K
    ablate = [v for v in a.timing_ablation.split(",") if v]
    if ablate:
        K.set_timing_ablation(ablate)
        print(f"[bench] TIMING ABLATION {ablate}: results are numerically wrong", file=sys.stderr, flush=True)
    mp = a.parallelism == "mp"
    dp1 = a.parallelism == "dp1proc"
    assert not (dp1 and world > 1), "dp1proc is one process"
    method = "MP" if mp else ("DP" if dp1 else ("DDP" if world > 1 else "singleGPU"))
    cfg = TrainConfig(train_method=method, batch_size=a.batch, img_size=a.img, dtype=a.dtype,
                      backend=a.backend, model=a.model, bucket_mb=a.bucket_mb, lr=1e-4,
                      grad_comm_dtype=a.grad_comm_dtype, comm_overlap=a.comm_overlap,
                      microbatches=a.microbatches, stages=a.stages, mp_cut=a.mp_cut, mp_replicas=a.mp_replicas)
    mp_info = None
    if mp:
        from distributedpytorch_amd.config import mp_plan
        mpp = mp_plan(cfg, world // max(1, a.mp_replicas) if world > 1 else a.stages)
        mp_info = {"cut_mode": mpp.mode, "placement": str(mpp.placement), "microbatches": mpp.microbatches,
                   "policy": mpp.policy, **mpp.info}
    model = build_model(a.model)
    nparams = count_params(model)
    n_rep = 1
    if dp1:
        ngpu = torch.cuda.device_count()
        n_rep = a.replicas or ngpu
        devs = [torch.device(f"cuda:{i % ngpu}") for i in range(n_rep)]
        strat = DPStrategy(cfg, model.to(devs[0]), devs)
        same_dev = len({d.index for d in devs}) < n_rep
    elif mp and world > 1:
        strat = PipelineDistStrategy(cfg, model, device)
    elif mp:
        strat = PipelineLocalStrategy(cfg, model.to(device), [device] * a.stages)
    else:
        strat = DDPStrategy(cfg, model, device) if world > 1 else SingleDevice(cfg, model, device)
    backend = resolve_backend(a.backend, device, a.dtype, model)

    pool = []
    for i in range(a.pool):
        # dp1proc: the global batch on cuda:0, scattered to the replicas inside the step (reference -t DP)
        # mp: the ranks of one pipeline share a batch (a row-split plan reads every rank's rows of it)
        data_rank = rank // max(1, world // max(1, a.mp_replicas)) if (mp and world > 1) else rank
        img, mask = synthetic_batch(a.batch * n_rep, a.img[0], a.img[1], 3, seed=1000 * data_rank + i, device=device)
        pool.append((img, mask.float().unsqueeze(1)))

    masked = None
    if a.reserve_cus:
        masked = K.cu_masked_stream(device, a.reserve_cus)
        masked.wait_stream(torch.cuda.current_stream(device))
        eng = getattr(getattr(strat, "compute", None), "blocks", None)
        if eng is not None and getattr(eng, "side", None) is not None:
            eng.side = K.cu_masked_stream(device, a.reserve_cus)
            if hasattr(eng, "side2"):
                eng.side2 = K.cu_masked_stream(device, a.reserve_cus)
        torch.cuda.set_stream(masked)
        print(f"[bench] compute on CU-masked streams: {masked.cus} CUs, {a.reserve_cus} reserved", file=sys.stderr)

    graphed = None
    if a.graph and dp1:
        from distributedpytorch_amd.trainer import GraphedDP
        graphed = GraphedDP(strat, *pool[0])
    elif a.graph and world == 1 and not mp:
        from distributedpytorch_amd.trainer import GraphedStep
        graphed = GraphedStep(strat, *pool[0])

    if a.infer:
        assert not mp and world == 1, "--infer: single device"
        strat.model.eval()

    def step(i):
        x, t = pool[i % len(pool)]
        if a.infer:
            with torch.no_grad():
                return strat.compute.probs(x).mean()
        return graphed(x, t) if graphed is not None else strat.train_step(x, t)

    t_w0 = time.perf_counter()
    loss = None
    for i in range(a.warmup):
        loss = step(i)
        if rank == 0:
            torch.cuda.synchronize()
            print(f"[bench] warmup step {i + 1}/{a.warmup} done at {time.perf_counter() - t_w0:.1f}s", file=sys.stderr,
                  flush=True)
    torch.cuda.synchronize()
    warm_s = time.perf_counter() - t_w0
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(a.steps + 1)] if (world > 1 or dp1) else None
    if evs:
        evs[0].record()
    host_s = 0.0          # host time inside the step calls: the launch/issue cost (asynchronous kernels)
    for i in range(a.steps):
        h0 = time.perf_counter()
        loss = step(a.warmup + i)
        host_s += time.perf_counter() - h0
        if evs:
            evs[i + 1].record()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    el = torch.tensor([elapsed], dtype=torch.float64, device=device)
    if world > 1:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    elapsed = float(el.item())
    rank_ms = None
    if world > 1:   # per-rank mean device ms/step of the timed steps -> min / max over ranks
        mine = sum(evs[i].elapsed_time(evs[i + 1]) for i in range(a.steps)) / a.steps
        allr = [torch.zeros(1, dtype=torch.float64, device=device) for _ in range(world)]
        dist.all_gather(allr, torch.tensor([mine], dtype=torch.float64, device=device))
        rank_ms = [round(float(v.item()), 3) for v in allr]
    if mp and world > 1:  # the loss lives on the head pipeline stage; rank 0 prints it
        lt = (loss.detach().float().reshape(1) if loss is not None
              else torch.zeros(1, device=device))
        dist.broadcast(lt, src=strat.pipe.head_rank)
        loss = lt
    final_loss = float(loss.item()) if loss is not None else float("nan")

    # dp: every rank trains its own --batch images (weak scaling); mp: the ranks of a pipeline share one
    # batch, each of the --mp-replicas pipelines trains its own
    R = max(1, a.mp_replicas) if mp and world > 1 else 1
    S = world // R if mp and world > 1 else (a.stages if mp else 1)
    imgs = a.batch * (R if mp else world * n_rep) * a.steps
    value = imgs / elapsed
    ms = 1000.0 * elapsed / a.steps
    # vs_baseline: like for like only, i.e. null unless stock PyTorch-ROCm was measured at THIS per-GPU
    # batch (it was at batch 32: 909.6 img/s; at the bench's batch 256 its MIOpen find does not finish in
    # 1080 s, so there is no like-for-like number).  The batch-32 equal-batch ratio and this run's
    # quotient over stock-at-32 stay in vs_baseline_basis as context.
    vs = cross = None
    per_gpu_batch = a.batch if not mp else a.batch // max(1, S)
    # like for like only: one real GPU, the stock run's config (a multi-rank or replica run would compare
    # against N x the single-GPU stock rate, and stock DDP / DP were never measured)
    same_device_ranks = os.environ.get("DPA_SAME_DEVICE", "0") == "1"
    if STOCK_BASELINE_PER_GPU and not a.infer and a.dtype == "bf16" and world == 1 and not dp1 and not mp:
        cross = round(value / STOCK_BASELINE_PER_GPU, 4)
        if (per_gpu_batch == STOCK_BASELINE_BATCH and a.img == (512, 512) and a.model == "unet"
                and not same_device_ranks and a.backend != "torch"):
            vs = cross
    if mp:
        par = f"mp{S}x{strat.pipe.M}mb" + ("" if world > 1 else "-1gpu") + (f"-dp{R}" if R > 1 else "")
    elif dp1:
        par = f"dp1proc{n_rep}" + ("-shared-gpu" if same_dev else "")
    else:
        par = f"dp{world}"
    out = {
        "metric": BASELINE_METRIC if not a.infer else "images/sec inference UNet 512x512 bf16 (eval forward)", "value": round(value, 2), "unit": "images/s", "n_gpus": world,
        "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(ms, 3), "higher_is_better": True,
        "scaling": "strong" if (mp and R == 1) else "weak", "vs_baseline": vs,
        # context only: stock PyTorch-ROCm (MIOpen, bf16 autocast) was measured at batch 32; the
        # equal-batch ratio there and this run over stock-at-32 (cross_batch_ratio, different batches
        # unless --batch 32)
        "vs_baseline_basis": {"kind": ("stock_measured_at_this_batch" if vs is not None else
                                       "null: stock PyTorch-ROCm measured only on one GPU at batch 32 (its MIOpen "
                                       "find did not finish in 1080 s at b256)"),
                              "stock_per_gpu_img_s": STOCK_BASELINE_PER_GPU, "stock_per_gpu_batch": STOCK_BASELINE_BATCH,
                              "this_per_gpu_batch": per_gpu_batch,
                              "cross_batch_ratio": cross},
        "dtype": a.dtype,
        "data": "synthetic (GPU-generated images + ellipse masks), random-init weights",
        "config": {"model": f"{a.model} (reference 4-level UNet, base 32, {nparams} params)" if a.model == "unet"
                   else a.model, "global_batch": a.batch * (R if mp else world * n_rep),
                   "per_gpu_batch": per_gpu_batch,
                   "seq_len": a.img[0] * a.img[1], "image_hw": list(a.img),
                   "parallelism": par, "backend": backend,
                   "mp_cut": (str(getattr(strat.pipe, "pl", None) or strat.pipe.plan) if mp else None),
                   "mp_plan": mp_info, "bucket_mb": a.bucket_mb,
                   "grad_comm_dtype": a.grad_comm_dtype, "comm_overlap": a.comm_overlap,
                   "hip_graph": graphed is not None, "reserve_cus": a.reserve_cus},
        "final_loss": round(final_loss, 5) if final_loss == final_loss else None, "warmup_s": round(warm_s, 2),
        "host_ms_per_step": round(1000.0 * host_s / a.steps, 3),
        "peak_mem_gb": round(torch.cuda.max_memory_allocated(device) / 2 ** 30, 2),
        # the run's non-default kernel switches (ops/config.py; empty = the shipped dispatch)
        "kernel_config": {k: v for k, v in K.CFG.non_default().items()},
    }
    if ablate:
        out["INVALID_timing_ablation"] = ablate
    if dp1:
        # host issue (one thread per replica + the autograd walk) vs device time per step: above 1 the step
        # is host-bound and more replicas per process would not scale
        dev_ms = sum(evs[i].elapsed_time(evs[i + 1]) for i in range(a.steps)) / a.steps
        out["dp1proc"] = {"replicas": n_rep, "devices": sorted({d.index for d in devs}),
                          "native_clique": strat.dp.comm is not None, "device_ms_per_step_dev0": round(dev_ms, 3),
                          "host_ms_per_step": out["host_ms_per_step"],
                          "host_over_device": round(out["host_ms_per_step"] / max(dev_ms, 1e-9), 3)}
    if a.comm_probe:
        assert world == 1 and not mp and not dp1 and hasattr(strat, "space")
        from distributedpytorch_amd.utils.comm_probe import CommProbe
        probe = CommProbe(strat.space, bucket_mb=a.bucket_mb)
        res = None
        for i in range(3):      # outside the timed region: each probed step synchronises
            probe.start_step()
            step(i)
            res = probe.finish_step()
        out["comm_probe"] = res
    if not a.infer and a.model in PRESETS:
        # achieved model FLOP rate: forward FLOPs (analytic layer table) x 3 for forward + dgrad + wgrad
        fwd_gflop = sum(r[3] for r in layer_table(PRESETS[a.model], a.img[0], a.img[1]))
        out["model_gflop_per_image"] = round(3 * fwd_gflop, 2)
        out["achieved_tflops"] = round(value * 3 * fwd_gflop / 1e3, 1)
    if world > 1:
        be = dist.get_backend()
        out["rccl_world"] = {"backend": be, "world_size": world, "rccl": be == "nccl",
                             "rccl_version": (".".join(map(str, torch.cuda.nccl.version())) if be == "nccl" else None)}
        out["rank_ms_per_step"] = {"min": min(rank_ms), "max": max(rank_ms), "per_rank": rank_ms}
    red = getattr(strat, "reducer", None)
    if red is not None and world > 1:  # all-reduce time not hidden behind backward, last step, every rank
        c = red.exposed_comm_ms()
        mine = torch.tensor([c if c is not None else -1.0], dtype=torch.float64, device=device)
        allc = [torch.zeros_like(mine) for _ in range(world)]
        dist.all_gather(allc, mine)
        vals = [float(v.item()) for v in allc]
        out["exposed_comm_ms"] = ({"min": round(min(vals), 3), "max": round(max(vals), 3)}
                                  if min(vals) >= 0 else None)
        out["exposed_comm_ms_last_step"] = round(c, 3) if c is not None else None
    if rank == 0:
        line = json.dumps(out)
        print(line, flush=True)
        if a.out:
            with open(a.out, "a") as f:
                f.write(line + "\n")
    hb.set()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
