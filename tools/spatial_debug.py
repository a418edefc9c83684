#!/usr/bin/env python3
"""Row-split pipeline on the HIP engine vs the single-device HIP step, one GPU (gloo ranks on cuda:0):
loss error and the worst gradient cosine per parameter, for a few engine variants (debug aid for
parallel/spatial_pipe.py; tests/test_hip_multirank.py holds the pass/fail form)."""
import os
import socket
import sys

import torch
import torch.multiprocessing as mp

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def worker(rank, world, port, variant, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), DPA_SAME_DEVICE="1")
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from distributedpytorch_amd.config import TrainConfig
        from distributedpytorch_amd.data.synthetic import synthetic_batch
        from distributedpytorch_amd.models.unet import build_model
        from distributedpytorch_amd.parallel.spatial import SpatialPlan
        from distributedpytorch_amd.parallel.spatial_pipe import SpatialGPipe
        from distributedpytorch_amd.trainer import SingleDevice
        M = variant.get("M", 2)
        B = 2 * M
        torch.manual_seed(0)
        model = build_model("unet")
        ref = build_model("unet")
        ref.load_state_dict(model.state_dict())
        img, mask = synthetic_batch(B, 128, 128, 3, seed=7)
        x, t = img.cuda(), mask.float().unsqueeze(1).cuda()
        sd = SingleDevice(TrainConfig(backend="hip", lr=1e-3), ref, "cuda:0")
        sd.optimizer.zero_grad()
        lref = sd.forward_loss(x, t)
        (lref * B).backward()
        torch.cuda.synchronize()
        gref = {n: p.grad.detach().clone() for n, p in ref.named_parameters()}
        model = model.cuda()
        plan = SpatialPlan(**variant["plan"])
        pipe = SpatialGPipe(model, plan, M, backend=variant.get("backend", "hip"), dtype="bf16", img_hw=(128, 128))
        if "defer" in variant and hasattr(pipe.blocks, "defer_wgrad"):
            pipe.blocks.defer_wgrad = variant["defer"]
        pipe.space.zero_grad()
        loss = pipe.train_step(x, t, B, (128, 128), loss_scale=float(B))
        torch.cuda.synchronize()
        cos = {}
        for n, p in model.named_parameters():
            if p.requires_grad:
                a, b = p.grad.double().reshape(-1), gref[n].double().reshape(-1)
                cos[n] = round((a @ b / (a.norm() * b.norm()).clamp_min(1e-30)).item(), 5)
        q.put((rank, abs(loss.item() - lref.item()) / abs(lref.item()), cos, None))
    except Exception as e:
        import traceback
        q.put((rank, None, {}, repr(e) + traceback.format_exc()[-1500:]))
    finally:
        dist.destroy_process_group()


def run(variant, world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    ps = [ctx.Process(target=worker, args=(r, world, port, variant, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted([q.get(timeout=300) for _ in ps], key=lambda r: r[0])
    for p in ps:
        p.join(timeout=30)
    return res


if __name__ == "__main__":
    V2 = dict(S=2, inner_cuts=(1, 3, 6, 8), inner_owner=(0, 1, 0), L=1)
    C2 = dict(S=2, inner_cuts=(1, 4, 8), inner_owner=(0, 1), L=1)
    variants = [("v M2", dict(plan=V2)), ("v M2 nodefer", dict(plan=V2, defer=1)), ("v M1", dict(plan=V2, M=1)),
                ("contig M2", dict(plan=C2)), ("contig M1", dict(plan=C2, M=1)),
                ("v M2 torch-bf16", dict(plan=V2, backend="torch"))]
    for name, v in variants:
        res = run(v, 2)
        for rank, lrel, cos, err in res:
            if err:
                print(name, rank, "ERROR", err, flush=True)
                continue
            worst = sorted(cos.items(), key=lambda kv: kv[1])[:4]
            print(f"{name:18s} rank {rank} loss_rel {lrel:.2e} worst {worst}", flush=True)
