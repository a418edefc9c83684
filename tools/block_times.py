#!/usr/bin/env python3
"""Per-block forward / backward time table of a UNet on the HIP engine, one GPU, for the pipeline
schedule model (distributedpytorch_amd/parallel/schedule.py).

For every microbatch size, one real forward pass provides each block's inputs; then every block
(enc_l, mid, dec_i, head; the last decoder block is timed together with the head, whose forward and
backward it fuses) is run in isolation on copies of those inputs: forward, backward with random
output gradients, and backward with the side-stream weight-gradient kernels skipped (timing
ablation: the deferrable part of the backward is bwd - bwd_nowgrad).  Medians over --reps runs,
CUDA events around each call.  The optimizer step (fused Adam over the flat buffer) is timed once
and split over the blocks by parameter count.  Every block except the head is also timed as its two
halves (``units``: part a / part b of a DoubleConv cut between its convs, models/blocks.py) -- the
conv-level stage boundaries of parallel/schedule.py.

    python tools/block_times.py --model unet --img 512 --mbs 8 16 32 64 128 256 --out profiles/block_times_unet_512_r04.json
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--model", default="unet")
    ap.add_argument("--img", type=int, default=512)
    ap.add_argument("--mbs", type=int, nargs="+", default=[8, 16, 32, 64, 128, 256])
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--out", default=None)
    ap.add_argument("--blocks", nargs="*", default=None, help="time only these blocks (e.g. dec4), for profiling")
    a = ap.parse_args()

    from distributedpytorch_amd.compute import make_blocks
    from distributedpytorch_amd.data.synthetic import synthetic_batch
    from distributedpytorch_amd.models.blocks import block_kind, n_blocks, skip_name
    from distributedpytorch_amd.models.unet import build_model
    from distributedpytorch_amd.ops import kernels as K
    from distributedpytorch_amd.optim import FlatParameterSpace, FusedAdam

    dev = torch.device("cuda:0")
    torch.manual_seed(0)
    model = build_model(a.model).to(dev)
    space = FlatParameterSpace(model, device=dev)
    opt = FusedAdam(space, lr=1e-4, weight_decay=1e-8)
    B = make_blocks(model, "hip", "bf16", dev)
    depth = model.cfg.depth
    nb = n_blocks(depth)

    def ev():
        return torch.cuda.Event(enable_timing=True)

    def timed(fn, reps):
        ts = []
        for _ in range(reps):
            s, e = ev(), ev()
            s.record()
            fn()
            e.record()
            torch.cuda.synchronize()
            ts.append(s.elapsed_time(e))
        ts.sort()
        return ts[len(ts) // 2]

    # the HIP engine's Functions hang off an anchor leaf and write weight gradients into the flat buffer
    params = [p for p in model.parameters() if p.requires_grad] + ([B.anchor] if hasattr(B, "anchor") else [])
    acc = []        # the leaves whose .grad is accumulated: parameters and the block input

    def leaf(t):
        return t.detach().requires_grad_(True)

    def xleaf(t):
        # the block input's gradient is accumulated (a stage boundary receives it); a skip is not: within a
        # stage the encoder consumes the decoder's strided skip gradient directly, and materialising it
        # into a leaf's .grad (a layout-changing copy of the concat-buffer view) is not engine work
        v = leaf(t)
        acc[:] = params + [v]
        return v

    table = {"model": a.model, "img": [a.img, a.img], "depth": depth, "widths": list(model.cfg.widths),
             "mid_width": model.cfg.mid_width, "blocks": [f"{k}{i}" if k in ("enc", "dec") else k
                                                          for k, i in (block_kind(b, depth) for b in range(nb))],
             "per_mb": {}, "note": "ms per block; the last decoder block includes the fused head (head = 0)"}
    for mb in a.mbs:
        x, m = synthetic_batch(mb, a.img, a.img, 3, seed=mb, device=dev)
        t = m.float().unsqueeze(1).contiguous()
        # one real forward: the inputs of every block (skips stay views of the encoder's concat buffers)
        ins = {}
        env = {"x": B.prep(x)}
        with torch.no_grad():
            for idx in range(nb - 1):
                kind, i = block_kind(idx, depth)
                if kind == "enc":
                    ins[idx] = {"x": env["x"]}
                    s, env["x"] = B.enc(i, env["x"])
                    env[skip_name(i)] = s
                elif kind == "mid":
                    ins[idx] = {"x": env["x"]}
                    env["x"] = B.mid(env["x"])
                else:
                    nm = skip_name(depth - 1 - i)
                    ins[idx] = {"x": env["x"], "skip": env[nm]}
                    env["x"] = B.dec(i, env["x"], env[nm])
        fwd, bwd, bwd_nw = [], [], []
        ufwd, ubwd, ubwd_nw = [], [], []          # per half-block unit: (b, a), (b, b) for b < nb - 1, then head
        for idx in range(nb):
            kind, i = block_kind(idx, depth)
            if kind == "head":
                fwd.append(0.0), bwd.append(0.0), bwd_nw.append(0.0)
                continue
            if a.blocks and table["blocks"][idx] not in a.blocks:
                fwd.append(0.0), bwd.append(0.0), bwd_nw.append(0.0)
                ufwd.extend([0.0, 0.0]), ubwd.extend([0.0, 0.0]), ubwd_nw.extend([0.0, 0.0])
                continue
            inp = ins[idx]
            last = idx == nb - 2

            def run():
                acc[:] = params
                xin = xleaf(inp["x"]) if idx > 0 else inp["x"]
                if kind == "enc":
                    return B.enc(i, xin)
                if kind == "mid":
                    return (B.mid(xin),)
                sk = inp["skip"]
                base = sk._base if sk._base is not None else sk
                B._cats[sk.data_ptr()] = base          # the decoder reuses the encoder's concat buffer
                if last:
                    B.expect_target(t)
                    y = B.dec(i, xin, leaf(sk))
                    return (B.head_partials(y, t),)
                return (B.dec(i, xin, leaf(sk)),)

            fwd.append(timed(lambda: run(), a.reps))

            def back():
                o = run()
                s_, e_ = ev(), ev()
                s_.record()
                torch.autograd.backward(o, [torch.ones_like(v) if v.dim() == 1 else
                                            torch.randn_like(v) * 1e-3 for v in o], inputs=acc)
                e_.record()
                return s_, e_

            def tback(reps):
                ts = []
                for _ in range(reps):
                    s_, e_ = back()
                    torch.cuda.synchronize()
                    ts.append(s_.elapsed_time(e_))
                ts.sort()
                return ts[len(ts) // 2]

            bwd.append(tback(a.reps))
            K.set_timing_ablation({"wgrad"})      # timing ablation: skip the deferrable weight gradients
            try:
                bwd_nw.append(tback(a.reps))
            finally:
                K.set_timing_ablation(())
            print(f"mb {mb:4d} {table['blocks'][idx]:6s} fwd {fwd[-1]:8.3f} bwd {bwd[-1]:8.3f} "
                  f"bwd-wgrad {bwd_nw[-1]:8.3f} ms", flush=True)
            # the block's two halves (a pipeline cut between its convs, models/blocks.py): part a from the
            # block input, part b from part a's output
            with torch.no_grad():
                if kind == "enc":
                    a_out = B.enc_a(i, inp["x"])
                elif kind == "mid":
                    a_out = B.mid_a(inp["x"])
                else:
                    sk = inp["skip"]
                    B._cats[sk.data_ptr()] = sk._base if sk._base is not None else sk
                    a_out = B.dec_a(i, inp["x"], sk)
            for part in ("a", "b"):
                def run_part():
                    acc[:] = params
                    if part == "b":
                        xin = xleaf(a_out)
                        if kind == "enc":
                            return B.enc_b(i, xin)
                        return ((B.mid_b if kind == "mid" else (lambda v: B.dec_b(i, v)))(xin),)
                    xin = xleaf(inp["x"]) if idx > 0 else inp["x"]
                    if kind == "enc":
                        return (B.enc_a(i, xin),)
                    if kind == "mid":
                        return (B.mid_a(xin),)
                    sk = inp["skip"]
                    B._cats[sk.data_ptr()] = sk._base if sk._base is not None else sk
                    return (B.dec_a(i, xin, leaf(sk)),)

                def back_part(reps):
                    ts = []
                    for _ in range(reps):
                        o = run_part()
                        s_, e_ = ev(), ev()
                        s_.record()
                        torch.autograd.backward(o, [torch.randn_like(v) * 1e-3 for v in o], inputs=acc)
                        e_.record()
                        torch.cuda.synchronize()
                        ts.append(s_.elapsed_time(e_))
                    ts.sort()
                    return ts[len(ts) // 2]

                ufwd.append(timed(lambda: run_part(), a.reps))
                ubwd.append(back_part(a.reps))
                K.set_timing_ablation({"wgrad"})
                try:
                    ubwd_nw.append(back_part(a.reps))
                finally:
                    K.set_timing_ablation(())
                print(f"mb {mb:4d} {table['blocks'][idx]:6s}.{part} fwd {ufwd[-1]:8.3f} bwd {ubwd[-1]:8.3f} "
                      f"bwd-wgrad {ubwd_nw[-1]:8.3f} ms", flush=True)
            del a_out
        ufwd.append(0.0), ubwd.append(0.0), ubwd_nw.append(0.0)     # the head unit (fused into the last block)
        table["per_mb"][str(mb)] = {"fwd": fwd, "bwd": bwd, "bwd_nowgrad": bwd_nw,
                                    "units": {"fwd": ufwd, "bwd": ubwd, "bwd_nowgrad": ubwd_nw}}
        del ins, env, x, m, t
        torch.cuda.empty_cache()
    # optimizer step, split over the blocks by parameter count
    space.grad.normal_()
    t_opt = timed(lambda: opt.step(), a.reps)
    counts = [0] * nb
    from distributedpytorch_amd.parallel.pipeline import stage_param_names
    for b in range(nb):
        names = set(stage_param_names(model, b, b + 1))
        counts[b] = sum(p.numel() for n, p in model.named_parameters() if n in names)
    tot = sum(counts)
    table["opt_ms"] = [t_opt * c / tot for c in counts]
    print(f"optimizer step {t_opt:.3f} ms", flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(table, f, indent=1)


if __name__ == "__main__":
    main()
