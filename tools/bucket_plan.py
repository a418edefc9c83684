#!/usr/bin/env python3
"""DDP / DP gradient bucket plan for the UNet: which parameters each bucket holds, when its
gradients become final in the backward, and how much all-reduce time is left exposed after the
backward ends, for candidate bucket sizes.

Inputs
* the flat gradient layout (``FlatParameterSpace``: backward order, head first, encoder level 1 last)
  and ``parallel.ddp.bucket_plan`` -- exactly what the trainer uses;
* the per-block backward time on the compute stream, measured: the defaults below are read off the
  rocprofv3 kernel timeline of one training step at batch 256 per GPU, 512x512
  (``profiles/hip_b256_512_timeline_r02.txt``; block boundaries = the head / decoder level /
  bottleneck / encoder level kernels in launch order).  ``--block-ms`` takes another JSON map;
* an all-reduce cost model  t(B) = alpha + 2 (N-1)/N * B / busbw  with a per-collective latency
  alpha and a bus bandwidth for the whole-node ring/tree RCCL picks on the 8-GPU xGMI mesh (7 links
  x ~153 GB/s per GPU).  Both are ASSUMPTIONS (``--alpha-us``, ``--busbw``); the bench JSON's
  ``exposed_comm_ms_last_step`` measures the real exposed time of a run.

Simulation: one collective stream; bucket b starts at max(ready_b, end_{b-1}); exposed = end of the
last bucket - end of the backward.  Only the LAST bucket can be exposed in practice: the decoder's
full-resolution layers (>40 ms of backward) hide everything before it, and what matters is that
the last bucket -- the encoder parameters whose gradients finish last -- is small.

    python tools/bucket_plan.py [--world 8] [--busbw 150] [--alpha-us 30]
"""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

# compute-stream backward time per block at batch 256 / 512^2 (ms), in backward order
BLOCK_MS = {"head": 1.75, "dec4": 10.64, "dec3": 9.77, "dec2": 9.53, "dec1": 8.19, "mid": 3.97,
            "enc4": 4.09, "enc3": 4.68, "enc2": 4.73, "enc1": 5.99}


def block_of(name: str) -> str:
    p = name.split(".")
    if p[0] == "segmap":
        return "head"
    if p[0] == "mid":
        return "mid"
    lvl = int("".join(ch for ch in p[1] if ch.isdigit()))
    return ("dec" if p[0] == "decoder" else "enc") + str(lvl)


def simulate(space, bucket_mb, block_ms, world, alpha_us, busbw):
    from distributedpytorch_amd.parallel.ddp import bucket_plan
    order = list(block_ms)
    t_end, acc = {}, 0.0
    for b in order:
        acc += block_ms[b]
        t_end[b] = acc
    bwd_end = acc
    buckets, _ = bucket_plan(space, bucket_mb, 1.0)
    rows, prev = [], 0.0
    for s, e, f, l in buckets:
        blocks = {block_of(n) for n in space.names[f:l]}
        ready = max(t_end[b] for b in blocks)
        nbytes = (e - s) * 4
        t = alpha_us / 1e3 + 2 * (world - 1) / world * nbytes / (busbw * 1e9) * 1e3
        start = max(ready, prev)
        prev = start + t
        rows.append((nbytes / 2 ** 20, sorted(blocks, key=order.index), ready, start, prev))
    return rows, bwd_end, max(0.0, prev - bwd_end)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--busbw", type=float, default=150.0, help="RCCL all-reduce bus bandwidth, GB/s (assumed)")
    ap.add_argument("--alpha-us", type=float, default=30.0, help="per-collective latency, us (assumed)")
    ap.add_argument("--block-ms", type=str, default=None, help="JSON {block: backward ms} in backward order")
    ap.add_argument("--sizes", type=float, nargs="+", default=[1, 2, 4, 8, 16, 25])
    a = ap.parse_args()
    from distributedpytorch_amd.models.unet import build_model
    from distributedpytorch_amd.optim import FlatParameterSpace
    block_ms = json.loads(a.block_ms) if a.block_ms else BLOCK_MS
    space = FlatParameterSpace(build_model("unet"))
    print(f"UNet grads {space.numel * 4 / 2 ** 20:.2f} MiB fp32; world {a.world}; model t = {a.alpha_us:.0f} us + "
          f"2(N-1)/N B / {a.busbw:.0f} GB/s; backward {sum(block_ms.values()):.1f} ms")
    best = None
    for mb in a.sizes:
        rows, bwd_end, exposed = simulate(space, mb, block_ms, a.world, a.alpha_us, a.busbw)
        print(f"\nbucket_mb {mb:g}: {len(rows)} buckets, exposed all-reduce {exposed * 1e3:.0f} us")
        for sz, blocks, ready, start, end in rows:
            print(f"  {sz:6.2f} MiB  {','.join(blocks):28s} ready {ready:6.2f} ms  comm {start:6.2f}-{end:6.2f} ms")
        key = (round(exposed, 4), len(rows))
        if best is None or key < best[0]:
            best = (key, mb)
    print(f"\nlowest exposed time (fewest collectives on ties): bucket_mb {best[1]:g}")


if __name__ == "__main__":
    main()
