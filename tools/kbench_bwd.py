#!/usr/bin/env python3
"""Fused conv backward (csrc/bwd_stream.hip) vs the kernels it replaces, at the UNet's layer shapes.

For each full-resolution conv (512^2 / 256^2, 32/64 channels) times, at the given batch:
  fused : one bwd_stream pass (dx + dW + db) + the slab reduction
  split : dgrad (igemm stream/halo) on the compute stream || weight gradient (wgrad_stream +
          reduce) on a side stream -- the production schedule before the fused kernel
  serial: the same two launches back to back on one stream
Usage: python tools/kbench_bwd.py [--batch 256] [--iters 10]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from distributedpytorch_amd.ops import kernels as K  # noqa: E402

SHAPES = [  # (name, H=W, Cin, Cout, epilogue)
    ("dec4.c2 / enc1.c2 32->32 @512", 512, 32, 32, "mask"),
    ("dec4.c1 64(cat)->32 @512", 512, 64, 32, "split"),
    ("enc2.c1 32->64 @256", 256, 32, 64, "plain"),
    ("enc2.c2 / dec3.c2 64->64 @256", 256, 64, 64, "mask"),
]


def pack_dgrad(w):
    flat = w.reshape(-1).float().cuda().contiguous()
    Cout, Cin = w.shape[:2]
    kd = K.round_up(9 * Cout, 32)
    d = K.PackDesc(flat.data_ptr(), 0, 1, Cout, Cin, Cout, Cin, kd)
    descs = torch.frombuffer(bytearray(bytes(d)), dtype=torch.uint8).cuda()
    packed = torch.empty(Cin * kd, dtype=torch.bfloat16, device="cuda")
    K.pack_weights(packed, descs, 1, Cin * kd)
    return packed, kd


def timeit(fn, iters):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / iters


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--only-fused", action="store_true", help="time the fused kernel only (counter runs)")
    a = ap.parse_args()
    side = torch.cuda.Stream()
    print(f"batch {a.batch}: ms per call (GB/s of the fused pass's compulsory bytes)")
    for name, hw, ci, co, epi in SHAPES:
        N = a.batch
        g = (torch.randn(N, hw, hw, co, device="cuda") * 0.1).to(torch.bfloat16)
        x = torch.relu(torch.randn(N, hw, hw, ci, device="cuda")).to(torch.bfloat16)
        w = torch.randn(co, ci, 3, 3) * 0.05
        wd, kd = pack_dgrad(w)
        gw = torch.zeros(co * ci * 9, device="cuda")
        gb = torch.zeros(co, device="cuda")
        dx = torch.empty(N, hw, hw, ci, dtype=torch.bfloat16, device="cuda")
        lo = torch.empty(N, hw, hw, ci // 2, dtype=torch.bfloat16, device="cuda")
        hi = torch.empty(N, hw, hw, ci - ci // 2, dtype=torch.bfloat16, device="cuda")

        def fused():
            if epi == "split":
                K.conv_bwd_fused(g, x, wd, kd, gw, gb, mask=False, dx=lo, dx2=hi, split=ci // 2)
            else:
                K.conv_bwd_fused(g, x, wd, kd, gw, gb, mask=epi == "mask", dx=dx)

        def dgrad():
            kw = dict(Ngemm=ci, Kpad=kd, KH=3, KW=3, stride=1, pad=1, Cs=co, out_grid=(N, hw, hw))
            if epi == "split":
                K.igemm(g, wd, lo, y2=hi, split=ci // 2, **kw)
            else:
                K.igemm(g, wd, dx, mask=x if epi == "mask" else None, **kw)

        def wgrad():
            K.wgrad(g, x, kind=0, grid=(N, hw, hw), M=co, Nc=ci, s=1, pad=1, KW=3, gw=gw, gb=gb, Nreal=ci)

        def split_streams():
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):
                wgrad()
            dgrad()
            torch.cuda.current_stream().wait_stream(side)

        def serial():
            wgrad()
            dgrad()

        tf = timeit(fused, a.iters)
        ts = tq = float("nan") if a.only_fused else 0.0
        if not a.only_fused:
            ts = timeit(split_streams, a.iters)
            tq = timeit(serial, a.iters)
        nbytes = N * hw * hw * 2 * (co + 2 * ci)
        flops = 2 * 2 * N * hw * hw * 9 * ci * co
        print(f"{name:34s} fused {tf:7.3f} ({nbytes / tf / 1e6:6.0f} GB/s, {flops / tf / 1e9:5.0f} TF)  "
              f"split-streams {ts:7.3f}  serial {tq:7.3f}  speedup {ts / tf:4.2f}x", flush=True)
        del g, x, dx, lo, hi
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
