#!/usr/bin/env python3
"""Ceiling of the LDS-DMA GEMM skeleton (csrc/igemm_glds.hip) on a plain square GEMM: the kernel run as
a 1x1 convolution (M = pixels, N = output channels, K = input channels) next to hipBLASLt (torch.matmul)
on the same bf16 operands, uniform random data.  Usage: python tools/gemm_skeleton.py [--n 8192]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributedpytorch_amd.ops import kernels as K  # noqa: E402


def timeit(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for _ in range(reps):
        s.record()
        fn()
        e.record()
        torch.cuda.synchronize()
        ts.append(s.elapsed_time(e) * 1e3)
    ts.sort()
    return ts[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, nargs="*", default=[4096, 8192])
    ap.add_argument("--cfgs", type=int, nargs="*", default=[3, 8, 11])
    a = ap.parse_args()
    for n in a.n:
        W = 128
        H = n // W
        x = (torch.rand(1, H, W, n, device="cuda") * 2 - 1).to(torch.bfloat16)
        w = (torch.rand(n, n, device="cuda") * 2 - 1).to(torch.bfloat16)
        y = torch.empty(1, H, W, n, device="cuda", dtype=torch.bfloat16)
        flops = 2.0 * n * n * n
        x2, wt = x.view(n, n), w.t()
        t = timeit(lambda: torch.matmul(x2, wt))
        print(f"N={n:5d} hipBLASLt (torch.matmul)  {t:9.1f} us {flops / t / 1e6:7.1f} TF", flush=True)
        ref = torch.matmul(x2, wt).float()
        for c in a.cfgs:
            fn = lambda: K.igemm(x, w, y, Ngemm=n, Kpad=n, KH=1, KW=1, stride=1, pad=0, Cs=n, out_grid=(1, H, W),
                                 path="glds", variant=c)
            try:
                t = timeit(fn)
                err = float((y.view(n, n).float() - ref).abs().max() / ref.abs().max())
                print(f"N={n:5d} igemm_glds cfg {c:<3d}        {t:9.1f} us {flops / t / 1e6:7.1f} TF  (max rel err {err:.1e})",
                      flush=True)
            except Exception as e:  # noqa: BLE001
                print(f"N={n:5d} igemm_glds cfg {c:<3d} n/a ({str(e)[:60]})", flush=True)


if __name__ == "__main__":
    main()
