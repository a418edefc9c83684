#!/usr/bin/env python3
"""Transposed-conv (k2 s2) weight gradient: the library kernel (kernels.wgrad kind 1) against a library-GEMM
form -- per kernel row i, G_i[(n,h,w)][(j,co)] = g[n][2h+i][2w+j][co] gathered dense (one copy of half the
gradient), then dW_i = G_i^T X on hipBLASLt with fp32 output (torch.mm out_dtype) -- timing and max deviation.
Usage: python tools/deconv_wgrad_probe.py [--batch 256] [--img 512]"""
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
    return sorted(ts)[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--img", type=int, default=512)
    a = ap.parse_args()
    B, S = a.batch, a.img
    for name, h, Cin, Cout in [("D1 512->256", S // 16, 512, 256), ("D2 256->128", S // 8, 256, 128),
                               ("D3 128->64", S // 4, 128, 64)]:
        x = torch.randn(B, h, h, Cin, device="cuda").to(torch.bfloat16)
        g = torch.randn(B, 2 * h, 2 * h, Cout, device="cuda").to(torch.bfloat16)
        gw = torch.zeros(Cin * Cout * 4, device="cuda")
        gb = torch.zeros(Cout, device="cuda")
        t_lib = timeit(lambda: K.wgrad(g, x, kind=1, grid=(B, h, h), M=Cout, Nc=Cin, s=2, pad=0, KW=2, gw=gw, gb=gb,
                                       Nreal=Cin))
        X = x.reshape(-1, Cin)

        def blas():
            gv = g.view(B, h, 2, h, 2 * Cout)
            outs = []
            for i in range(2):
                Gi = gv[:, :, i].reshape(-1, 2 * Cout)                # copy: [P, (j, co)]
                outs.append(torch.mm(Gi.t(), X, out_dtype=torch.float32))   # [(j, co), ci]
            return outs
        t_blas = timeit(blas)
        # reference: out[tap][co][ci] with tap = 2 i + j, same fp32 GEMM of the same bf16 operands
        gw.zero_()
        K.wgrad(g, x, kind=1, grid=(B, h, h), M=Cout, Nc=Cin, s=2, pad=0, KW=2, gw=gw, gb=gb, Nreal=Cin)
        o = blas()
        alt = torch.stack([o[i].view(2, Cout, Cin)[j] for i in range(2) for j in range(2)])   # [tap][co][ci]
        lib = gw.view(Cin, Cout, 2, 2).permute(2, 3, 1, 0).reshape(4, Cout, Cin)              # ConvT [ci][co][i][j]
        dev = ((alt - lib).abs().max() / lib.abs().max()).item()
        flops = 2.0 * B * h * h * Cin * Cout * 4
        print(f"{name}: kernel {t_lib:8.1f} us ({flops / t_lib / 1e6:6.1f} TF)  copy+hipBLASLt {t_blas:8.1f} us "
              f"({flops / t_blas / 1e6:6.1f} TF)  max rel dev {dev:.1e}", flush=True)


if __name__ == "__main__":
    main()
