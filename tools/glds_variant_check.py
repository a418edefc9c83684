#!/usr/bin/env python3
"""A new LDS-DMA GEMM variant against the production one on the deep UNet conv shapes: bitwise
comparison of the outputs (both accumulate K in the same order) and interleaved timings.
Usage: python tools/glds_variant_check.py --base 3 --new 14 [--batch 256] [--img 512]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributedpytorch_amd.ops import kernels as K  # noqa: E402
from tools.kbench import timeit  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--base", type=int, default=3)
    ap.add_argument("--new", type=int, nargs="*", default=[14])
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--img", type=int, default=512)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    B, S = a.batch, a.img
    torch.manual_seed(0)
    # (name, H, Cin, Cout): fwd GEMM N = Cout, dgrad GEMM N = Cin
    layers = [("L1 128->64", S // 2, 128, 64), ("L2 64->128", S // 4, 64, 128), ("L2 128->128", S // 4, 128, 128),
              ("L2 256->128", S // 4, 256, 128), ("L3 128->256", S // 8, 128, 256), ("L3 256->256", S // 8, 256, 256),
              ("L3 512->256", S // 8, 512, 256), ("mid 256->512", S // 16, 256, 512), ("mid 512->512", S // 16, 512, 512)]
    bad = 0
    for name, H, Cin, Cout in layers:
        x = torch.randn(B, H, H, Cin, device=dev).to(torch.bfloat16)
        g = torch.randn(B, H, H, Cout, device=dev).to(torch.bfloat16)
        if a.only and not any(o in name for o in a.only.split(",")):
            continue
        for kind in ("fwd", "dgrad"):
            if kind == "fwd":
                src, N, Cs = x, Cout, Cin
            else:
                src, N, Cs = g, Cin, Cout
            # base 0 = the production (auto) path; glds variants need N % 128 (cfg 15) / N % 256 (others)
            if N % 128 or (N % 256 and a.base != 0 and a.base != 15) or Cs % 64:
                continue
            Kp = 9 * Cs
            w = (torch.randn(N, Kp, device=dev) * (1.0 / Kp ** 0.5)).to(torch.bfloat16)
            # the production epilogues: bias + ReLU (forward), ReLU-backward mask (dgrad)
            extra = (dict(bias=torch.randn(N, device=dev) * 0.1, relu=True) if kind == "fwd" else
                     dict(mask=torch.randn(B, H, H, N, device=dev).to(torch.bfloat16)))
            outs = {}
            fns = {}
            for v in [a.base] + a.new:
                if v not in (0, 15) and N % 256:
                    continue
                y = torch.empty(B, H, H, N, device=dev, dtype=torch.bfloat16)
                fn = (lambda y=y, v=v: K.igemm(src, w, y, Ngemm=N, Kpad=Kp, KH=3, KW=3, stride=1, pad=1, Cs=Cs,
                                             out_grid=(B, H, H), path="glds" if v else "auto", variant=v, **extra))
                fn()
                torch.cuda.synchronize()
                outs[v], fns[v] = y, fn
            flops = 2.0 * B * H * H * N * Kp
            ts = {v: [] for v in fns}
            for _ in range(3):
                for v, fn in fns.items():
                    ts[v].append(timeit(fn, a.reps))
            line = f"{name:14s} {kind:5s}"
            for v in fns:
                t = sorted(ts[v])[1]
                same = "" if v == a.base else (" =" if torch.equal(outs[v], outs[a.base]) else " DIFF")
                if same == " DIFF":
                    d = ((outs[v].float() - outs[a.base].float()).abs().max() / outs[a.base].float().abs().max()).item()
                    same += f"({d:.1e})"
                    if d > 1e-2:     # a different K order (the auto path's kernel) rounds differently
                        bad += 1
                line += f"  c{v}: {t:8.1f} us {flops / t / 1e6:6.1f} TF{same}"
            print(line, flush=True)
    print("mismatches:", bad)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
