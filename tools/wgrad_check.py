#!/usr/bin/env python3
"""Deep-layer conv3x3 weight gradients at the bench batch against an fp32 reference (nine shifted fp32
GEMMs over the same bf16 operands): max relative deviation of each kernel path, and run-to-run bitwise
equality.  Usage: python tools/wgrad_check.py [--batch 256] [--img 512] [--paths band,gemm]"""
import argparse
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributedpytorch_amd.ops import kernels as K  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--img", type=int, default=512)
    ap.add_argument("--paths", default="band,band128,gemm,stream")
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    B, S = a.batch, a.img
    torch.manual_seed(0)
    layers = [("L2 64->128", S // 4, 64, 128), ("L2 128->128", S // 4, 128, 128), ("L2 256->128", S // 4, 256, 128),
              ("L3 128->256", S // 8, 128, 256), ("L3 256->256", S // 8, 256, 256), ("L3 512->256", S // 8, 512, 256),
              ("mid 256->512", S // 16, 256, 512), ("mid 512->512", S // 16, 512, 512)]
    for name, H, Cin, Cout in layers:
        if a.only and not any(o in name for o in a.only.split(",")):
            continue
        x = torch.randn(B, H, H, Cin, device="cuda").to(torch.bfloat16)
        g = torch.randn(B, H, H, Cout, device="cuda").to(torch.bfloat16)
        xp = F.pad(x.float(), (0, 0, 1, 1, 1, 1))
        g2 = g.float().reshape(-1, Cout).t().contiguous()
        ref = torch.stack([g2 @ xp[:, kh:kh + H, kw:kw + H].reshape(-1, Cin) for kh in range(3) for kw in range(3)], -1)
        bref = g2.sum(1)
        del xp
        line = f"{name:14s}"
        for p in a.paths.split(","):
            outs = []
            try:
                for _ in range(2):
                    gw = torch.zeros(Cout * Cin * 9, device="cuda")
                    gb = torch.zeros(Cout, device="cuda")
                    K.wgrad(g, x, kind=0, grid=(B, H, H), M=Cout, Nc=Cin, s=1, pad=1, KW=3, gw=gw, gb=gb, Nreal=Cin,
                            path=p)
                    outs.append((gw.view(Cout, Cin, 9), gb))
            except Exception as e:  # noqa: BLE001
                line += f"  {p}: n/a ({str(e)[:30]})"
                continue
            torch.cuda.synchronize()
            gw, gb = outs[0]
            ew = ((gw - ref).abs().max() / ref.abs().max()).item()
            eb = ((gb - bref).abs().max() / bref.abs().max()).item()
            same = torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
            line += f"  {p}: dW {ew:.1e} db {eb:.1e} {'bitwise-repeatable' if same else 'NOT REPEATABLE'}"
        print(line, flush=True)


if __name__ == "__main__":
    main()
