#!/usr/bin/env python3
"""Cost of the BatchNorm partial sums in the row-block GEMM epilogue (csrc/igemm_glds.hip
glds_epilogue_bns): the deep BN-UNet convs (forward: bias, statistics of the output; dgrad: BN-output
mask, backward partials) with and without ``bn_stats``, interleaved; plus the separate statistics pass
(bn_partial via kernels.bn_fwd / bn_bwd without slab) the epilogue replaces.
Usage: python tools/kbench_bn_epi.py [--batch 256] [--img 512]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributedpytorch_amd.ops import kernels as K  # noqa: E402
from tools.kbench import timeit  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--img", type=int, default=512)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--only", default="")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    B, S = a.batch, a.img
    torch.manual_seed(0)
    layers = [("L2 64->128", S // 4, 64, 128), ("L2 128->128", S // 4, 128, 128), ("L3 128->256", S // 8, 128, 256),
              ("L3 256->256", S // 8, 256, 256), ("mid 512->512", S // 16, 512, 512)]
    for name, H, Cin, Cout in layers:
        if a.only and not any(o in name for o in a.only.split(",")):
            continue
        for kind in ("fwd", "dgrad"):
            src_c, N = (Cin, Cout) if kind == "fwd" else (Cout, Cin)
            if N % 128 or src_c % 64:
                continue
            x = torch.randn(B, H, H, src_c, device=dev).to(torch.bfloat16)
            Kp = 9 * src_c
            w = (torch.randn(N, Kp, device=dev) * (1.0 / Kp ** 0.5)).to(torch.bfloat16)
            y = torch.empty(B, H, H, N, device=dev, dtype=torch.bfloat16)
            extra = (dict(bias=torch.randn(N, device=dev) * 0.1) if kind == "fwd" else
                     dict(mask=torch.randn(B, H, H, N, device=dev).clamp_min(0).to(torch.bfloat16)))
            bn = torch.nn.BatchNorm2d(N).to(dev)
            z = torch.randn(B, H, H, N, device=dev).to(torch.bfloat16)
            saved = K.bn_fwd(z, torch.empty_like(z), bn, train=True)
            gamma = torch.zeros(N, device=dev)

            def conv(stats):
                K.igemm(x, w, y, Ngemm=N, Kpad=Kp, KH=3, KW=3, stride=1, pad=1, Cs=src_c, out_grid=(B, H, H),
                        bn_stats=stats, **extra)

            def plain():
                conv(None)

            def fused():
                st = []
                conv(st)
                assert st, "no statistics from the epilogue"

            slab = []
            conv(slab)

            def bn_op(stats):    # the BN op that consumes the sums: with a slab it skips its statistics pass
                if kind == "fwd":
                    K.bn_fwd(y, z, bn, train=True, stats=stats)
                else:
                    K.bn_bwd(y, z, saved, bn, gamma, gamma.clone(), stats=stats)

            ts = {"plain": [], "bn_epi": [], "bn_pass": [], "bn_slab": []}
            for _ in range(3):
                ts["plain"].append(timeit(plain, a.reps))
                ts["bn_epi"].append(timeit(fused, a.reps))
                ts["bn_pass"].append(timeit(lambda: bn_op(None), a.reps))
                ts["bn_slab"].append(timeit(lambda: bn_op(slab), a.reps))
            med = {k: sorted(v)[1] for k, v in ts.items()}
            print(f"{name:13s} {kind:5s} conv {med['plain']:8.1f} us  +BN epilogue {med['bn_epi'] - med['plain']:+7.1f}  "
                  f"BN op with stats pass {med['bn_pass']:8.1f} us, with epilogue slab {med['bn_slab']:8.1f} us "
                  f"(saves {med['bn_pass'] - med['bn_slab']:6.1f})  net {med['bn_pass'] - med['bn_slab'] - (med['bn_epi'] - med['plain']):+7.1f}",
                  flush=True)


if __name__ == "__main__":
    main()
