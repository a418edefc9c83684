#!/usr/bin/env python3
"""Deep-layer conv3x3 weight gradients at the bench batch: the row-streaming (csrc/halo.hip), dense-GEMM
(csrc/wgrad_gemm.hip) and band-staged (csrc/wgrad_band.hip: 256- and 128-output-channel forms) paths
interleaved in one process, plus the max deviation of each from the gemm path's result (accuracy against
fp32: tools/wgrad_check.py).  Usage: python tools/kbench_wgrad_deep.py [--batch 256] [--img 512]"""
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
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--paths", default="stream,gemm,band,band128")
    ap.add_argument("--only", default="", help="comma-separated layer-name substrings")
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
        flops = 2.0 * B * H * H * Cout * Cin * 9
        res, line = {}, f"{name:14s}"
        for p in a.paths.split(","):
            gw = torch.zeros(Cout * Cin * 9, device="cuda")
            gb = torch.zeros(Cout, device="cuda")
            fn = lambda p=p, gw=gw, gb=gb: K.wgrad(g, x, kind=0, grid=(B, H, H), M=Cout, Nc=Cin, s=1, pad=1, KW=3,  # noqa: E731
                                                  gw=gw, gb=gb, Nreal=Cin, path=p)
            try:
                fn()
                torch.cuda.synchronize()
                ref = gw.clone()
                t = timeit(fn, a.reps)
                res[p] = ref
                line += f"  {p}: {t:8.1f} us {flops / t / 1e6:6.1f} TF"
            except Exception as e:  # noqa: BLE001
                line += f"  {p}: n/a ({str(e)[:40]})"
        if "gemm" in res:
            for p, r in res.items():
                if p != "gemm":
                    d = ((r - res["gemm"]).abs().max() / res["gemm"].abs().max()).item()
                    line += f"  |{p}-gemm|={d:.1e}"
        print(line, flush=True)


if __name__ == "__main__":
    main()
