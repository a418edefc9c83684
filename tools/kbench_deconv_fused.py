#!/usr/bin/env python3
"""Times the full-resolution fused transposed-conv forward (csrc/deconv.hip deconv_fwd) at the UNet's
D3 / D4 shapes into a concat-buffer half.  Usage: python tools/kbench_deconv_fused.py [--batch 256]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from distributedpytorch_amd.ops import kernels as K  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    for name, h, cin, cout in (("D3 128->64 @128->256", 128, 128, 64), ("D4 64->32 @256->512", 256, 64, 32)):
        x = torch.randn(a.batch, h, h, cin, device="cuda").to(torch.bfloat16)
        cat = torch.empty(a.batch, 2 * h, 2 * h, 2 * cout, device="cuda", dtype=torch.bfloat16)
        wf = (torch.randn(4 * cout * cin, device="cuda") * 0.05).to(torch.bfloat16)
        b = torch.zeros(cout, device="cuda")
        dense = torch.empty(a.batch, 2 * h, 2 * h, cout, device="cuda", dtype=torch.bfloat16)
        for label, out in (("concat half", cat[..., cout:]), ("dense", dense)):
            fn = lambda: K.deconv_fwd_fused(x, wf, b, out)
            fn()
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            ts = []
            for _ in range(a.reps):
                s.record()
                fn()
                e.record()
                torch.cuda.synchronize()
                ts.append(s.elapsed_time(e) * 1e3)
            t = sorted(ts)[len(ts) // 2]
            gb = (x.numel() + a.batch * 4 * h * h * cout) * 2 / 1e9
            print(f"{name:24s} {label:12s} {t:9.1f} us  {gb / t * 1e3:6.2f} TB/s", flush=True)
        del x, cat, dense


if __name__ == "__main__":
    main()
