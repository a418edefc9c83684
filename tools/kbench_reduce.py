#!/usr/bin/env python3
"""Slab-reduction kernel sweep (csrc/wgrad.hip dpa_wgrad_reduce_cfg) on the slab shapes a real step
produces: one training step of the UNet (batch --batch, 512^2) and optionally the UNet-XL 8-stage
pipeline (--xl) is run with the reduce launches logged, then every distinct (splits, T, M, Nc, bias)
is timed with the 32-element kernel (g0) and the quad kernel at 1..64 split groups (g1..g64), plus
the auto choice.  Usage: python tools/kbench_reduce.py [--batch 256] [--xl]"""
import argparse
import collections
import ctypes
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from distributedpytorch_amd.ops import _lib, kernels as K  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=256)
    ap.add_argument("--xl", action="store_true")
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    L = _lib.lib()
    seen = collections.Counter()
    real = L.dpa_wgrad_reduce

    def logged(slab, bslab, gw, gb, splits, T, M, Nc, Nreal, mode, st):
        seen[(splits.value, T.value, M.value, Nc.value, Nreal.value, mode.value, bslab is not None)] += 1
        return real(slab, bslab, gw, gb, splits, T, M, Nc, Nreal, mode, st)

    L.dpa_wgrad_reduce = logged
    import bench
    argv = ["bench.py", "--steps", "1", "--warmup", "0", "--batch", str(a.batch)]
    if a.xl:
        argv = ["bench.py", "--steps", "1", "--warmup", "0", "--model", "unet-xl", "--img", "1024", "--batch", "16",
                "--parallelism", "mp", "--stages", "8", "--microbatches", "4"]
    sys.argv = argv
    bench.main()
    L.dpa_wgrad_reduce = real
    torch.cuda.synchronize()
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    tot_best = tot_auto = tot_old = 0.0
    for (splits, T, M, Nc, Nreal, mode, hb), n in sorted(seen.items(), key=lambda kv: -kv[0][0] * kv[0][2] * kv[0][3]):
        slab = torch.randn(splits * T * M * Nc + splits * M, device="cuda")
        bslab = slab[splits * T * M * Nc:] if hb else None
        gw = torch.zeros(M * Nreal * T, device="cuda")
        gb = torch.zeros(M, device="cuda")
        res = {}
        for g in (0, -1, -2, 1, 2, 4, 8, 16, 32, 64):
            def run():
                return L.dpa_wgrad_reduce_cfg(K._p(slab), K._p(bslab), K._p(gw), K._p(gb), splits, T, M, Nc, Nreal,
                                              mode, g, st)
            if run() != 0:
                continue
            ts = []
            for _ in range(a.reps):
                s.record()
                run()
                e.record()
                torch.cuda.synchronize()
                ts.append(s.elapsed_time(e) * 1e3)
            res[g] = sorted(ts)[len(ts) // 2]
        best = min((v, g) for g, v in res.items() if g != -1)   # g-2: tiled
        mb = splits * T * M * Nc * 4 / 2 ** 20
        print(f"splits {splits:5d} T {T} M {M:4d} Nc {Nc:4d} bias {int(hb)} x{n:3d}  {mb:8.1f} MiB  old {res[0]:7.1f} us  "
              f"auto {res[-1]:7.1f} us  best g{best[1]} {best[0]:7.1f} us  "
              + " ".join(f"g{g}:{v:.0f}" for g, v in res.items() if g > 0 or g == -2), flush=True)
        tot_old += n * res[0]
        tot_auto += n * res[-1]
        tot_best += n * best[0]
    print(f"per-step totals: old {tot_old / 1e3:.2f} ms, auto {tot_auto / 1e3:.2f} ms, best {tot_best / 1e3:.2f} ms")


if __name__ == "__main__":
    main()
