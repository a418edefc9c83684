#!/usr/bin/env python3
"""Per-layer kernel micro-benchmark on one MI355X: times every conv path (stream / halo / generic,
fwd + dgrad) and the weight-gradient kernels for the UNet layer shapes at a given batch/resolution,
all variants interleaved in one process (guide §5.4 rule 24).  Prints one line per (layer, path):
microseconds and TFLOP/s.  Usage: python tools/kbench.py [--batch 32] [--img 512] [--reps 10]"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributedpytorch_amd.ops import kernels as K  # noqa: E402


def timeit(fn, reps):
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
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--img", type=int, default=512)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--only", default="")
    ap.add_argument("--cfgs", type=int, nargs="*", default=[], help="extra generic tile configs to time")
    ap.add_argument("--no-wgrad", action="store_true")
    ap.add_argument("--svar", type=int, nargs="*", default=[], help="streaming-conv variants to time")
    ap.add_argument("--gvar", type=int, nargs="*", default=[], help="LDS-DMA (glds) kernel configs to time")
    ap.add_argument("--hvar", type=int, nargs="*", default=[], help="row-halo kernel configs to time")
    ap.add_argument("--wsvar", type=int, nargs="*", default=[], help="row-streaming wgrad tile configs to time")
    ap.add_argument("--wpaths", default="stream,halo,generic", help="weight-gradient paths to time (also: rows)")
    ap.add_argument("--dwcfg", type=int, nargs="*", default=[], help="transposed-conv wgrad tile configs to time")
    ap.add_argument("--paths", default="stream,halo,generic", help="default paths to time")
    ap.add_argument("--layout-probe", action="store_true",
                    help="full-res memory-bound ops on concat halves (ld=2C) vs dense tensors (ld=C)")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    B, S = a.batch, a.img
    # (name, H, Cin, Cout)
    layers = [("L0 32->32", S, 32, 32), ("L0 64->32", S, 64, 32), ("L1 32->64", S // 2, 32, 64),
              ("L1 64->64", S // 2, 64, 64), ("L1 128->64", S // 2, 128, 64), ("L2 64->128", S // 4, 64, 128),
              ("L2 128->128", S // 4, 128, 128), ("L2 256->128", S // 4, 256, 128), ("L3 128->256", S // 8, 128, 256), ("L3 256->256", S // 8, 256, 256), ("L3 512->256", S // 8, 512, 256),
              ("mid 512->512", S // 16, 512, 512)]
    for name, H, Cin, Cout in layers:
        if a.only and not any(o in name for o in a.only.split(",")):
            continue
        x = torch.randn(B, H, H, Cin, device=dev).to(torch.bfloat16)
        g = torch.randn(B, H, H, Cout, device=dev).to(torch.bfloat16)
        y = torch.empty(B, H, H, Cout, device=dev, dtype=torch.bfloat16)
        dx = torch.empty(B, H, H, Cin, device=dev, dtype=torch.bfloat16)
        kf, kd = K.round_up(9 * Cin, 32), K.round_up(9 * Cout, 32)
        wf = (torch.randn(Cout * kf, device=dev) * 0.05).to(torch.bfloat16)
        wd = (torch.randn(Cin * kd, device=dev) * 0.05).to(torch.bfloat16)
        bias = torch.zeros(Cout, device=dev)
        flops = 2.0 * B * H * H * Cin * Cout * 9
        variants = [(p, p, 0, 0) for p in a.paths.split(",") if p] + \
            [(f"gen.c{c}", "generic", c, 0) for c in a.cfgs] + [(f"strm.v{v}", "stream", 0, v) for v in a.svar] + \
            [(f"glds.c{v}", "glds", 0, v) for v in a.gvar] + [(f"halo.c{v}", "halo", 0, v) for v in a.hvar]
        for label, path, cfg, var in variants:
            try:
                t = timeit(lambda: K.igemm(x, wf, y, Ngemm=Cout, Kpad=kf, KH=3, KW=3, stride=1, pad=1, Cs=Cin,
                                           out_grid=(B, H, H), bias=bias, relu=True, path=path, cfg=cfg, variant=var), a.reps)
                print(f"{name:14s} fwd   {label:8s} {t:9.1f} us {flops / t / 1e6:7.1f} TF", flush=True)
            except Exception as e:  # path not eligible for this shape
                print(f"{name:14s} fwd   {label:8s}  n/a ({str(e)[:40]})", flush=True)
            try:
                t = timeit(lambda: K.igemm(g, wd, dx, Ngemm=Cin, Kpad=kd, KH=3, KW=3, stride=1, pad=1, Cs=Cout,
                                           out_grid=(B, H, H), mask=x, path=path, cfg=cfg, variant=var), a.reps)
                print(f"{name:14s} dgrad {label:8s} {t:9.1f} us {flops / t / 1e6:7.1f} TF", flush=True)
            except Exception as e:
                print(f"{name:14s} dgrad {label:8s}  n/a ({str(e)[:40]})", flush=True)
        gw = torch.zeros(Cout * Cin * 9, device=dev)
        gb = torch.zeros(Cout, device=dev)
        wvars = [(p, p, 0) for p in (() if a.no_wgrad else a.wpaths.split(","))] + \
            [(f"strm.w{v}", "stream", v) for v in a.wsvar]
        for label, path, wv in wvars:
            K.WGRAD_STREAM_CFG = wv if path == "stream" else 0
            try:
                t = timeit(lambda: K.wgrad(g, x, kind=0, grid=(B, H, H), M=Cout, Nc=Cin, s=1, pad=1, KW=3, gw=gw,
                                           gb=gb, Nreal=Cin, path=path), a.reps)
                print(f"{name:14s} wgrad {label:8s} {t:9.1f} us {flops / t / 1e6:7.1f} TF", flush=True)
            except Exception as e:
                print(f"{name:14s} wgrad {label:8s}  n/a ({str(e)[:40]})", flush=True)
        K.WGRAD_STREAM_CFG = 0
        del x, g, y, dx
    if a.layout_probe:
        C, H = 32, S
        for ld in (2 * C, C):
            big = torch.randn(B, H, H, ld, device=dev).to(torch.bfloat16)
            big2 = torch.randn(B, H, H, ld, device=dev).to(torch.bfloat16)
            skip, dskip = big[..., :C], big2[..., :C]
            dpool = torch.randn(B, H // 2, H // 2, C, device=dev).to(torch.bfloat16)
            g = torch.empty(B, H, H, C, device=dev, dtype=torch.bfloat16)
            t = timeit(lambda: K.pool_bwd(skip, dskip, dpool, g), a.reps)
            gb = (3 * B * H * H * C * 2 + B * H * H * C // 2) / 1e9
            print(f"pool_bwd ld={ld:3d}      {t:9.1f} us {gb / t * 1e3:7.2f} TB/s(useful)", flush=True)
            x = torch.randn(B, H // 2, H // 2, 2 * C, device=dev).to(torch.bfloat16)
            wf = (torch.randn(4 * C * 2 * C, device=dev) * 0.05).to(torch.bfloat16)
            for path, var in (("generic", 0), ("glds", 2)):
                t = timeit(lambda: K.igemm(x, wf, big[..., ld - C:], Ngemm=4 * C, Kpad=2 * C, KH=1, KW=1, stride=1,
                                           pad=0, Cs=2 * C, out_grid=(B, H // 2, H // 2), mode=1, Cout=C, path=path,
                                           variant=var), a.reps)
                gb = (B * H * H * C * 2 + B * H * H * C // 2) / 1e9
                print(f"deconv4 fwd ld={ld:3d} {path:7s} {t:9.1f} us {gb / t * 1e3:7.2f} TB/s(useful)", flush=True)
            del big, big2
    # transposed convs (k2 s2): fwd = 1x1 GEMM scattered into the concat buffer, dgrad = stride-2 gather
    for name, h, Cin, Cout in [("D1 512->256", S // 16, 512, 256), ("D2 256->128", S // 8, 256, 128),
                               ("D3 128->64", S // 4, 128, 64), ("D4 64->32", S // 2, 64, 32)]:
        if a.only and not any(o in name for o in a.only.split(",")):
            continue
        x = torch.randn(B, h, h, Cin, device=dev).to(torch.bfloat16)
        cat = torch.empty(B, 2 * h, 2 * h, 2 * Cout, device=dev, dtype=torch.bfloat16)
        wf = (torch.randn(4 * Cout * Cin, device=dev) * 0.05).to(torch.bfloat16)
        wd = (torch.randn(Cin * 4 * Cout, device=dev) * 0.05).to(torch.bfloat16)
        dx = torch.empty(B, h, h, Cin, device=dev, dtype=torch.bfloat16)
        flops = 2.0 * B * h * h * Cin * Cout * 4
        for label, path, var in [("generic", "generic", 0)] + [(f"glds.c{v}", "glds", v) for v in a.gvar]:
            for kind in ("fwd", "dgrad"):
                try:
                    if kind == "fwd":
                        fn = lambda: K.igemm(x, wf, cat[..., Cout:], Ngemm=4 * Cout, Kpad=Cin, KH=1, KW=1, stride=1,
                                             pad=0, Cs=Cin, out_grid=(B, h, h), mode=1, Cout=Cout, path=path,
                                             variant=var)
                    else:
                        fn = lambda: K.igemm(cat[..., Cout:], wd, dx, Ngemm=Cin, Kpad=4 * Cout, KH=2, KW=2, stride=2,
                                             pad=0, Cs=Cout, out_grid=(B, h, h), mask=x, path=path, variant=var)
                    t = timeit(fn, a.reps)
                    print(f"{name:14s} {kind:5s} {label:8s} {t:9.1f} us {flops / t / 1e6:7.1f} TF", flush=True)
                except Exception as e:
                    print(f"{name:14s} {kind:5s} {label:8s}  n/a ({str(e)[:40]})", flush=True)
        gw = torch.zeros(Cin * Cout * 4, device=dev)
        gb = torch.zeros(Cout, device=dev)
        for c in [0] + a.dwcfg:
            try:
                t = timeit(lambda: K.wgrad(cat[..., Cout:], x, kind=1, grid=(B, h, h), M=Cout, Nc=Cin, s=2, pad=0, KW=2,
                                           gw=gw, gb=gb, Nreal=Cin, cfg=c), a.reps)
                print(f"{name:14s} wgrad cfg{c:<5d} {t:9.1f} us {flops / t / 1e6:7.1f} TF", flush=True)
            except Exception as e:
                print(f"{name:14s} wgrad cfg{c:<5d}  n/a ({str(e)[:40]})", flush=True)


if __name__ == "__main__":
    main()
