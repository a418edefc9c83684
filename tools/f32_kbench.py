#!/usr/bin/env python3
"""Per-layer timing of the fp32 engine's GEMM kernels (csrc/fp32.hip) on the UNet at one batch: conv3x3
forward, dgrad and weight gradient, transposed-conv forward / dgrad / weight gradient; achieved TFLOP/s
against the 157 TFLOP/s fp32-MFMA peak.

    python tools/f32_kbench.py --batch 16 --img 512 [--wgrad-big both]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _modes(opt, current):
    return {"default": [current], "off": [False], "on": [True], "both": [False, True]}[opt]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--img", default="512", help="H or HxW (e.g. 640x960, the reference default)")
    ap.add_argument("--model", default="unet")
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--wgrad-big", choices=["default", "off", "on", "both"], default="default",
                    help="time the conv weight gradients with the 256 x 256 tile too (deep layers)")
    ap.add_argument("--igemm-wide", choices=["default", "off", "on", "both"], default="default",
                    help="time the conv forward / dgrad with the 256-pixel 8-wave tile too")
    ap.add_argument("--wgrad-px", choices=["default", "off", "on", "both"], default="default",
                    help="time the generic weight gradients with the pixel-major LDS form too")
    ap.add_argument("--conv-halo", default="default",
                    help="comma list of DPA_F32_CONV_HALO modes to time the conv forward / dgrad with (last printed first)")
    ap.add_argument("--wgrad-c4", choices=["default", "off", "on", "both"], default="default",
                    help="time the first conv's weight gradient with the 4-channel form too")
    ap.add_argument("--wgrad3-halves", choices=["default", "off", "on", "both"], default="default",
                    help="time the 64-input-channel halo weight gradients as two 32-column halves too")
    a = ap.parse_args()
    from distributedpytorch_amd.models import hip_unet_f32 as E
    from distributedpytorch_amd.models.unet import build_model
    from distributedpytorch_amd.ops import fp32 as F32
    dev = torch.device("cuda:0")
    cfg = build_model(a.model).cfg
    N = a.batch
    H0, W0 = (int(v) for v in a.img.split("x")) if "x" in a.img else (int(a.img), int(a.img))
    convs, deconvs = [], []
    w = list(cfg.widths)
    cin, h, wd = 3, H0, W0
    for l, c in enumerate(w):
        convs.append((f"enc{l}.c1", (h, wd), cin, c)), convs.append((f"enc{l}.c2", (h, wd), c, c))
        cin, h, wd = c, h // 2, wd // 2
    convs.append(("mid.c1", (h, wd), cin, cfg.mid_width)), convs.append(("mid.c2", (h, wd), cfg.mid_width, cfg.mid_width))
    cin = cfg.mid_width
    for i, c in enumerate(reversed(w)):
        deconvs.append((f"dec{i}.up", (h, wd), cin, c))
        h, wd = h * 2, wd * 2
        convs.append((f"dec{i}.c1", (h, wd), 2 * c, c)), convs.append((f"dec{i}.c2", (h, wd), c, c))
        cin = c

    def t(fn):
        fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(a.reps):
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            fn()
            e.record()
            torch.cuda.synchronize()
            ts.append(s.elapsed_time(e))
        return sorted(ts)[len(ts) // 2]

    tot = {"fwd": 0.0, "dgrad": 0.0, "wgrad": 0.0}
    print(f"{'layer':10s} {'HxW':>9s} {'ci':>4s} {'co':>4s} | {'fwd ms':>7s} {'TF/s':>6s} | {'dgrad':>7s} {'TF/s':>6s} | "
          f"{'wgrad':>7s} {'TF/s':>6s}")
    for name, (hh, ww), ci, co in convs:
        cs = 4 if ci == 3 else ci
        x = torch.randn(N, hh, ww, cs, device=dev)
        m = torch.nn.Conv2d(ci, co, 3, padding=1).to(dev)
        layer = E._L(m, "conv", cs)
        eng = E.F32Engine([layer], dev)
        eng.side = None                      # time the kernels themselves, on the current stream
        eng.ensure_packed()
        ge = torch.randn(N, hh, ww, co, device=dev)
        fl = 2.0 * N * hh * ww * co * ci * 9
        wmodes = _modes(a.igemm_wide, F32.IGEMM_WIDE)
        hmodes = [F32.CONV_HALO] if a.conv_halo == "default" else [int(v) for v in a.conv_halo.split(",")]
        if len(hmodes) > 1:
            wmodes = [F32.IGEMM_WIDE] * len(hmodes)
        tfs, tds = [], []
        for k, wide in enumerate(wmodes):
            F32.IGEMM_WIDE = wide
            F32.CONV_HALO = hmodes[min(k, len(hmodes) - 1)]
            tfs.append(t(lambda: E._conv_fwd(eng, layer, x)))
            tds.append(t(lambda: E._conv_dgrad(eng, layer, ge)) if ci != 3 else 0.0)
        tf, td = tfs[-1], tds[-1]
        modes = _modes(a.wgrad_big, F32.USE_WGRAD_BIG)
        pxm = _modes(a.wgrad_px, F32.WGRAD_PX)
        hvm = _modes(a.wgrad3_halves, F32.WGRAD3_HALVES)
        c4m = _modes(a.wgrad_c4, F32.WGRAD_C4)
        if len(pxm) > 1 or len(hvm) > 1 or len(c4m) > 1:
            modes = [F32.USE_WGRAD_BIG] * 2
        tws = []
        for k, big in enumerate(modes):
            F32.USE_WGRAD_BIG = big
            F32.WGRAD_PX = pxm[min(k, len(pxm) - 1)]
            F32.WGRAD3_HALVES = hvm[min(k, len(hvm) - 1)]
            F32.WGRAD_C4 = c4m[min(k, len(c4m) - 1)]
            tws.append(t(lambda: E._conv_wgrad(eng, layer, ge, x)))
        tw = tws[-1]
        tot["fwd"] += tf
        tot["dgrad"] += td
        tot["wgrad"] += tw
        extra = "" if len(tws) == 1 else f" (other form: {tws[0]:7.3f} {fl / tws[0] / 1e9:6.1f})"
        if len(tfs) > 1:
            extra += f" [other fwd {tfs[0]:7.3f} dgrad {tds[0]:7.3f}]"
        print(f"{name:10s} {hh:4d}x{ww:<4d} {ci:4d} {co:4d} | {tf:7.3f} {fl / tf / 1e9:6.1f} | {td:7.3f} "
              f"{(fl / td / 1e9 if td else 0):6.1f} | {tw:7.3f} {fl / tw / 1e9:6.1f}{extra}", flush=True)
        del x, ge
    for name, (hh, ww), ci, co in deconvs:
        x = torch.randn(N, hh, ww, ci, device=dev)
        wt = torch.randn(ci, co, 2, 2, device=dev) * 0.05
        b = torch.zeros(co, device=dev)
        gy = torch.randn(N, 2 * hh, 2 * ww, co, device=dev)
        fl = 2.0 * N * hh * ww * ci * co * 4
        y = torch.empty(N, 2 * hh, 2 * ww, co, device=dev)
        wf = F32.pack_deconv_fwd(wt)
        tf = t(lambda: F32.igemm(x, wf, y, Ngemm=4 * co, Kpad=ci, KH=1, KW=1, stride=1, pad=0, Cs=ci,
                                 out_grid=(N, hh, ww), bias=b, mode=1, Cout=co))
        gx = torch.empty(N, hh, ww, ci, device=dev)
        wd = F32.pack_deconv_dgrad(wt)
        td = t(lambda: F32.igemm(gy, wd, gx, Ngemm=ci, Kpad=4 * co, KH=2, KW=2, stride=2, pad=0, Cs=co,
                                 out_grid=(N, hh, ww)))
        gw = torch.zeros(ci, co, 2, 2, device=dev)
        tw = t(lambda: F32.wgrad(x, gy, gw, None, KH=2, KW=2, s=2, pad=0))
        tot["fwd"] += tf
        tot["dgrad"] += td
        tot["wgrad"] += tw
        print(f"{name:10s} {hh:4d}x{ww:<4d} {ci:4d} {co:4d} | {tf:7.3f} {fl / tf / 1e9:6.1f} | {td:7.3f} "
              f"{fl / td / 1e9:6.1f} | {tw:7.3f} {fl / tw / 1e9:6.1f}", flush=True)
    print("totals ms: " + ", ".join(f"{k} {v:.2f}" for k, v in tot.items()))


if __name__ == "__main__":
    main()
