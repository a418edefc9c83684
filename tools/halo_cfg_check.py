#!/usr/bin/env python3
"""64-output-channel conv3x3 paths against each other on the UNet shapes the row-halo kernel took before round 6
(256^2 128->64 forward, 128^2 128->64 dgrad with the ReLU mask): the row-halo tile configs and the auto path
(the slice-staged ping-pong 64 x 512 kernel, igemm_slp_kernel<EP, 64>), each against row-halo cfg 4 (bitwise:
same per-output accumulation order) and an fp32 reference.
Usage: python tools/halo_cfg_check.py [--batch 8] [--cfgs 11 13]"""
import argparse
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributedpytorch_amd.ops import kernels as K  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--cfgs", type=int, nargs="*", default=[11, 12, 13, 14])
    a = ap.parse_args()
    torch.manual_seed(0)
    for H, Cin, Cout, masked in ((256, 128, 64, False), (128, 128, 64, True), (64, 256, 64, False), (32, 64, 64, True)):
        x = torch.randn(a.batch, H, H, Cin, device="cuda").to(torch.bfloat16)
        kf = K.round_up(9 * Cin, 32)
        w = (torch.randn(Cout, 3, 3, Cin, device="cuda") * 0.05).to(torch.bfloat16)
        wf = torch.zeros(Cout, kf, device="cuda", dtype=torch.bfloat16)
        wf[:, :9 * Cin] = w.reshape(Cout, -1)
        bias = None if masked else torch.randn(Cout, device="cuda") * 0.1
        mask = torch.randn(a.batch, H, H, Cout, device="cuda").to(torch.bfloat16) if masked else None
        ref = F.conv2d(x.permute(0, 3, 1, 2).float(), w.permute(0, 3, 1, 2).float(), bias, padding=1).permute(0, 2, 3, 1)
        ref = ref * (mask.float() > 0) if masked else ref.relu()
        outs = {}
        for label, path, var in [("halo.c4", "halo", 4), ("auto", "auto", 0)] + [(f"halo.c{c}", "halo", c) for c in a.cfgs]:
            y = torch.empty(a.batch, H, H, Cout, device="cuda", dtype=torch.bfloat16)
            try:
                K.igemm(x, wf.reshape(-1), y, Ngemm=Cout, Kpad=kf, KH=3, KW=3, stride=1, pad=1, Cs=Cin,
                        out_grid=(a.batch, H, H), bias=bias, relu=not masked, mask=mask, path=path, variant=var)
            except Exception as e:  # noqa: BLE001
                print(f"{H}^2 {Cin}->{Cout} {label}: n/a ({str(e)[:40]})", flush=True)
                continue
            torch.cuda.synchronize()
            outs[label] = y
            err = ((y.float() - ref).abs().max() / ref.abs().max()).item()
            same = "" if label == "halo.c4" or "halo.c4" not in outs else \
                (" bitwise = halo.c4" if torch.equal(y, outs["halo.c4"]) else " differs from halo.c4")
            print(f"{H}^2 {Cin}->{Cout} {'dgrad' if masked else 'fwd'} {label}: rel err {err:.2e}{same}", flush=True)


if __name__ == "__main__":
    main()
